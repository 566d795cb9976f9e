/* Pre-include this header (gcc -include prelude.h) to build the reference's UNMODIFIED
 * plonk.h / plonk-test.c against libplonkhip: it defines the include guards FE_H, HF_H,
 * G1_H, G2_H, POLY_H, SRS_H and MATRIX_H first, so the reference's own #include "poly.h" /
 * "srs.h" / "matrix.h" (src/plonk.h:6-10) become no-ops and poly_mul / srs_eval_at_s (the hot
 * path) and poly_divide / poly_eval / matrix_mul / matrix_inv resolve to the GPU (calls of toy
 * size: to the host code of plk_host.h).
 * (A plain -I is not enough: a quoted include searches the includer's directory first.)
 * Link with -lplonkhip. */
#ifndef PLONKHIP_PRELUDE_H
#define PLONKHIP_PRELUDE_H
#include "hf.h"
#include "gf.h"
#include "g1.h"
#include "g2.h"
#include "poly.h"
#include "srs.h"
#include "matrix.h"

/* Build-time policy for a drop-in build (no source change in the reference): with
 * -DPLK_DROPIN_SHARD_MIN=m, srs_eval_at_s splits every MSM of >= m points over the devices of
 * plk_init_devices / PLK_DEVICE="0,1,..." (the tests build the reference's programs with m = 1
 * to run every commitment through the shards). */
#ifdef PLK_DROPIN_SHARD_MIN
__attribute__((constructor)) static void plk_dropin_shard_policy(void) {
  (void)plk_set_option(PLK_OPT_MSM_SHARD_MIN, PLK_DROPIN_SHARD_MIN);
}
#endif
/* -DPLK_DROPIN_HOST_WORK=w: the small-size policy's threshold for this program (include/plk_host.h;
 * 0 sends every call to the GPU, as the tests' forced-GPU builds of the reference programs do) */
#ifdef PLK_DROPIN_HOST_WORK
__attribute__((constructor)) static void plk_dropin_host_policy(void) {
  (void)plk_set_option(PLK_OPT_DROPIN_HOST_WORK, PLK_DROPIN_HOST_WORK);
}
#endif
#endif
