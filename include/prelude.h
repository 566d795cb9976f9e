/* Pre-include this header (gcc -include prelude.h) to build the reference's UNMODIFIED
 * plonk.h / plonk-test.c against libplonkhip: it defines the include guards FE_H, HF_H,
 * G1_H, G2_H, POLY_H, SRS_H and MATRIX_H first, so the reference's own #include "poly.h" /
 * "srs.h" / "matrix.h" (src/plonk.h:6-10) become no-ops and poly_mul / srs_eval_at_s (the hot
 * path) and poly_divide / poly_eval / matrix_mul / matrix_inv resolve to the GPU.
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
#endif
