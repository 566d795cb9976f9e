/* The drop-in headers' small-size policy: a call whose host work is about one GPU
 * round trip or less is computed here, on the calling thread; every larger call goes to the GPU
 * through the C ABI (include/plonkhip.h).
 *
 * Why: a host-buffer call into libplonkhip costs 25-35 us however small it is (a launch or two,
 * the staged copies, a stream synchronize), and the reference's own toy prove
 * (src/plonk-test.c, 4 gates) makes ~100 of them, each over <= 22 bytes -- 1.2 ms through the GPU
 * against the reference's 17.6 us on the CPU.  The threshold is the library option
 * PLK_OPT_DROPIN_HOST_WORK (plk_set_option; default 32768, 0 = every call on the GPU), compared
 * with a cost estimate in roughly nanoseconds of the loops below at -O2:
 *   poly_mul        la * lb                 (one integer multiply-add per term)
 *   poly_divide     2 * (nl - dl + 1) * dl  (hf_mul + hf_sub per term)
 *   poly_eval       2 * len
 *   srs_eval_at_s   300 * n                 (g1_mul + g1_add: about 10 GF(101) inversions per point;
 *                                            the reference's fold measures ~285 ns per point)
 *   matrix_mul      m * k * n
 *   matrix_inv      4 * n^3                 (Gauss-Jordan on the n x 2n augmented matrix)
 * At the default the whole toy prove stays on the host, while every config-sized call (C2-C5:
 * 2^16+ points, 2^19-coefficient products) goes to the GPU.
 *
 * This is product code of the drop-in, restated from the reference's definitions (cited per
 * function) over this directory's hf.h / g1.h; the results are the reference's bytes for ANY
 * input bytes, non-canonical encodings included, exactly as the GPU path's. It is not a fallback:
 * which side runs a call depends on its size only, and a large call without a GPU still fails
 * loudly (PLK_ERR_NODEV). */
#ifndef PLK_HOST_H
#define PLK_HOST_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "hf.h"
#include "g1.h"
#include "plonkhip.h"

/* a * b, saturated (cost estimates only) */
static inline uint64_t plk_host_mul_(uint64_t a, uint64_t b) {
  return (a && b > UINT64_MAX / a) ? UINT64_MAX : a * b;
}

/* true when a call of this cost estimate runs on the host */
static inline int plk_host_small_(uint64_t work) {
  int64_t t = plk_get_option(PLK_OPT_DROPIN_HOST_WORK);
  return t > 0 && work <= (uint64_t)t;
}

static inline HF plk_hf_(uint8_t v) {
  HF h = {v};
  return h;
}

static inline size_t plk_host_trim_(const uint8_t *c, size_t n) {
  while (n > 1 && c[n - 1] == 0) n--;
  return n;
}

/* src/poly.h:106-122 (la, lb >= 1).  The reference adds hf_mul(a_i, b_j) into a zeroed
 * coefficient with hf_add; every hf_mul result is a residue in [0, 16] and hf_add of two residues is
 * their sum mod 17, so coefficient k is (sum over i + j = k of a_i b_j) mod 17 -- each raw product
 * < 2^16 is reduced exactly either way.  Output-stationary: one reduction per coefficient.
 * out: la + lb - 1 bytes; returns the trimmed length. */
static inline size_t plk_host_poly_mul(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out) {
  const size_t rl = la + lb - 1;
  for (size_t k = 0; k < rl; k++) {
    const size_t lo = k >= lb ? k - lb + 1 : 0, hi = k < la ? k : la - 1;
    uint64_t s = 0;
    for (size_t i = lo; i <= hi; i++) s += (uint32_t)a[i] * b[k - i];
    out[k] = (uint8_t)(s % MODULO_HF);
  }
  return plk_host_trim_(out, rl);
}

/* src/poly.h:124-177, step for step in hf arithmetic (the remainder's raw bytes go through hf_sub
 * exactly as the reference's loop sends them).  q and r hold nl bytes each (>= 1); the divisor's lead
 * byte must be a GF(17) value (the reference indexes its inverse table out of bounds otherwise --
 * rejected here as by the library, plk_poly_divide). */
static inline int plk_host_poly_divide(const uint8_t *num, size_t nl, const uint8_t *den, size_t dl, uint8_t *q,
                                       size_t *ql, uint8_t *r, size_t *rl) {
  const uint8_t lead = den[dl - 1];
  if (lead >= MODULO_HF) return PLK_ERR_ARG;
  const HF inv = hf_inv(plk_hf_(lead));
  for (size_t i = 0; i < nl; i++) {
    r[i] = num[i];
    q[i] = 0;
  }
  if (nl == 0) q[0] = 0;
  for (size_t i = nl; i-- > dl - 1;) {   /* i = nl - 1 down to dl - 1 */
    const HF c = hf_mul(plk_hf_(r[i]), inv);
    q[i - (dl - 1)] = c.value;
    for (size_t j = 0; j < dl; j++) r[i - j] = hf_sub(plk_hf_(r[i - j]), hf_mul(c, plk_hf_(den[dl - 1 - j]))).value;
  }
  *ql = plk_host_trim_(q, nl >= dl ? nl - dl + 1 : 1);
  size_t n = dl - 1 < nl ? dl - 1 : nl;
  *rl = n ? plk_host_trim_(r, n) : 0;
  return PLK_OK;
}

/* Horner, src/poly.h:265-272 */
static inline uint8_t plk_host_poly_eval(const uint8_t *c, size_t len, uint8_t x) {
  HF y = hf_zero();
  for (size_t i = len; i-- > 0;) y = hf_add(hf_mul(y, plk_hf_(x)), plk_hf_(c[i]));
  return y.value;
}

/* srs_eval_at_s's fold, src/srs.h:59-66: acc = g1_add(acc, g1_mul(P_i, c_i)) from the identity, in
 * point order (order matters for non-canonical encodings; for group elements any order agrees) */
static inline G1 plk_host_msm(const G1 *pts, const HF *sc, size_t n) {
  G1 acc = g1_identity();
  for (size_t i = 0; i < n; i++) {
    G1 t = g1_mul(&pts[i], sc[i].value);
    acc = g1_add(&acc, &t);
  }
  return acc;
}

/* src/matrix.h:82-97: out[i][j] = sum_k a[i][k] b[k][j] mod 17 (hf_add of residues, as poly_mul) */
static inline void plk_host_matrix_mul(const uint8_t *a, size_t m, size_t k, const uint8_t *b, size_t n,
                                       uint8_t *out) {
  for (size_t i = 0; i < m; i++)
    for (size_t j = 0; j < n; j++) {
      uint64_t s = 0;
      for (size_t t = 0; t < k; t++) s += (uint32_t)a[i * k + t] * b[t * n + j];
      out[i * n + j] = (uint8_t)(s % MODULO_HF);
    }
}

#endif /* PLK_HOST_H */
