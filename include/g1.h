/* Drop-in for the reference's src/g1.h: affine points of y^2 = x^3 + 3 over GF(101)
 * (src/g1.h:8-107).  Same guard, 3-byte struct layout {x, y, infinite}, names and formulas;
 * restated from scratch.  Single-point ops stay on the host; the multi-scalar
 * multiplication that dominates the prover is srs_eval_at_s in srs.h (GPU). */
#ifndef G1_H
#define G1_H

#include <stdbool.h>
#include <stdint.h>
#include "gf.h"

typedef struct {
  GF x, y;
  bool infinite;
} G1;

static inline G1 g1_new(uint64_t x, uint64_t y) {
  G1 p = {f101((int64_t)x), f101((int64_t)y), false};
  return p;
}
static inline G1 g1_generator(void) { return g1_new(1, 2); }
static inline G1 g1_identity(void) {
  G1 p = {{0}, {0}, true};
  return p;
}
static inline bool g1_is_on_curve(const G1 *p) {
  if (p->infinite) return true;
  return gf_equal(gf_pow(p->y, 2), gf_add(gf_pow(p->x, 3), f101(3)));
}

/* tangent slope 3x^2 / 2y; the identity and points with y == 0 double to the identity */
static inline G1 g1_double(const G1 *a) {
  if (a->infinite || a->y.value == 0) return g1_identity();
  GF m = gf_div(gf_mul(f101(3), gf_mul(a->x, a->x)), gf_mul(f101(2), a->y));
  GF m2 = gf_mul(m, m);
  GF xr = gf_sub(m2, gf_mul(f101(2), a->x));
  GF yr = gf_sub(gf_mul(m, gf_sub(gf_mul(f101(3), a->x), m2)), a->y);
  return g1_new(xr.value, yr.value);
}

/* chord slope; equal x: inverse points give the identity, otherwise double */
static inline G1 g1_add(const G1 *a, const G1 *b) {
  if (a->infinite) return *b;
  if (b->infinite) return *a;
  if (gf_equal(a->x, b->x)) {
    if (gf_add(a->y, b->y).value == 0) return g1_identity();
    return g1_double(a);
  }
  GF m = gf_mul(gf_sub(b->y, a->y), gf_inv(gf_sub(b->x, a->x)));
  GF xr = gf_sub(gf_sub(gf_mul(m, m), a->x), b->x);
  GF yr = gf_sub(gf_mul(m, gf_sub(a->x, xr)), a->y);
  return g1_new(xr.value, yr.value);
}

static inline G1 g1_neg(G1 *a) {
  if (a->infinite) return *a;
  return g1_new(a->x.value, gf_neg(a->y).value);
}

/* LSB-first double-and-add */
static inline G1 g1_mul(const G1 *p, uint64_t k) {
  G1 acc = g1_identity(), run = *p;
  for (; k; k >>= 1) {
    if (k & 1) acc = g1_add(&acc, &run);
    run = g1_double(&run);
  }
  return acc;
}

static inline GF g1_generator_subgroup_size(void) { return f101(17); }

#endif /* G1_H */
