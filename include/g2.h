/* Drop-in for the reference's src/g2.h (src/g2.h:8-84): the twisted G2 points carried in the
 * SRS.  Needed only so SRS keeps its layout and srs_create its two G2 entries; verifier
 * side, not on the hot path.  Same guard, struct and names; restated from scratch. */
#ifndef G2_H
#define G2_H

#include <stdint.h>
#include "gf.h"

typedef struct {
  GF x, y;
} G2;

static inline G2 g2_new(uint64_t x, uint64_t y) {
  G2 p = {f101((int64_t)x), f101((int64_t)y)};
  return p;
}
static inline G2 g2_generator(void) { return g2_new(36, 31); }
static inline uint64_t g2_embedding_degree(void) { return 2; }
static inline G2 g2_neg(G2 *p) { return g2_new(p->x.value, gf_neg(p->y).value); }

/* y is the coefficient of u with u^2 = -2, so the slope terms carry 1/(-2) factors
 * exactly as src/g2.h:32-66 does. */
static inline G2 g2_add(const G2 *p, const G2 *q) {
  const GF two = f101(2), three = f101(3), ntwo = gf_neg(f101(2));
  GF x, y;
  if (gf_equal(p->x, q->x) && gf_equal(p->y, q->y)) {
    GF m = gf_div(gf_mul(three, gf_mul(p->x, p->x)), gf_mul(two, p->y));
    GF ninv = gf_inv(ntwo);
    GF mm = gf_mul(gf_mul(m, m), ninv);
    x = gf_sub(mm, gf_mul(two, p->x));
    y = gf_sub(gf_mul(gf_mul(ninv, m), gf_sub(gf_mul(three, p->x), mm)), p->y);
  } else {
    GF m = gf_div(gf_sub(q->y, p->y), gf_sub(q->x, p->x));
    GF mm = gf_mul(gf_mul(m, m), ntwo);
    x = gf_sub(gf_sub(mm, p->x), q->x);
    y = gf_sub(gf_mul(m, gf_sub(p->x, x)), p->y);
  }
  return g2_new(x.value, y.value);
}

/* LSB-first double-and-add without an explicit identity (src/g2.h:68-84) */
static inline G2 g2_mul(G2 base, uint64_t k) {
  G2 acc = {{0}, {0}};
  int have = 0;
  for (; k; k >>= 1) {
    if (k & 1) {
      if (have) acc = g2_add(&acc, &base);
      else { acc = base; have = 1; }
    }
    base = g2_add(&base, &base);
  }
  return acc;
}

#endif /* G2_H */
