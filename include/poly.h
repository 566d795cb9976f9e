/* Drop-in for the reference's src/poly.h: polynomials over GF(17) (src/poly.h:10-321).
 * Same guard, POLY layout, names and semantics (constructor trims trailing zeros, results
 * are freshly malloc'ed and freed with poly_free).  poly_mul -- the prover's hot
 * polynomial operation (17 calls per proof) -- runs on the GPU through plk_poly_mul
 * (exact NTT / direct convolution, include/plonkhip.h), and so do poly_divide and poly_eval
 * (plk_poly_divide, plk_poly_eval), except calls of toy size, which stay on
 * the host (plk_host.h: SURVEY 8(b)'s small-size policy).  The other operations are O(n)
 * coefficient copies and scalings, host code restated from scratch. */
#ifndef POLY_H
#define POLY_H

#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include "hf.h"
#include "plonkhip.h"
#include "plk_host.h"

typedef struct {
  HF *coeffs;
  size_t len;
} POLY;

static inline void *poly_xalloc_(size_t n, const char *who) {
  void *p = calloc(n ? n : 1, 1);
  if (!p) {
    fprintf(stderr, "Memory allocation failed in %s\n", who);
    exit(EXIT_FAILURE);
  }
  return p;
}

/* copy + trim trailing zeros (keeps at least one coefficient) */
static POLY poly_new_internal(const HF *coeffs, size_t len) {
  while (len > 1 && coeffs[len - 1].value == 0) len--;
  POLY p;
  p.len = len;
  p.coeffs = (HF *)poly_xalloc_(len, "poly_new_internal");
  if (len) memcpy(p.coeffs, coeffs, len);
  return p;
}
static inline POLY poly_new(const HF *coeffs, size_t len) { return poly_new_internal(coeffs, len); }
static inline POLY poly_zero(void) { HF z = {0}; return poly_new(&z, 1); }
static inline POLY poly_one(void) { HF o = {1}; return poly_new(&o, 1); }
static inline bool poly_is_zero(const POLY *p) {
  for (size_t i = 0; i < p->len; i++)
    if (p->coeffs[i].value) return false;
  return true;
}

/* adds b to the constant term IN PLACE and returns the same storage (src/poly.h:67-70) */
static inline POLY poly_add_hf(POLY *a, const HF b) {
  a->coeffs[0] = hf_add(a->coeffs[0], b);
  return *a;
}

static inline POLY poly_addsub_(const POLY *a, const POLY *b, int sub, const char *who) {
  size_t n = a->len > b->len ? a->len : b->len;
  HF *c = (HF *)poly_xalloc_(n, who);
  for (size_t i = 0; i < n; i++) {
    HF x = i < a->len ? a->coeffs[i] : hf_zero();
    HF y = i < b->len ? b->coeffs[i] : hf_zero();
    c[i] = sub ? hf_sub(x, y) : hf_add(x, y);
  }
  POLY r = poly_new(c, n);
  free(c);
  return r;
}
static inline POLY poly_add(const POLY *a, const POLY *b) { return poly_addsub_(a, b, 0, "poly_add"); }
static inline POLY poly_sub(const POLY *a, const POLY *b) { return poly_addsub_(a, b, 1, "poly_sub"); }

/* GPU: product over GF(17), trimmed (reference schoolbook src/poly.h:106-122); toy sizes on the host */
static inline POLY poly_mul(const POLY *a, const POLY *b) {
  size_t rl = a->len + b->len - 1;
  HF *c = (HF *)poly_xalloc_(rl, "poly_mul");
  size_t n = 0;
  if (a->len && b->len && plk_host_small_(plk_host_mul_(a->len, b->len))) {
    POLY r;
    r.len = plk_host_poly_mul((const uint8_t *)a->coeffs, a->len, (const uint8_t *)b->coeffs, b->len, (uint8_t *)c);
    r.coeffs = c;
    return r;
  }
  int rc = plk_poly_mul((const uint8_t *)a->coeffs, a->len, (const uint8_t *)b->coeffs, b->len,
                        (uint8_t *)c, &n);
  if (rc != PLK_OK) {
    fprintf(stderr, "poly_mul failed on the GPU (libplonkhip error %d): %s\n", rc, plk_last_error());
    exit(EXIT_FAILURE);
  }
  POLY r;
  r.len = n;
  r.coeffs = c; /* already trimmed to n; the tail of the buffer is unused */
  return r;
}

/* long division num = quot * den + rem (src/poly.h:124-177) on the GPU (plk_poly_divide:
 * parallel chain scans for x^m-type divisors such as Z_H and x - z, the reference's loop on the
 * device otherwise) */
static inline void poly_divide(const POLY *num, const POLY *den, POLY *quot, POLY *rem) {
  if (poly_is_zero(den)) {
    fprintf(stderr, "Division by zero polynomial in poly_divide\n");
    exit(EXIT_FAILURE);
  }
  size_t nl = num->len, dl = den->len;
  HF *q = (HF *)poly_xalloc_(nl, "poly_divide");
  HF *r = (HF *)poly_xalloc_(nl, "poly_divide");
  size_t ql = 0, rl = 0;
  int rc;
  if (plk_host_small_(plk_host_mul_(2 * (nl >= dl ? nl - dl + 1 : 1), dl))) {
    rc = plk_host_poly_divide((const uint8_t *)num->coeffs, nl, (const uint8_t *)den->coeffs, dl, (uint8_t *)q, &ql,
                              (uint8_t *)r, &rl);
    if (rc != PLK_OK) {
      fprintf(stderr, "poly_divide: divisor lead byte %u is not a GF(17) value (reference behaviour undefined)\n",
              den->coeffs[dl - 1].value);
      exit(EXIT_FAILURE);
    }
  } else {
    rc = plk_poly_divide((const uint8_t *)num->coeffs, nl, (const uint8_t *)den->coeffs, dl, (uint8_t *)q, &ql,
                         (uint8_t *)r, &rl);
  }
  if (rc != PLK_OK) {
    fprintf(stderr, "poly_divide failed on the GPU (libplonkhip error %d): %s\n", rc, plk_last_error());
    exit(EXIT_FAILURE);
  }
  quot->coeffs = q;   /* already trimmed to ql / rl; the tails of the buffers are unused */
  quot->len = ql;
  rem->coeffs = r;
  rem->len = rl;
}

static inline POLY poly_scale(const POLY *p, HF s) {
  if (s.value == 0) return poly_zero();
  HF *c = (HF *)poly_xalloc_(p->len, "poly_scale");
  for (size_t i = 0; i < p->len; i++) c[i] = hf_mul(p->coeffs[i], s);
  POLY r = poly_new(c, p->len);
  free(c);
  return r;
}

static inline POLY poly_shift(const POLY *p, size_t shift) {
  if (poly_is_zero(p)) return poly_zero();
  HF *c = (HF *)poly_xalloc_(p->len + shift, "poly_shift");
  memcpy(c + shift, p->coeffs, p->len);
  POLY r = poly_new(c, p->len + shift);
  free(c);
  return r;
}

static inline POLY poly_slice(const POLY *p, size_t start, size_t end) {
  if (start >= end || end > p->len) {
    fprintf(stderr, "Invalid slice indices in poly_slice\n");
    exit(EXIT_FAILURE);
  }
  return poly_new(p->coeffs + start, end - start);
}

static inline POLY poly_negate(const POLY *p) {
  HF *c = (HF *)poly_xalloc_(p->len, "poly_negate");
  for (size_t i = 0; i < p->len; i++) c[i] = hf_neg(p->coeffs[i]);
  POLY r = poly_new(c, p->len);
  free(c);
  return r;
}

static inline void poly_free(POLY *p) {
  free(p->coeffs);
  p->coeffs = NULL;
  p->len = 0;
}

/* Horner (src/poly.h:265-272) on the GPU (plk_poly_eval: exact for every byte value); toy sizes on the host */
static inline HF poly_eval(const POLY *p, HF x) {
  HF y = {0};
  if (plk_host_small_(plk_host_mul_(2, p->len))) {
    y.value = plk_host_poly_eval((const uint8_t *)p->coeffs, p->len, x.value);
    return y;
  }
  int rc = plk_poly_eval((const uint8_t *)p->coeffs, p->len, x.value, &y.value);
  if (rc != PLK_OK) {
    fprintf(stderr, "poly_eval failed on the GPU (libplonkhip error %d): %s\n", rc, plk_last_error());
    exit(EXIT_FAILURE);
  }
  return y;
}

/* prod_i (x - points[i]) */
static inline POLY poly_z(const HF *points, size_t len) {
  POLY acc = poly_one();
  for (size_t i = 0; i < len; i++) {
    HF c[2] = {hf_neg(points[i]), hf_one()};
    POLY t = poly_new(c, 2);
    POLY nxt = poly_mul(&acc, &t);
    poly_free(&acc);
    poly_free(&t);
    acc = nxt;
  }
  return acc;
}

/* sum_j y_j prod_{i != j} (x - x_i) / (x_j - x_i) */
static inline POLY poly_lagrange(const HF *xs, const HF *ys, size_t len) {
  POLY l = poly_zero();
  for (size_t j = 0; j < len; j++) {
    POLY lj = poly_one();
    for (size_t i = 0; i < len; i++) {
      if (i == j) continue;
      HF dinv = hf_inv(hf_sub(xs[j], xs[i]));
      if (dinv.value == 0) {
        fprintf(stderr, "Error: Lagrange polynomial x points must be unique\n");
        exit(EXIT_FAILURE);
      }
      HF c[2] = {hf_neg(hf_mul(dinv, xs[i])), dinv};
      POLY t = poly_new(c, 2);
      POLY nxt = poly_mul(&lj, &t);
      poly_free(&lj);
      poly_free(&t);
      lj = nxt;
    }
    POLY s = poly_scale(&lj, ys[j]);
    POLY nl = poly_add(&l, &s);
    poly_free(&l);
    poly_free(&lj);
    poly_free(&s);
    l = nl;
  }
  return l;
}

#endif /* POLY_H */
