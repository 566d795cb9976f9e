/* Drop-in for the reference's src/gf.h: GF(101), the curve base field (src/gf.h:8-182).
 * Same guard (FE_H), type and names; restated from scratch, static inline. */
#ifndef FE_H
#define FE_H

#include <stdbool.h>
#include <stdint.h>
#include "hf.h"

#define MODULO_GF 101

typedef struct {
  uint8_t value; /* canonical range [0, 100] */
} GF;

static inline GF gf_new(int64_t v) {
  int64_t r = v % MODULO_GF;
  GF g = {(uint8_t)(r < 0 ? r + MODULO_GF : r)};
  return g;
}
static inline GF f101(int64_t v) { return gf_new(v); }
static inline GF gf_zero(void) { GF g = {0}; return g; }
static inline GF gf_one(void) { GF g = {1}; return g; }
static inline bool is_odd(uint64_t n) { return (n & 1) != 0; }
static inline bool gf_equal(GF a, GF b) { return a.value == b.value; }

/* 16-bit sum / signed 16-bit difference with one conditional correction (src/gf.h:87-107) */
static inline GF gf_add(GF a, GF b) {
  uint16_t s = (uint16_t)(a.value + b.value);
  GF g = {(uint8_t)(s >= MODULO_GF ? s - MODULO_GF : s)};
  return g;
}
static inline GF gf_sub(GF a, GF b) {
  int16_t d = (int16_t)((int16_t)a.value - (int16_t)b.value);
  GF g = {(uint8_t)(d < 0 ? d + MODULO_GF : d)};
  return g;
}
static inline GF gf_mul(GF a, GF b) {
  GF g = {(uint8_t)(((uint16_t)a.value * (uint16_t)b.value) % MODULO_GF)};
  return g;
}
static inline GF gf_neg(GF a) {
  GF g = {(uint8_t)(a.value ? MODULO_GF - a.value : 0)};
  return g;
}
static inline GF gf_pow(GF base, uint64_t e) {
  GF r = gf_one();
  for (; e; e >>= 1) {
    if (is_odd(e)) r = gf_mul(r, base);
    base = gf_mul(base, base);
  }
  return r;
}
/* Fermat: a^(p-2); 0 maps to 0 */
static inline GF gf_inv(GF a) { return gf_pow(a, MODULO_GF - 2); }
static inline GF gf_div(GF a, GF b) { return gf_mul(a, gf_inv(b)); }
static inline GF gf_from_hf(HF h) { return gf_new(h.value); }

#endif /* FE_H */
