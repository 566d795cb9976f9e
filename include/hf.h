/* Drop-in for the reference's src/hf.h: GF(17), the scalar field.  Same include guard,
 * type and function names/semantics (src/hf.h:9-203), restated from scratch; the host
 * arithmetic here is not on the hot path (coefficient math of poly_mul runs on the GPU
 * behind poly.h).  Functions are static inline so any number of translation units may
 * include the header (the reference's headers are single-TU only). */
#ifndef HF_H
#define HF_H

#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define MODULO_HF 17

typedef struct {
  uint8_t value; /* canonical range [0, 16] */
} HF;

static inline HF hf_new(int64_t v) {
  int64_t r = v % MODULO_HF;
  HF h = {(uint8_t)(r < 0 ? r + MODULO_HF : r)};
  return h;
}
static inline HF f17(int64_t v) { return hf_new(v); }
static inline HF hf_zero(void) { HF h = {0}; return h; }
static inline HF hf_one(void) { HF h = {1}; return h; }
static inline bool hf_equal(HF a, HF b) { return a.value == b.value; }

/* 8-bit sum / signed 8-bit difference with one conditional correction, as src/hf.h:79-97 */
static inline HF hf_add(HF a, HF b) {
  uint8_t s = (uint8_t)(a.value + b.value);
  HF h = {(uint8_t)(s >= MODULO_HF ? s - MODULO_HF : s)};
  return h;
}
static inline HF hf_sub(HF a, HF b) {
  int8_t d = (int8_t)((int8_t)a.value - (int8_t)b.value);
  HF h = {(uint8_t)(d < 0 ? d + MODULO_HF : d)};
  return h;
}
static inline HF hf_mul(HF a, HF b) {
  HF h = {(uint8_t)(((uint16_t)a.value * (uint16_t)b.value) % MODULO_HF)};
  return h;
}
static inline HF hf_neg(HF a) {
  HF h = {(uint8_t)(a.value ? MODULO_HF - a.value : 0)};
  return h;
}
static inline HF hf_pow(HF base, uint64_t e) {
  HF r = hf_one();
  for (; e; e >>= 1) {
    if (e & 1) r = hf_mul(r, base);
    base = hf_mul(base, base);
  }
  return r;
}

/* a * a^-1 = 1 mod 17; entry 0 is 0 (the reference's x/0 == 0 convention) */
static const uint8_t hf_inverses[MODULO_HF] = {0, 1, 9, 6, 13, 7, 3, 5, 15, 2, 12, 14, 10, 4, 11, 8, 16};

static inline HF hf_inv(HF a) { HF h = {hf_inverses[a.value]}; return h; }
static inline HF hf_div(HF a, HF b) { return hf_mul(a, hf_inv(b)); }

#endif /* HF_H */
