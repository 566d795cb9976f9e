/* Drop-in for the reference's src/matrix.h (GF(17) matrices, row-major HF bytes): same guard,
 * MATRIX layout, names and error text.  matrix_mul and matrix_inv -- what plonk_new builds the
 * Vandermonde inverse with (src/plonk.h:105-113) and interpolate_at_h applies
 * (src/plonk.h:162-195) -- run on the GPU through plk_matrix_mul / plk_matrix_inv
 * (include/plonkhip.h), toy sizes on the host (plk_host.h); the accessors are host
 * code restated from scratch. */
#ifndef MATRIX_H
#define MATRIX_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "hf.h"
#include "plonkhip.h"
#include "plk_host.h"

typedef struct {
  size_t m;  /* rows */
  size_t n;  /* columns */
  HF *v;     /* m * n values, row-major */
} MATRIX;

static inline MATRIX matrix_zero(size_t m, size_t n) {
  MATRIX r = {m, n, (HF *)calloc(m * n + 1, sizeof(HF))};
  if (!r.v) {
    fprintf(stderr, "Memory allocation failed in matrix_zero\n");
    exit(EXIT_FAILURE);
  }
  return r;
}

static inline MATRIX matrix_new(HF *v, size_t m, size_t n) {
  MATRIX r = {m, n, (HF *)malloc(m * n + 1)};
  if (!r.v) {
    fprintf(stderr, "Memory allocation failed in matrix_new\n");
    exit(EXIT_FAILURE);
  }
  if (m != 0 && n != 0) memcpy(r.v, v, m * n);
  return r;
}

static inline HF matrix_get(const MATRIX *a, size_t row, size_t col) {
  if (row >= a->m || col >= a->n) {
    fprintf(stderr, "Index out of bounds in matrix_get\n");
    exit(EXIT_FAILURE);
  }
  return a->v[row * a->n + col];
}

static inline void matrix_set(MATRIX *a, size_t row, size_t col, HF value) {
  if (row >= a->m || col >= a->n) {
    fprintf(stderr, "Index out of bounds in matrix_set\n");
    exit(EXIT_FAILURE);
  }
  a->v[row * a->n + col] = value;
}

static inline void matrix_free(MATRIX *a) {
  free(a->v);
  a->v = NULL;
  a->m = 0;
  a->n = 0;
}

static inline MATRIX matrix_add(const MATRIX *a, const MATRIX *b) {
  if (a->m != b->m || a->n != b->n) {
    fprintf(stderr, "Matrix dimensions must match for additoin\n");
    exit(EXIT_FAILURE);
  }
  MATRIX r = matrix_zero(a->m, a->n);
  for (size_t i = 0; i < a->m * a->n; i++) r.v[i] = hf_add(a->v[i], b->v[i]);
  return r;
}

static inline void matrix_gpu_fail_(const char *who, int rc) {
  fprintf(stderr, "%s failed on the GPU (libplonkhip error %d): %s\n", who, rc, plk_last_error());
  exit(EXIT_FAILURE);
}

static inline MATRIX matrix_mul(const MATRIX *a, const MATRIX *b) {
  if (a->n != b->m) {
    fprintf(stderr, "Matrix multiplication error: Dimensions (%zu x %zu) and (%zu x %zu) incompatible.\n", a->m,
            a->n, b->m, b->n);
    exit(EXIT_FAILURE);
  }
  MATRIX r = matrix_zero(a->m, b->n);
  if (plk_host_small_(plk_host_mul_(plk_host_mul_(a->m, a->n), b->n))) {
    plk_host_matrix_mul((const uint8_t *)a->v, a->m, a->n, (const uint8_t *)b->v, b->n, (uint8_t *)r.v);
    return r;
  }
  int rc = plk_matrix_mul((const uint8_t *)a->v, a->m, a->n, (const uint8_t *)b->v, b->n, (uint8_t *)r.v);
  if (rc != PLK_OK) matrix_gpu_fail_("matrix_mul", rc);
  return r;
}

/* in-place Gauss-Jordan on the device (the same pivot order as the reference) */
static inline void matrix_gauss_jordan(MATRIX *a);

static inline MATRIX matrix_inv(const MATRIX *a) {
  if (a->m != a->n) {
    fprintf(stderr, "Only square matrices can be inverted\n");
    exit(EXIT_FAILURE);
  }
  const size_t n = a->n;
  if (plk_host_small_(plk_host_mul_(4 * n, plk_host_mul_(n, n)))) {
    /* src/matrix.h:150-176: Gauss-Jordan on [a | I], the right half is the inverse.  A raw pivot byte
       would make the reference read past hf_inverses: rejected as by plk_matrix_inv */
    for (size_t i = 0; i < n * n; i++)
      if (a->v[i].value >= MODULO_HF) {
        fprintf(stderr, "matrix_inv: entry %zu = %u is not a GF(17) value (reference behaviour undefined)\n", i,
                a->v[i].value);
        exit(EXIT_FAILURE);
      }
    MATRIX aug = matrix_zero(n, 2 * n);
    for (size_t i = 0; i < n; i++) {
      memcpy(aug.v + i * 2 * n, a->v + i * n, n);
      aug.v[i * 2 * n + n + i] = hf_one();
    }
    matrix_gauss_jordan(&aug);
    MATRIX r = matrix_zero(n, n);
    for (size_t i = 0; i < n; i++) memcpy(r.v + i * n, aug.v + i * 2 * n + n, n);
    matrix_free(&aug);
    return r;
  }
  MATRIX r = matrix_zero(a->n, a->n);
  int rc = plk_matrix_inv((const uint8_t *)a->v, a->n, (uint8_t *)r.v);
  if (rc != PLK_OK) matrix_gpu_fail_("matrix_inv", rc);
  return r;
}

/* matrix_gauss_jordan on an arbitrary m x n matrix is only a helper of matrix_inv in the
 * reference (src/matrix.h:100-147); restated on the host for callers that use it directly. */
static inline void matrix_gauss_jordan(MATRIX *a) {
  size_t lead = 0;
  for (size_t r = 0; r < a->m; r++) {
    if (a->n <= lead) return;
    size_t i = r;
    while (a->v[i * a->n + lead].value == 0) {
      if (++i == a->m) {
        i = r;
        if (++lead == a->n) return;
      }
    }
    if (i != r)
      for (size_t k = 0; k < a->n; k++) {
        HF t = a->v[i * a->n + k];
        a->v[i * a->n + k] = a->v[r * a->n + k];
        a->v[r * a->n + k] = t;
      }
    HF div = a->v[r * a->n + lead];
    if (div.value != 0)
      for (size_t k = 0; k < a->n; k++) a->v[r * a->n + k] = hf_div(a->v[r * a->n + k], div);
    for (size_t ii = 0; ii < a->m; ii++) {
      if (ii == r) continue;
      HF mult = a->v[ii * a->n + lead];
      for (size_t k = 0; k < a->n; k++)
        a->v[ii * a->n + k] = hf_sub(a->v[ii * a->n + k], hf_mul(a->v[r * a->n + k], mult));
    }
    lead++;
  }
}

#endif /* MATRIX_H */
