/*
 * TEST INFRASTRUCTURE ONLY.  Host sanitizer build: the drop-in headers' host
 * code (include/gf.h hf.h g1.h srs.h poly.h matrix.h -- everything that does not call the GPU)
 * and the oracle restatement (oracle/oracle.c) exercised under -fsanitize=address,undefined
 * over every raw byte value and ragged sizes (0-length polynomials included).  Built and run by
 * `make -C oracle sanitize` (tests/test_sanitize_cpu.py); any report aborts with a non-zero exit.
 */
#include "prelude.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* oracle.c */
void orc_g1_add(const uint8_t *a, const uint8_t *b, uint8_t *out);
void orc_g1_double(const uint8_t *a, uint8_t *out);
void orc_g1_mul(const uint8_t *a, uint64_t k, uint8_t *out);
void orc_msm_fold(const uint8_t *pts, const uint8_t *sc, size_t n, uint8_t *out);
int orc_msm_dlog(const uint8_t *pts, const uint8_t *sc, size_t n, uint8_t *out);
size_t orc_poly_mul(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out);
size_t orc_poly_mul_ntt(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out);
int orc_poly_divide(const uint8_t *num, size_t ln, const uint8_t *den, size_t ld, uint8_t *q, size_t *lq, uint8_t *r,
                    size_t *lr);
uint8_t orc_poly_eval(const uint8_t *p, size_t len, uint8_t x);
void orc_matrix_mul(const uint8_t *a, size_t m, size_t k, const uint8_t *b, size_t n, uint8_t *out);
void orc_matrix_inv(const uint8_t *a, size_t n, uint8_t *out);

static uint64_t rs = 0x243F6A8885A308D3ull;
static uint64_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}
static void fill(uint8_t *p, size_t n, unsigned mod) {
  for (size_t i = 0; i < n; i++) p[i] = (uint8_t)(rnd() % mod);
}

int main(void) {
  unsigned long checks = 0;
  /* field and group ops of the drop-in headers over raw bytes */
  for (int a = 0; a < 256; a++)
    for (int b = 0; b < 256; b++) {
      GF x = {(uint8_t)a}, y = {(uint8_t)b};
      HF h = {(uint8_t)a}, k = {(uint8_t)(b % 17)};
      checks += gf_add(x, y).value + gf_sub(x, y).value + gf_mul(x, y).value + gf_div(x, y).value;
      checks += hf_add(h, k).value + hf_sub(h, k).value + hf_mul(h, k).value + hf_div(h, k).value;
    }
  for (int i = 0; i < 20000; i++) {
    uint8_t p[3], q[3], o1[3], o2[3];
    fill(p, 3, i & 1 ? 256 : 101);
    fill(q, 3, i & 2 ? 256 : 101);
    p[2] &= 1;
    q[2] &= 1;
    G1 P, Q;
    memcpy(&P, p, 3);
    memcpy(&Q, q, 3);
    G1 s = g1_add(&P, &Q), d = g1_double(&P), m = g1_mul(&P, rnd() % 300);
    orc_g1_add(p, q, o1);
    memcpy(o2, &s, 3);
    if (memcmp(o1, o2, 3)) { fprintf(stderr, "g1_add mismatch\n"); return 1; }
    checks += d.x.value + m.y.value + g1_is_on_curve(&P);
  }
  SRS srs = srs_create(f101(5), 64);
  checks += srs.g1s[0].x.value;
  srs_free(&srs);
  /* host polynomial helpers */
  for (int i = 0; i < 3000; i++) {
    size_t la = rnd() % 40, lb = rnd() % 40;
    HF *a = calloc(la + 1, 1), *b = calloc(lb + 1, 1);
    fill((uint8_t *)a, la, i & 1 ? 256 : 17);
    fill((uint8_t *)b, lb, 17);
    POLY A = poly_new(a, la), B = poly_new(b, lb);
    POLY s = poly_add(&A, &B), t = poly_sub(&A, &B), u = poly_scale(&A, b[0]), v = poly_shift(&B, rnd() % 5);
    POLY w = poly_negate(&A), z = poly_add_hf(&A, b[0]);   /* z aliases A (in place, as the reference) */
    if (A.len > 1) {
      POLY sl = poly_slice(&A, 0, A.len - 1);
      poly_free(&sl);
    }
    checks += s.len + t.len + u.len + v.len + w.len + z.len + poly_is_zero(&A);
    poly_free(&s); poly_free(&t); poly_free(&u); poly_free(&v); poly_free(&w);
    poly_free(&A); poly_free(&B);
    free(a);
    free(b);
  }
  /* the drop-in's small-size host path (include/plk_host.h) against the oracle over raw bytes */
  for (int i = 0; i < 2000; i++) {
    size_t la = 1 + rnd() % 80, lb = 1 + rnd() % 80, n = rnd() % 120;
    uint8_t *a = malloc(la), *b = malloc(lb), *o = malloc(la + lb), *o2 = malloc(la + lb);
    fill(a, la, i & 1 ? 256 : 17);
    fill(b, lb, i & 2 ? 256 : 17);
    if (i % 5 == 0) a[la - 1] = 0;
    size_t l1 = plk_host_poly_mul(a, la, b, lb, o), l2 = orc_poly_mul(a, la, b, lb, o2);
    if (l1 != l2 || memcmp(o, o2, l1)) { fprintf(stderr, "host poly_mul mismatch\n"); return 1; }
    uint8_t x = (uint8_t)rnd();
    if (plk_host_poly_eval(a, la, x) != orc_poly_eval(a, la, x)) { fprintf(stderr, "host poly_eval mismatch\n"); return 1; }
    size_t dl = 1 + rnd() % (lb < 9 ? lb : 9), q1, r1, q2, r2;
    uint8_t *q = malloc(la + 1), *r = malloc(la + 1), *qq = malloc(la + 1), *rr = malloc(la + 1);
    fill(b, dl, 17);
    b[dl - 1] = (uint8_t)(1 + rnd() % 16);
    if (plk_host_poly_divide(a, la, b, dl, q, &q1, r, &r1) != PLK_OK) { fprintf(stderr, "host divide rc\n"); return 1; }
    orc_poly_divide(a, la, b, dl, qq, &q2, rr, &r2);
    if (q1 != q2 || r1 != r2 || memcmp(q, qq, q1) || memcmp(r, rr, r1)) {
      fprintf(stderr, "host poly_divide mismatch\n");
      return 1;
    }
    uint8_t *pts = malloc(3 * n + 1), *sc = malloc(n + 1), m1[3], m2[3];
    fill(pts, 3 * n, i & 4 ? 256 : 101);
    fill(sc, n, i & 8 ? 256 : 17);
    for (size_t j = 0; j < n; j++) pts[3 * j + 2] &= 1;   /* a bool flag byte outside {0, 1} is UB in C */
    G1 h = plk_host_msm((const G1 *)pts, (const HF *)sc, n);
    memcpy(m1, &h, 3);
    orc_msm_fold(pts, sc, n, m2);
    if (memcmp(m1, m2, 3)) { fprintf(stderr, "host msm mismatch\n"); return 1; }
    size_t mm = 1 + rnd() % 7, kk = 1 + rnd() % 7, nn = 1 + rnd() % 7;
    uint8_t A[49], B[49], C1[49], C2[49];
    fill(A, mm * kk, 256);
    fill(B, kk * nn, 256);
    plk_host_matrix_mul(A, mm, kk, B, nn, C1);
    orc_matrix_mul(A, mm, kk, B, nn, C2);
    if (memcmp(C1, C2, mm * nn)) { fprintf(stderr, "host matrix_mul mismatch\n"); return 1; }
    checks += l1 + q1 + r1 + m1[0];
    free(a); free(b); free(o); free(o2); free(q); free(r); free(qq); free(rr); free(pts); free(sc);
  }
  /* matrices: host accessors and the restated Gauss-Jordan */
  for (int n = 1; n <= 17; n++) {
    MATRIX M = matrix_zero((size_t)n, (size_t)n), N = matrix_zero((size_t)n, (size_t)n);
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) matrix_set(&M, (size_t)r, (size_t)c, (HF){(uint8_t)(rnd() % 17)});
    memcpy(N.v, M.v, (size_t)(n * n));
    MATRIX S = matrix_add(&M, &N);
    matrix_gauss_jordan(&N);
    checks += matrix_get(&S, 0, 0).value + N.v[0].value;
    matrix_free(&M); matrix_free(&N); matrix_free(&S);
  }
  /* the oracle over ragged sizes and raw bytes */
  for (int i = 0; i < 400; i++) {
    size_t n = rnd() % 3000;
    uint8_t *pts = malloc(3 * n + 1), *sc = malloc(n + 1), out[3];
    fill(pts, 3 * n, i & 1 ? 256 : 101);
    fill(sc, n, 256);
    orc_msm_fold(pts, sc, n, out);
    checks += (unsigned long)orc_msm_dlog(pts, sc, n, out);
    free(pts);
    free(sc);
    size_t la = 1 + rnd() % 700, lb = 1 + rnd() % 700;
    uint8_t *a = malloc(la), *b = malloc(lb), *o = malloc(la + lb), *o2 = malloc(la + lb);
    fill(a, la, i & 2 ? 256 : 17);
    fill(b, lb, 17);
    size_t l1 = orc_poly_mul(a, la, b, lb, o);
    size_t l2 = orc_poly_mul_ntt(a, la, b, lb, o2);
    if (l1 != l2 || memcmp(o, o2, l1)) { fprintf(stderr, "poly_mul mismatch\n"); return 1; }
    size_t lq, lr;
    uint8_t *q = malloc(la + 1), *r = malloc(la + 1);
    b[lb - 1] = (uint8_t)(1 + rnd() % 16);
    checks += (unsigned long)orc_poly_divide(a, la, b, lb, q, &lq, r, &lr) + lq + lr;
    checks += orc_poly_eval(a, la, (uint8_t)rnd());
    free(a); free(b); free(o); free(o2); free(q); free(r);
    size_t m = 1 + rnd() % 9, k = 1 + rnd() % 9, nn = 1 + rnd() % 9;
    uint8_t *A = malloc(m * k), *B = malloc(k * nn), *C = malloc(m * nn), *I = malloc(m * m);
    fill(A, m * k, 256);
    fill(B, k * nn, 256);
    orc_matrix_mul(A, m, k, B, nn, C);
    fill(A, m * m < m * k ? m * m : m * k, 17);
    if (m <= k) orc_matrix_inv(A, m, I);
    checks += C[0];
    free(A); free(B); free(C); free(I);
  }
  printf("sanitize ok (%lu)\n", checks);
  return 0;
}
