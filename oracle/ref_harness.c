/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * Byte-buffer shim over the UNMODIFIED reference headers of kazuakiishiguro/plonk.c.
 * The headers are compiled where they lie (-I /root/reference/src, see oracle/Makefile);
 * nothing from them is copied here.  The shim only marshals plain byte arrays into the
 * reference's own structs and calls the reference functions, so that
 *   - tests/golden/make_golden.py can record golden vectors from the real reference, and
 *   - bench.py's cpu_baseline leg can time the real reference MSM / poly_mul
 * through ctypes.  Output: oracle/_ref/libplonkref.so (git-ignored, travels to the GPU box).
 *
 * Entry points and the reference functions they call:
 *   ref_g1_*          -> g1_add / g1_double / g1_mul / g1_is_on_curve   src/g1.h:26-103
 *   ref_msm           -> srs_eval_at_s                                  src/srs.h:53-68
 *   ref_poly_mul      -> poly_mul                                       src/poly.h:106-122
 *   ref_poly_divide   -> poly_divide                                    src/poly.h:124-177
 *   ref_poly_eval     -> poly_eval                                      src/poly.h:265-272
 *   ref_matrix_mul    -> matrix_mul                                     src/matrix.h:79-96
 *   ref_matrix_inv    -> matrix_inv (Gauss-Jordan)                      src/matrix.h:100-176
 *   ref_interpolate4  -> plonk_new + interpolate_at_h                   src/plonk.h:53,162
 *   ref_prove4        -> srs_create + plonk_new + plonk_prove           src/srs.h:18, src/plonk.h:53,223
 *   ref_plonk4_data   -> srs_create + plonk_new: h, k1_h, k2_h, h_pows_inv, z_h_x, g1s
 *
 * The same file compiled with `-include include/prelude.h -DPLK_NO_FORK` (target
 * _ref/libplonkref_dropin.so) is the DROP-IN demonstration: the reference's unmodified
 * plonk.h prover, with poly_mul / srs_eval_at_s resolved to libplonkhip (GPU).
 */
#include <stdint.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "plonk.h"

_Static_assert(sizeof(G1) == 3, "reference G1 is {GF x, GF y, bool infinite} = 3 bytes");
_Static_assert(sizeof(HF) == 1, "reference HF is one byte");
_Static_assert(sizeof(PROOF) == 34, "reference PROOF is 9 G1 + 7 HF = 34 bytes");

static G1 load_g1(const uint8_t *p) { G1 g; memcpy(&g, p, 3); return g; }
static void store_g1(uint8_t *p, G1 g) { memcpy(p, &g, 3); }

size_t ref_sizeof_g1(void) { return sizeof(G1); }
size_t ref_sizeof_proof(void) { return sizeof(PROOF); }

int ref_g1_is_on_curve(const uint8_t *a) { G1 g = load_g1(a); return g1_is_on_curve(&g); }

void ref_g1_add(const uint8_t *a, const uint8_t *b, uint8_t *out) {
  G1 x = load_g1(a), y = load_g1(b);
  store_g1(out, g1_add(&x, &y));
}

void ref_g1_double(const uint8_t *a, uint8_t *out) {
  G1 x = load_g1(a);
  store_g1(out, g1_double(&x));
}

void ref_g1_mul(const uint8_t *a, uint64_t k, uint8_t *out) {
  G1 x = load_g1(a);
  store_g1(out, g1_mul(&x, k));
}

/* MSM: the SRS is exactly n points, the polynomial exactly n coefficients (untrimmed). */
void ref_msm(const uint8_t *pts, const uint8_t *sc, size_t n, uint8_t *out) {
  SRS srs;
  memset(&srs, 0, sizeof srs);
  srs.g1s = (G1 *)pts;
  srs.len = n;
  POLY vs = {(HF *)sc, n};
  store_g1(out, srs_eval_at_s(&srs, &vs));
}

/* Returns the trimmed length; out must hold la+lb-1 bytes. */
size_t ref_poly_mul(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out) {
  POLY A = {(HF *)a, la}, B = {(HF *)b, lb};
  POLY r = poly_mul(&A, &B);
  memcpy(out, r.coeffs, r.len);
  size_t len = r.len;
  poly_free(&r);
  return len;
}

void ref_poly_divide(const uint8_t *num, size_t ln, const uint8_t *den, size_t ld,
                     uint8_t *q, size_t *lq, uint8_t *r, size_t *lr) {
  POLY N = {(HF *)num, ln}, D = {(HF *)den, ld}, Q, R;
  poly_divide(&N, &D, &Q, &R);
  memcpy(q, Q.coeffs, Q.len);
  memcpy(r, R.coeffs, R.len);
  *lq = Q.len;
  *lr = R.len;
  poly_free(&Q);
  poly_free(&R);
}

uint8_t ref_poly_eval(const uint8_t *p, size_t len, uint8_t x) {
  POLY P = {(HF *)p, len};
  HF X = {x};
  return poly_eval(&P, X).value;
}

void ref_matrix_mul(const uint8_t *a, size_t m, size_t k, const uint8_t *b, size_t n, uint8_t *out) {
  MATRIX A = matrix_new((HF *)a, m, k), B = matrix_new((HF *)b, k, n);
  MATRIX R = matrix_mul(&A, &B);
  memcpy(out, R.v, m * n);
  matrix_free(&A);
  matrix_free(&B);
  matrix_free(&R);
}

void ref_matrix_inv(const uint8_t *a, size_t n, uint8_t *out) {
  MATRIX A = matrix_new((HF *)a, n, n);
  MATRIX R = matrix_inv(&A);
  memcpy(out, R.v, n * n);
  matrix_free(&A);
  matrix_free(&R);
}

/* interpolate_at_h over the reference's 4-element H (plonk-test.c setup: secret 2, n 6). */
size_t ref_interpolate4(const uint8_t *values, uint8_t *out) {
  SRS srs = srs_create(f101(2), 6);
  PLONK plonk = plonk_new(srs, 4);
  POLY r = interpolate_at_h(&plonk, (const HF *)values, 4);
  memcpy(out, r.coeffs, r.len);
  size_t len = r.len;
  poly_free(&r);
  plonk_free(&plonk);
  return len;
}

/* The setup plonk_prove consumes (PLONK of plonk_new, SRS of srs_create; srs_mode as in
 * ref_prove4): h, k1_h, k2_h (4 each), h_pows_inv row-major (16), z_h_x (returns its len),
 * g1s (3 * (srs_n + 1) bytes). */
static SRS make_srs(uint8_t secret, size_t srs_n, int srs_mode) {
  SRS srs = srs_create(f101(secret), srs_n);
  if (srs_mode == 1) {
    G1 g = g1_generator();
    GF s = f101(secret), sp = s;
    for (size_t i = 0; i < srs.len; i++) {
      srs.g1s[i] = g1_mul(&g, sp.value);
      sp = gf_mul(sp, s);
    }
  }
  return srs;
}

size_t ref_plonk4_data(uint8_t secret, size_t srs_n, int srs_mode, uint8_t *h, uint8_t *k1,
                       uint8_t *k2, uint8_t *hinv, uint8_t *zh, uint8_t *g1s) {
  SRS srs = make_srs(secret, srs_n, srs_mode);
  memcpy(g1s, srs.g1s, 3 * srs.len);
  PLONK plonk = plonk_new(srs, 4);
  for (int i = 0; i < 4; i++) {
    h[i] = plonk.h[i].value;
    k1[i] = plonk.k1_h[i].value;
    k2[i] = plonk.k2_h[i].value;
    for (int c = 0; c < 4; c++) hinv[4 * i + c] = matrix_get(&plonk.h_pows_inv, i, c).value;
  }
  size_t zl = plonk.z_h_x.len;
  memcpy(zh, plonk.z_h_x.coeffs, zl);
  plonk_free(&plonk);
  return zl;
}

/*
 * One 4-gate prove through the reference plonk_prove, inside a forked child so that the
 * reference's assert()/exit() on an unsatisfiable instance cannot take the caller down.
 *   gates   : 5*4 bytes  q_m | q_l | q_r | q_o | q_c
 *   copies  : 3*4 (type, index) byte pairs = 24 bytes  c_a | c_b | c_c  (type 0=A 1=B 2=C)
 *   wires   : 3*4 bytes  a | b | c
 *   chal    : alpha beta gamma z v
 *   rnd     : 9 blinding scalars
 *   srs_mode: 0 = srs_create as is (all-identity G1s, src/srs.h:27-36)
 *             1 = same SRS length, g1s[i] overwritten with g1_mul(G, s^(i+1) mod 101)
 *                 so the commitments are not all the identity
 * Returns 0 and fills out[34] on success, -1 if the reference aborted/exited.
 */
static void prove4_body(const uint8_t *gates, const uint8_t *copies, const uint8_t *wires,
                        const uint8_t *chal, const uint8_t *rnd, uint8_t secret, size_t srs_n,
                        int srs_mode, uint8_t *buf) {
    {
    SRS srs = make_srs(secret, srs_n, srs_mode);
    PLONK plonk = plonk_new(srs, 4);
    CONSTRAINTS c;
    memset(&c, 0, sizeof c);
    c.num_constraints = 4;
    c.num_gates = 4;
    HF *q[5];
    for (int k = 0; k < 5; k++) {
      q[k] = malloc(4);
      memcpy(q[k], gates + 4 * k, 4);
    }
    c.q_m = q[0]; c.q_l = q[1]; c.q_r = q[2]; c.q_o = q[3]; c.q_c = q[4];
    COPY_OF *cp[3];
    for (int k = 0; k < 3; k++) {
      cp[k] = malloc(4 * sizeof(COPY_OF));
      for (int i = 0; i < 4; i++) {
        cp[k][i].type = (COPY_OF_TYPE)copies[8 * k + 2 * i];
        cp[k][i].index = copies[8 * k + 2 * i + 1];
      }
    }
    c.c_a = cp[0]; c.c_b = cp[1]; c.c_c = cp[2];
    ASSIGNMENTS as;
    as.len = 4;
    as.a = malloc(4); as.b = malloc(4); as.c = malloc(4);
    memcpy(as.a, wires, 4); memcpy(as.b, wires + 4, 4); memcpy(as.c, wires + 8, 4);
    CHALLENGE ch = {{chal[0]}, {chal[1]}, {chal[2]}, {chal[3]}, {chal[4]}};
    HF r9[9];
    memcpy(r9, rnd, 9);
    PROOF p = plonk_prove(&plonk, &c, &as, &ch, r9);
    memcpy(buf, &p, 34);
    for (int k = 0; k < 5; k++) free(q[k]);
    for (int k = 0; k < 3; k++) free(cp[k]);
    free(as.a); free(as.b); free(as.c);
    plonk_free(&plonk);
  }
}

/* in-process (no fork): for timing instances the reference accepts (bench.py's CPU baseline
 * of the toy circuit: srs_create + plonk_new + plonk_prove, as src/plonk-test.c does) */
void ref_prove4_inproc(const uint8_t *gates, const uint8_t *copies, const uint8_t *wires,
                       const uint8_t *chal, const uint8_t *rnd, uint8_t secret, size_t srs_n,
                       int srs_mode, uint8_t *out) {
  prove4_body(gates, copies, wires, chal, rnd, secret, srs_n, srs_mode, out);
}

int ref_prove4(const uint8_t *gates, const uint8_t *copies, const uint8_t *wires,
               const uint8_t *chal, const uint8_t *rnd, uint8_t secret, size_t srs_n,
               int srs_mode, uint8_t *out) {
#ifdef PLK_NO_FORK
  /* drop-in build (hot path on the GPU): a HIP context must not cross fork(), so the
   * prove runs in-process; only call it with instances the reference accepts. */
  prove4_body(gates, copies, wires, chal, rnd, secret, srs_n, srs_mode, out);
  return 0;
#else
  int fds[2];
  if (pipe(fds) != 0) return -1;
  pid_t pid = fork();
  if (pid < 0) return -1;
  if (pid == 0) {
    close(fds[0]);
    uint8_t buf[34];
    prove4_body(gates, copies, wires, chal, rnd, secret, srs_n, srs_mode, buf);
    ssize_t w = write(fds[1], buf, 34);
    _exit(w == 34 ? 0 : 3);
  }
  close(fds[1]);
  uint8_t buf[34];
  ssize_t got = 0;
  while (got < 34) {
    ssize_t k = read(fds[0], buf + got, 34 - got);
    if (k <= 0) break;
    got += k;
  }
  close(fds[0]);
  int status = 0;
  waitpid(pid, &status, 0);
  if (got != 34 || !WIFEXITED(status) || WEXITSTATUS(status) != 0) return -1;
  memcpy(out, buf, 34);
  return 0;
#endif
}
