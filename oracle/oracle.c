/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into, called by, or shipped with the
 * product path (plonk.c_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (oracle/liboracle.so via ctypes), and only as the checker.
 *
 * A from-scratch CPU restatement of the reference hot path of kazuakiishiguro/plonk.c,
 * operating on raw bytes with the reference's exact arithmetic (including its behaviour
 * on non-canonical bytes, so off-curve / garbage inputs fold the same way):
 *
 *   GF(101) add/sub/mul/neg/pow/inv ...... src/gf.h:24-33, 87-162
 *   G1 double / add / mul ................ src/g1.h:37-103
 *   MSM as a serial fold ................. src/srs.h:53-68   (srs_eval_at_s)
 *   poly_mul schoolbook + trailing trim .. src/poly.h:20-38, 106-122
 *   poly_divide / poly_eval .............. src/poly.h:124-177, 265-272
 *
 * plus two independent fast checkers used at sizes where the O(n^2) / serial forms are
 * too slow for a test:
 *   orc_msm_dlog      E(F101) is cyclic of order 102; a canonical on-curve input maps to
 *                     Z/102 by a discrete-log table and the MSM is an integer dot product
 *                     mod 102 (exact group isomorphism; cross-checked against the fold).
 *   orc_poly_mul_ntt  exact convolution by a CPU NTT over 998244353 (a different prime
 *                     from the GPU's BabyBear), reduced mod 17 and trimmed.
 * Parity of this restatement is pinned against golden vectors recorded from the compiled
 * reference (tests/golden/, made by tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define P_GF 101
#define P_HF 17

/* ---------------- GF(101) on raw bytes (src/gf.h) ---------------- */
static uint8_t f_new(int64_t v) { int64_t t = v % P_GF; if (t < 0) t += P_GF; return (uint8_t)t; }
static uint8_t f_add(uint8_t a, uint8_t b) { uint16_t s = (uint16_t)(a + b); if (s >= P_GF) s -= P_GF; return (uint8_t)s; }
static uint8_t f_sub(uint8_t a, uint8_t b) { int16_t d = (int16_t)a - (int16_t)b; if (d < 0) d += P_GF; return (uint8_t)d; }
static uint8_t f_mul(uint8_t a, uint8_t b) { return (uint8_t)(((uint16_t)a * (uint16_t)b) % P_GF); }
static uint8_t f_pow(uint8_t a, uint64_t e) {
  uint8_t r = 1, b = a;
  while (e) { if (e & 1) r = f_mul(r, b); e >>= 1; b = f_mul(b, b); }
  return r;
}
static uint8_t f_inv(uint8_t a) { return f_pow(a, P_GF - 2); }

/* ---------------- G1 (src/g1.h), 3 bytes {x, y, infinite} ---------------- */
typedef struct { uint8_t x, y, inf; } pt_t;

static pt_t pt_identity(void) { pt_t r = {0, 0, 1}; return r; }
static pt_t pt_make(uint8_t x, uint8_t y) { pt_t r = {f_new(x), f_new(y), 0}; return r; }

static pt_t pt_double(pt_t a) {
  if (a.inf || a.y == 0) return pt_identity();
  uint8_t m = f_mul(f_mul(3, f_mul(a.x, a.x)), f_inv(f_mul(2, a.y)));
  uint8_t m2 = f_mul(m, m);
  uint8_t xr = f_sub(m2, f_mul(2, a.x));
  uint8_t yr = f_sub(f_mul(m, f_sub(f_mul(3, a.x), m2)), a.y);
  return pt_make(xr, yr);
}

static pt_t pt_add(pt_t a, pt_t b) {
  if (a.inf) return b;
  if (b.inf) return a;
  if (a.x == b.x) {
    if (f_add(a.y, b.y) == 0) return pt_identity();
    return pt_double(a);
  }
  uint8_t m = f_mul(f_sub(b.y, a.y), f_inv(f_sub(b.x, a.x)));
  uint8_t xr = f_sub(f_sub(f_mul(m, m), a.x), b.x);
  uint8_t yr = f_sub(f_mul(m, f_sub(a.x, xr)), a.y);
  return pt_make(xr, yr);
}

static pt_t pt_mul(pt_t p, uint64_t k) {
  pt_t acc = pt_identity(), run = p;
  for (; k; k >>= 1) {
    if (k & 1) acc = pt_add(acc, run);
    run = pt_double(run);
  }
  return acc;
}

static pt_t ld(const uint8_t *p) { pt_t r = {p[0], p[1], p[2]}; return r; }
static void st(uint8_t *p, pt_t v) { p[0] = v.x; p[1] = v.y; p[2] = v.inf; }

void orc_g1_add(const uint8_t *a, const uint8_t *b, uint8_t *out) { st(out, pt_add(ld(a), ld(b))); }
void orc_g1_double(const uint8_t *a, uint8_t *out) { st(out, pt_double(ld(a))); }
void orc_g1_mul(const uint8_t *a, uint64_t k, uint8_t *out) { st(out, pt_mul(ld(a), k)); }
int orc_g1_is_on_curve(const uint8_t *a) {
  if (a[2]) return 1;
  return f_pow(a[1], 2) == f_add(f_pow(a[0], 3), 3);
}

/* srs_eval_at_s: left fold acc = acc + coeff_i * P_i, in index order (src/srs.h:58-65). */
void orc_msm_fold(const uint8_t *pts, const uint8_t *sc, size_t n, uint8_t *out) {
  pt_t acc = pt_identity();
  for (size_t i = 0; i < n; i++) acc = pt_add(acc, pt_mul(ld(pts + 3 * i), sc[i]));
  st(out, acc);
}

/* ---------------- discrete-log view of E(F101) (checker) ---------------- */
static int dl_ready;
static uint8_t dl_log[P_GF][P_GF]; /* 0xFF = not a point */
static pt_t dl_exp[102];
static pt_t dl_gen;

static int pt_order(pt_t p) {
  pt_t q = p;
  for (int k = 1; k <= 102; k++) {
    if (q.inf) return k;
    q = pt_add(q, p);
  }
  return -1;
}

static void dl_init(void) {
  if (dl_ready) return;
  /* generator: the first (x, then y) affine point of order 102 */
  int found = 0;
  for (int x = 0; x < P_GF && !found; x++)
    for (int y = 0; y < P_GF && !found; y++) {
      uint8_t b[3] = {(uint8_t)x, (uint8_t)y, 0};
      if (orc_g1_is_on_curve(b) && pt_order(ld(b)) == 102) { dl_gen = ld(b); found = 1; }
    }
  memset(dl_log, 0xFF, sizeof dl_log);
  pt_t q = pt_identity();
  for (int k = 0; k < 102; k++) {
    dl_exp[k] = q;
    if (!q.inf) dl_log[q.x][q.y] = (uint8_t)k;
    q = pt_add(q, dl_gen);
  }
  dl_ready = 1;
}

void orc_dlog_generator(uint8_t *out) { dl_init(); st(out, dl_gen); }

/* log of one point, -1 if the encoding is not canonical-on-curve */
int orc_dlog(const uint8_t *p) {
  dl_init();
  if (p[2] == 1) return (p[0] == 0 && p[1] == 0) ? 0 : -1;
  if (p[2] != 0 || p[0] >= P_GF || p[1] >= P_GF) return -1;
  uint8_t l = dl_log[p[0]][p[1]];
  return l == 0xFF ? -1 : l;
}

void orc_dlog_exp(int k, uint8_t *out) { dl_init(); st(out, dl_exp[((k % 102) + 102) % 102]); }

/* Sum c_i * log(P_i) mod 102; returns the log (0..101) or -1 if an input is irregular. */
int orc_msm_dlog(const uint8_t *pts, const uint8_t *sc, size_t n, uint8_t *out) {
  dl_init();
  uint64_t acc = 0;
  for (size_t i = 0; i < n; i++) {
    int l = orc_dlog(pts + 3 * i);
    if (l < 0) return -1;
    acc += (uint64_t)l * sc[i];
  }
  int r = (int)(acc % 102);
  if (out) st(out, dl_exp[r]);
  return r;
}

/* ---------------- polynomials over GF(17) (src/poly.h) ---------------- */
static size_t trim(const uint8_t *c, size_t len) {
  while (len > 1 && c[len - 1] == 0) len--;
  return len;
}

/* Schoolbook with the reference's per-step reductions; out holds la+lb-1 bytes. */
size_t orc_poly_mul(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out) {
  size_t rl = la + lb - 1;
  memset(out, 0, rl);
  for (size_t i = 0; i < la; i++) {
    for (size_t j = 0; j < lb; j++) {
      uint8_t prod = (uint8_t)(((uint16_t)a[i] * (uint16_t)b[j]) % P_HF);
      uint8_t s = (uint8_t)(out[i + j] + prod);
      if (s >= P_HF) s -= P_HF;
      out[i + j] = s;
    }
  }
  return trim(out, rl);
}

/* Independent exact checker: NTT over 998244353 (g = 3).  Valid while
 * min(la, lb) * 16 * 16 < 998244353 (inputs are first reduced mod 17). */
#define NP 998244353u
static uint32_t np_pow(uint64_t b, uint64_t e) {
  uint64_t r = 1; b %= NP;
  while (e) { if (e & 1) r = r * b % NP; b = b * b % NP; e >>= 1; }
  return (uint32_t)r;
}
static void np_ntt(uint32_t *a, size_t n, int inv) {
  for (size_t i = 1, j = 0; i < n; i++) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { uint32_t t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    uint64_t w = np_pow(3, (NP - 1) / len);
    if (inv) w = np_pow(w, NP - 2);
    for (size_t s = 0; s < n; s += len) {
      uint64_t t = 1;
      for (size_t k = 0; k < len / 2; k++) {
        uint32_t u = a[s + k];
        uint32_t v = (uint32_t)(a[s + k + len / 2] * t % NP);
        a[s + k] = u + v >= NP ? u + v - NP : u + v;
        a[s + k + len / 2] = u >= v ? u - v : u + NP - v;
        t = t * w % NP;
      }
    }
  }
  if (inv) {
    uint64_t ni = np_pow(n, NP - 2);
    for (size_t i = 0; i < n; i++) a[i] = (uint32_t)(a[i] * ni % NP);
  }
}

/* untrimmed product mod 17 into out[0, la + lb - 1) for la + lb - 1 <= 2^23 (998244353 =
 * 119 2^23 + 1: no larger power-of-two transform exists); 0 on allocation failure */
static int np_mul_raw(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out) {
  size_t rl = la + lb - 1, n = 1;
  while (n < rl) n <<= 1;
  uint32_t *fa = calloc(n, 4), *fb = calloc(n, 4);
  if (!fa || !fb) { free(fa); free(fb); return 0; }
  for (size_t i = 0; i < la; i++) fa[i] = a[i] % P_HF;
  for (size_t i = 0; i < lb; i++) fb[i] = b[i] % P_HF;
  np_ntt(fa, n, 0);
  np_ntt(fb, n, 0);
  for (size_t i = 0; i < n; i++) fa[i] = (uint32_t)((uint64_t)fa[i] * fb[i] % NP);
  np_ntt(fa, n, 1);
  for (size_t i = 0; i < rl; i++) out[i] = (uint8_t)(fa[i] % P_HF);
  free(fa);
  free(fb);
  return 1;
}

/* returns trimmed length, or 0 on allocation failure / size out of range.  Products longer
 * than 2^23 split the longer operand into chunks whose products fit 2^23 points and add the
 * shifted chunk products mod 17 (exact: each chunk product is). */
size_t orc_poly_mul_ntt_blocked(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out, size_t ms);

size_t orc_poly_mul_ntt(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out) {
  const size_t NMAX = (size_t)1 << 23;
  size_t rl = la + lb - 1;
  size_t mn = la < lb ? la : lb;
  if (mn * 256 >= NP) return orc_poly_mul_ntt_blocked(a, la, b, lb, out, (NP - 1) / 256);
  if (rl <= NMAX) return np_mul_raw(a, la, b, lb, out) ? trim(out, rl) : 0;
  if (la < lb) {   /* a := the longer operand */
    const uint8_t *t = a; a = b; b = t;
    size_t u = la; la = lb; lb = u;
  }
  const size_t h = NMAX - lb + 1;   /* chunk length: h + lb - 1 = 2^23 */
  uint8_t *part = malloc(NMAX);
  if (!part) return 0;
  memset(out, 0, rl);
  for (size_t s = 0; s < la; s += h) {
    const size_t cl = la - s < h ? la - s : h;
    if (!np_mul_raw(a + s, cl, b, lb, part)) { free(part); return 0; }
    for (size_t i = 0; i < cl + lb - 1; i++) out[s + i] = (uint8_t)((out[s + i] + part[i]) % P_HF);
  }
  free(part);
  return trim(out, rl);
}

/* Both operands too long for one exact product (min(la, lb) * 256 >= 998244353): the shorter
 * one in pieces of at most ms coefficients (ms * 256 < 998244353), each piece times the longer
 * operand by orc_poly_mul_ntt, the shifted piece products added mod 17 (exact: each is).  An
 * independent decomposition of the device's blocked products (other prime, other piece sizes);
 * small ms only to test the piece bookkeeping against the schoolbook. */
size_t orc_poly_mul_ntt_blocked(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out, size_t ms) {
  if (la == 0 || lb == 0 || ms == 0 || ms * 256 >= NP) return 0;
  if (la < lb) {   /* b := the shorter operand */
    const uint8_t *t = a; a = b; b = t;
    size_t u = la; la = lb; lb = u;
  }
  const size_t rl = la + lb - 1;
  uint8_t *part = malloc(la + ms);
  if (!part) return 0;
  memset(out, 0, rl);
  for (size_t s = 0; s < lb; s += ms) {
    const size_t bl = lb - s < ms ? lb - s : ms;
    memset(part, 0, la + bl - 1);
    if (!orc_poly_mul_ntt(a, la, b + s, bl, part)) { free(part); return 0; }
    for (size_t i = 0; i < la + bl - 1; i++) out[s + i] = (uint8_t)((out[s + i] + part[i]) % P_HF);
  }
  free(part);
  return trim(out, rl);
}

/* poly_divide (src/poly.h:124-177): long division with hf_inv by table (inv(0) = 0). */
static const uint8_t hf_inv_tab[17] = {0, 1, 9, 6, 13, 7, 3, 5, 15, 2, 12, 14, 10, 4, 11, 8, 16};
static uint8_t h_mul(uint8_t a, uint8_t b) { return (uint8_t)(((uint16_t)a * (uint16_t)b) % P_HF); }
static uint8_t h_sub(uint8_t a, uint8_t b) { int8_t d = (int8_t)a - (int8_t)b; if (d < 0) d += P_HF; return (uint8_t)d; }

int orc_poly_divide(const uint8_t *num, size_t ln, const uint8_t *den, size_t ld,
                    uint8_t *q, size_t *lq, uint8_t *r, size_t *lr) {
  int zero = 1;
  for (size_t i = 0; i < ld; i++) if (den[i]) zero = 0;
  if (zero) return -1;
  uint8_t *qq = calloc(ln ? ln : 1, 1), *rr = calloc(ln ? ln : 1, 1);
  memcpy(rr, num, ln);
  uint8_t li = hf_inv_tab[den[ld - 1] % P_HF];
  /* With a canonical numerator (every byte < 17) every value of the division stays canonical,
   * and then h_sub(x, h_mul(c, d)) == x whenever d = 0 mod 17: the divisor's zero coefficients
   * can be skipped (Z_H = x^n - 1 has two non-zero ones) -- the same bytes, O(q nnz) instead of
   * O(q ld).  A non-canonical byte is changed by h_sub(x, 0) (int8 arithmetic), so raw inputs
   * take the reference's full loop. */
  int canon = 1;
  for (size_t i = 0; i < ln && canon; i++) canon = num[i] < P_HF;
  long *nzj = NULL;
  long nnz = 0;
  if (canon) {
    nzj = malloc(ld * sizeof(long));
    if (nzj)
      for (long j = 0; j < (long)ld; j++)
        if (den[ld - 1 - j] % P_HF) nzj[nnz++] = j;
  }
  for (long i = (long)ln - 1; i >= (long)(ld - 1); i--) {
    uint8_t c = h_mul(rr[i], li);
    qq[i - (ld - 1)] = c;
    if (nzj) {
      for (long t = 0; t < nnz; t++) rr[i - nzj[t]] = h_sub(rr[i - nzj[t]], h_mul(c, den[ld - 1 - nzj[t]]));
    } else {
      for (long j = 0; j < (long)ld; j++) rr[i - j] = h_sub(rr[i - j], h_mul(c, den[ld - 1 - j]));
    }
  }
  free(nzj);
  size_t ql = ln >= ld ? ln - ld + 1 : 1;
  ql = trim(qq, ql);
  size_t rl = ld - 1;
  if (rl > ln) rl = ln;
  rl = trim(rr, rl);
  memcpy(q, qq, ql);
  memcpy(r, rr, rl);
  *lq = ql;
  *lr = rl;
  free(qq);
  free(rr);
  return 0;
}

uint8_t orc_poly_eval(const uint8_t *p, size_t len, uint8_t x) {
  uint8_t y = 0;
  for (long i = (long)len - 1; i >= 0; i--) {
    y = h_mul(y, x);
    uint8_t s = (uint8_t)(y + p[i]);
    if (s >= P_HF) s -= P_HF;
    y = s;
  }
  return y;
}

/* matrix_mul (src/matrix.h:79-96): row-major bytes, sum = hf_add(sum, hf_mul(a, b)) */
static uint8_t h_add(uint8_t a, uint8_t b) { uint8_t s = (uint8_t)(a + b); if (s >= P_HF) s -= P_HF; return s; }

void orc_matrix_mul(const uint8_t *a, size_t m, size_t k, const uint8_t *b, size_t n, uint8_t *out) {
  for (size_t i = 0; i < m; i++)
    for (size_t j = 0; j < n; j++) {
      uint8_t s = 0;
      for (size_t t = 0; t < k; t++) s = h_add(s, h_mul(a[i * k + t], b[t * n + j]));
      out[i * n + j] = s;
    }
}

/* matrix_inv (src/matrix.h:149-176): Gauss-Jordan on [M | I] (src/matrix.h:100-147) --
 * the first non-zero pivot at or below row r in column `lead` (moving right when a column is
 * all zero), row swap, normalisation by hf_div, elimination of every other row. */
void orc_matrix_inv(const uint8_t *a, size_t n, uint8_t *out) {
  const size_t c = 2 * n;
  uint8_t *g = calloc(n * c + 1, 1);
  for (size_t i = 0; i < n; i++) {
    memcpy(g + i * c, a + i * n, n);
    g[i * c + n + i] = 1;
  }
  size_t lead = 0;
  for (size_t r = 0; r < n; r++) {
    if (c <= lead) break;
    size_t i = r;
    int stop = 0;
    while (g[i * c + lead] == 0) {
      if (++i == n) {
        i = r;
        if (++lead == c) { stop = 1; break; }
      }
    }
    if (stop) break;
    if (i != r)
      for (size_t k = 0; k < c; k++) { uint8_t t = g[i * c + k]; g[i * c + k] = g[r * c + k]; g[r * c + k] = t; }
    const uint8_t div = g[r * c + lead];
    if (div) for (size_t k = 0; k < c; k++) g[r * c + k] = h_mul(g[r * c + k], hf_inv_tab[div % P_HF]);
    for (size_t ii = 0; ii < n; ii++) {
      if (ii == r) continue;
      const uint8_t mult = g[ii * c + lead];
      for (size_t k = 0; k < c; k++) g[ii * c + k] = h_sub(g[ii * c + k], h_mul(g[r * c + k], mult));
    }
    lead++;
  }
  for (size_t i = 0; i < n; i++) memcpy(out + i * n, g + i * c + n, n);
  free(g);
}

/* ---------------- seeded generators shared with SURVEY.md §8c ---------------- */
static uint64_t xs_next(uint64_t *s) {
  uint64_t x = *s;
  x ^= x << 13; x ^= x >> 7; x ^= x << 17;
  *s = x;
  return x;
}

/* SURVEY §8c MSM generator: xorshift64 seeded 0x9E3779B97F4A7C15; N draws -> points kG,
 * k = 1 + r%16; N draws -> scalars r%17; one more draw -> c[N-1] = 1 + r%16. */
void orc_gen_survey_msm(size_t n, uint8_t *pts, uint8_t *sc) {
  uint64_t s = 0x9E3779B97F4A7C15ull;
  pt_t g = {1, 2, 0}, kg[17];
  for (int k = 0; k < 17; k++) kg[k] = pt_mul(g, (uint64_t)k);
  for (size_t i = 0; i < n; i++) st(pts + 3 * i, kg[1 + xs_next(&s) % 16]);
  for (size_t i = 0; i < n; i++) sc[i] = (uint8_t)(xs_next(&s) % 17);
  if (n) sc[n - 1] = (uint8_t)(1 + xs_next(&s) % 16);
}

/* SURVEY §8c poly_mul generator: xorshift64 seeded 0x243F6A8885A308D3; per i draw a_i
 * then b_i (r%17); a[N-1] = b[N-1] = 1. */
void orc_gen_survey_poly(size_t n, uint8_t *a, uint8_t *b) {
  uint64_t s = 0x243F6A8885A308D3ull;
  for (size_t i = 0; i < n; i++) {
    a[i] = (uint8_t)(xs_next(&s) % 17);
    b[i] = (uint8_t)(xs_next(&s) % 17);
  }
  if (n) { a[n - 1] = 1; b[n - 1] = 1; }
}

/* h = h*31 + c (uint32), h0 = 0 */
uint32_t orc_digest31(const uint8_t *c, size_t len) {
  uint32_t h = 0;
  for (size_t i = 0; i < len; i++) h = h * 31u + c[i];
  return h;
}
