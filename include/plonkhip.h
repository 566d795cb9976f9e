/*
 * libplonkhip -- the C ABI between the reference's host code and the gfx950 kernels.
 *
 * The reference (kazuakiishiguro/plonk.c) has no plugin/FFI layer: plonk.h calls
 * srs_eval_at_s() and poly_mul() by name after #include "srs.h" / "poly.h"
 * (src/plonk.h:8-9).  The drop-in headers in this directory keep those exact signatures and
 * route the two hot functions through the entry points below; any other host language
 * binds the same symbols (see INTEGRATION.md for the ctypes / cgo stubs).
 *
 * Conventions
 *   - plain pointers and sizes only; a G1 is 3 bytes {x, y, infinite} exactly as the
 *     reference struct (src/g1.h:8-11), an HF is 1 byte (src/hf.h:15-17);
 *   - host-buffer entry points are synchronous: results are complete on return and no
 *     caller pointer is retained;
 *   - *_dev entry points take DEVICE pointers and a hipStream_t (as void*; NULL = the HIP
 *     null stream) and are asynchronous;
 *   - every entry point returns PLK_OK (0) or a PLK_ERR_* code; plk_last_error() gives text.
 *     The drop-in headers turn a non-zero code into the reference's convention
 *     (fprintf(stderr, ...) + exit(EXIT_FAILURE), e.g. src/srs.h:54-57);
 *   - there is no CPU fallback: without a usable GPU every compute entry point fails
 *     with PLK_ERR_NODEV.  (The drop-in HEADERS keep calls of toy size on the host by their own
 *     restated code, include/plk_host.h -- SURVEY 8(b)'s small-size policy, sized by
 *     PLK_OPT_DROPIN_HOST_WORK; the library itself never computes on the CPU.)
 */
#ifndef PLONKHIP_H
#define PLONKHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  PLK_OK = 0,
  PLK_ERR_HIP = 1,    /* a HIP runtime call failed */
  PLK_ERR_ARG = 2,    /* bad argument (NULL pointer, empty polynomial, ...) */
  PLK_ERR_RANGE = 3,  /* size outside what the exact algorithm supports */
  PLK_ERR_NODEV = 4,  /* no usable GPU */
  PLK_ERR_NOMEM = 5   /* device allocation failed */
};

/* ---- lifetime ------------------------------------------------------------------------ */
int plk_init(int device);            /* select device (<0: $PLK_DEVICE or 0); idempotent */
/* Several GPUs in one process (SURVEY 8(b) plk_init(n_gpus), 8(e)): ids[0] is the primary
 * device (everything runs there as after plk_init(ids[0])); plk_msm_g1 -- srs_eval_at_s, the
 * reference's commitment -- splits an MSM of at least PLK_OPT_MSM_SHARD_MIN points into n
 * contiguous point ranges, one per entry, each uploaded over its own device's link from its own
 * host thread and reduced to a partial discrete log there; the N 4-byte partials are summed
 * on the host (the result returns to the host anyway).  Ids may repeat (several shards on one
 * GPU).  Calling again replaces the list; n = 1 goes back to one device.  PLK_DEVICE="0,1,2,3"
 * does the same at implicit initialisation.  1 <= n <= 16. */
int plk_init_devices(const int *ids, int n);
int plk_devices(int *ids, int cap);  /* the shard list (or the one device); returns its length */
void plk_shutdown(void);
const char *plk_last_error(void);
int plk_device_count(void);
const char *plk_version(void);

/* ---- options --------------------------------------------------------------------------
 * Every default is the production setting; the others exist for A/B measurement and for tests
 * that force a rarely taken path.  None changes a result: every setting gives the same bytes.
 * The library reads no environment variable except PLK_DEVICE (device selection).  Options
 * marked [init] shape tables built by plk_init and may only be set before it (PLK_ERR_ARG
 * after). */
enum {
  PLK_OPT_TINY_CALLS = 1,        /* 1: toy-size host calls through mapped pinned memory; 0: staged copies */
  PLK_OPT_PROVE_SYNC = 2,        /* 0: a proof's end is seen by polling its completion word; 1: stream sync */
  PLK_OPT_POLY_BLOCK_L = 3,      /* blocked poly_mul piece lengths; 0 = the exact-range maxima       */
  PLK_OPT_POLY_BLOCK_S = 4,      /*   (both set: forces the blocked path with those pieces, >= 33)   */
  PLK_OPT_NTT_F29 = 5,           /* 1: poly_mul over F29 where exact; 0: BabyBear only                */
  PLK_OPT_NTT_SHARE = 6,         /* 1: an operand given twice in one batch is transformed once        */
  PLK_OPT_NTT_SHARED_FIX = 7,    /* 1: shared operands' lo = 0 pass in its own launch (auto), 0 off, 2 forced */
  PLK_OPT_NTT_T13_MIN_K = 8,     /* [init] 21: 2^13-element tiles from 2^k points up (13..27)        */
  PLK_OPT_NTT_CENTER_BLOCKS = 9, /* 0: resident blocks of the center kernel from the CU count        */
  PLK_OPT_MSM_THREADS = 10,      /* MSM launch geometry overrides (0 = the built-in choice):          */
  PLK_OPT_MSM_MAX_BLOCKS = 11,   /*   threads 256/512/1024, resident blocks, groups in flight 1/2/4, */
  PLK_OPT_MSM_GROUPS = 12,       /*   table copies 1/8, half groups for single MSMs (1 = on)          */
  PLK_OPT_MSM_COPIES = 13,
  PLK_OPT_MSM_HALF = 14,
  PLK_OPT_MSM_SHARD_MIN = 15,    /* multi-device plk_msm_g1: split from this many points (2^16)      */
  PLK_OPT_NTT_CENTER_SUM = 16,   /* 1: a sum group's products added in its leader's center item      */
  PLK_OPT_MSM_HOST_LANES = 17,   /* one device: plk_msm_g1 of >= MSM_SHARD_MIN points runs its SRS memcmp,
                                    staging and uploads on this many host threads (1: one); read by
                                    plk_init / plk_init_devices */
  PLK_OPT_PROVE_DERIVE_T2A = 18, /* 1: round 3's A2 B2 from a_x b_x by an elementwise pass (0: its own product;
                                    2, the default: that pass inside the t_2 product's first forward pass when
                                    it runs on 2^13 tiles -- one launch fewer -- else as 1) */
  PLK_OPT_NTT_TABLE_SHARE = 19,  /* 1: a table pass runs several arrays of one tile per block (column words read once) */
  PLK_OPT_NTT_LAUNCH_LOG = 20,   /* diagnostics: 1 records the NTT passes' launch plans (plk_ntt_launch_log) */
  PLK_OPT_PROVE_FUSE_DIV = 21,   /* 1: round 5's numerators and their divisions by x - z, x - z omega in one
                                    launch (single-pass suffix scan); 0: numerators, then the apply launch */
  PLK_OPT_PROVE_SRS_LOGS = 22,   /* 1: the prover's commitments read its SRS in log form (1 B per point,
                                    converted once at plk_prover_create); 0: the G1 form (3 B) */
  PLK_OPT_PROVE_PACK_FUSE = 23,  /* 1 (with PROVE_SRS_LOGS): commitments, trimmed lengths and the proof packing
                                    in one launch (commit_pack_kernel); 0: the MSM, then trim_pack_kernel */
  PLK_OPT_PROVE_EARLY_COMMITS = 24, /* 1 (with PROVE_PACK_FUSE): the 7 commitments that do not wait for round 5
                                       run as extra rows of round 5's scan launch; 2: of round 4's evaluation
                                       launch */
  PLK_OPT_PROVE_HELPER_COPY = 25, /* 1: helpers of plk_prover_attach_helpers on the proving device itself take
                                     the distinct-device input path (their inputs copied into their own rows,
                                     the rest pointed at a poison row): a one-GPU test of that branch */
  PLK_OPT_PROVE_EVAL_AGG = 26,   /* 1: round 4's evaluation rows also store round 5's scan-chunk aggregates, so
                                    both round-5 divisions finish in ONE launch (lincomb_agg_divide_kernel);
                                    0: the numerators + aggregates launch, then the apply launch */
  PLK_OPT_PROVE_GRAPH = 27,      /* 1: plk_prover_rounds_dev replays its launches as a HIP graph captured on the
                                    first call with the same input addresses, preprocessed state and options
                                    (per call only the scalar file and the completion word are set; a call
                                    the graph cannot serve runs direct launches) -- measured equal, off */
  PLK_OPT_DROPIN_HOST_WORK = 28, /* drop-in headers (include/plk_host.h): a call whose host cost estimate (about
                                    ns: la*lb MACs for poly_mul, 300 per MSM point, ...) is at most this stays
                                    on the host; 32768 ~ one GPU round trip; 0: every call on the GPU.  The
                                    library reads it only through plk_get_option */
  PLK_OPT_COUNT = 29
};
int plk_set_option(int opt, int64_t value);   /* PLK_ERR_ARG: unknown option or value out of range */
/* Diagnostics for the roofline tools: with PLK_OPT_NTT_LAUNCH_LOG = 1 every NTT pass launch
 * is recorded as 8 ints {kind (0 forward, 1 inverse, 2 center, 3 shared lo = 0 pass), tile bits,
 * pass bits, log2 size, arrays / products, arrays per block, center pass units, field (0 F29,
 * 1 BabyBear)}; this copies up to cap records into out (8 ints each), clears the log and returns
 * the count. */
int plk_ntt_launch_log(int32_t *out, int cap);
int64_t plk_get_option(int opt);              /* -1 for an unknown option */

/* ---- host-buffer entry points (what the drop-in headers call) ------------------------ */

/* Replaces the body of srs_eval_at_s (src/srs.h:53-68):
 *   out = sum_{i<n} g1_mul(points[i], scalars[i]) folded left with g1_add.
 * points: n x 3 bytes, scalars: n bytes (HF.value, any byte value), out: 3 bytes.
 * The caller keeps the reference's degree check (vs->len > srs->len) before calling. */
int plk_msm_g1(const uint8_t *points, const uint8_t *scalars, size_t n, uint8_t out[3]);

/* Replaces the body of poly_mul (src/poly.h:106-122):
 *   out[0 .. la+lb-1) = a * b over GF(17); *out_len = length after the reference's
 *   trailing-zero trim (src/poly.h:20-38), >= 1.  out must hold la+lb-1 bytes.
 *   la == 0 or lb == 0 mirrors the reference: *out_len = (la+lb-1 > 0), out[0] = 0.
 *   Any shape with la + lb - 1 < 2^32: products beyond one transform's exact range
 *   (min(la, lb) >= 7,864,320 or more than 2^27 output coefficients) run as in-range piece
 *   products accumulated mod 17 (the _dev form then needs plk_poly_mul_workspace bytes). */
int plk_poly_mul(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, uint8_t *out,
                 size_t *out_len);

/* ---- device-resident entry points (bench, multi-GPU, pipelines) ---------------------- */

/* Result record of one MSM, 2176 bytes of device memory.  Zero it once
 * (plk_msm_result_init); every launch leaves its internal words at zero again, so a record
 * can be reused by the next launch on the same stream.  The arrival words of the blocks of
 * one launch live on separate 128-byte lines (serialised device-scope atomics on one line
 * cost ~10 ns each: ~3 us for 256 blocks on a single word). */
typedef struct {
  uint64_t top;        /* internal: arrival word over the shards */
  uint32_t log;        /* discrete log of the result w.r.t. plk_dlog_generator(), 0..101 */
  uint32_t irregular;  /* > 0: some input was not a canonical group element -> g1 invalid,
                          run plk_msm_g1_serial_dev for the reference's exact raw fold */
  uint8_t g1[4];       /* {x, y, infinite, 0} */
  uint32_t pad[27];
  uint64_t shard[16][16]; /* internal: arrival words shard[s][0] (two per XCD): [31:0] sum,
                             [47:32] ticket, [63:48] bad; one 128-byte line each */
} plk_msm_result_t;

int plk_msm_result_init(plk_msm_result_t *d_res, void *stream);
int plk_msm_g1_dev(const uint8_t *d_points, const uint8_t *d_scalars, size_t n,
                   plk_msm_result_t *d_res, void *stream);
/* A batch of independent MSMs of n points each in ONE launch: MSM b reads
 * d_points + b * points_stride and d_scalars + b * scalars_stride and writes d_res[b].
 * (E.g. the commitments of one prover round, or many proofs' commitments at once.) */
int plk_msm_g1_batch_dev(const uint8_t *d_points, size_t points_stride, const uint8_t *d_scalars,
                         size_t scalars_stride, size_t n, int batch, plk_msm_result_t *d_res,
                         void *stream);
int plk_msm_g1_serial_dev(const uint8_t *d_points, const uint8_t *d_scalars, size_t n,
                          plk_msm_result_t *d_res, void *stream);
/* out3 = EXP[(sum of count partial logs) mod 102] -- combines per-shard partials after a
 * collective sum (multi-GPU point-range sharding). */
int plk_msm_combine_dev(const uint32_t *d_logs, int count, uint8_t *d_out3, void *stream);
/* batch of already-summed logs (element i at d_logs[i * stride]) -> d_out4[4 i ..] =
 * {x, y, infinite, 0} of EXP[log mod 102]; one launch for a whole batch of MSMs. */
int plk_msm_finalize_dev(const uint32_t *d_logs, int batch, int stride, uint8_t *d_out4,
                         void *stream);
/* the order-102 generator the logs refer to (the first affine point of order 102 in (x, y)
 * order) */
int plk_dlog_generator(uint8_t out[3]);

/* poly_mul on device buffers: d_out holds la+lb-1 bytes (not overlapping d_a / d_b); *d_out_nz
 * receives the trimmed length (0 = the zero polynomial, i.e. length 1).  d_work:
 * plk_poly_mul_workspace() bytes. */
size_t plk_poly_mul_workspace(size_t la, size_t lb);
int plk_poly_mul_dev(const uint8_t *d_a, size_t la, const uint8_t *d_b, size_t lb, uint8_t *d_out,
                     uint32_t *d_out_nz, void *d_work, void *stream);

/* A batch of independent poly_mul products on device buffers (the prover's round-3 products
 * run this way; replaces a sequence of poly_mul calls, src/poly.h:106-122): products of one
 * transform size share each pass's launch, and operands given by the same pointer and length
 * are transformed once.  acc = 1 ADDS the product into the preceding job's output (a sum group:
 * a leader and up to two members of its transform size, none with a longer product than the
 * leader's; the members' out is not written; the whole sum must fit the transform's exact
 * range, else PLK_ERR_RANGE).  Outputs are
 * untrimmed (la + lb - 1 bytes) and must not overlap any job's inputs (the last pass still reads
 * input bytes for the top coefficients of wrapped products).  d_work: at least the largest single
 * job's plk_poly_mul_workspace() (a sum group of g products: g times its member's); products run
 * in launches of up to 12, cut between sum groups; plk_poly_mul_batch_workspace() bytes run every
 * size group at full width. */
typedef struct {
  const uint8_t *a;
  size_t la;
  const uint8_t *b;
  size_t lb;
  uint8_t *out;
  int acc;
} plk_polymul_job_t;
size_t plk_poly_mul_batch_workspace(const plk_polymul_job_t *jobs, int n);
int plk_poly_mul_batch_dev(const plk_polymul_job_t *jobs, int n, void *d_work, size_t work_bytes, void *stream);

/* Radix-2 NTT over BabyBear p = 15*2^27+1 on 2^log_n Montgomery-form u32, in place:
 * forward = DIF natural -> bit-reversed; inverse = DIT bit-reversed -> natural, unscaled. */
int plk_ntt_dev(uint32_t *d_data, int log_n, int inverse, void *stream);
/* batch independent transforms of 2^log_n points, array b at d_data + b 2^log_n; the arrays
 * share each pass's launch (the prover's products run the same way). */
int plk_ntt_batch_dev(uint32_t *d_data, int log_n, int batch, int inverse, void *stream);
/* The same over F29 p = 7*2^26+1 -- the field poly_mul and the device prover transform in
 * (lazy reduction inside, ~7 integer VALU per butterfly against ~10 for BabyBear): Montgomery
 * form (R = 2^32) u32 < p in, fully reduced out, root of order 2^log_n = 3^((p-1)/2^log_n);
 * log_n 13..26. */
int plk_ntt29_dev(uint32_t *d_data, int log_n, int inverse, void *stream);
int plk_ntt29_batch_dev(uint32_t *d_data, int log_n, int batch, int inverse, void *stream);

/* ---- the ops around the hot path ---------------------------------
 * Byte-exact restatements of the reference's host ops on the GPU, for every byte value
 * (non-canonical HF bytes included: the kernels fall back to the reference's serial loop on the
 * device where the parallel form would differ).  The drop-in headers call them. */

/* Replaces poly_eval (src/poly.h:265-272): Horner at x, *y = the reference's HF byte. */
int plk_poly_eval(const uint8_t *p, size_t len, uint8_t x, uint8_t *y);
/* n evaluations in one launch (the prover's ~40 evaluations, src/plonk.h:345-347, 527-533,
 * 567, 574; the grand-product loop src/plonk.h:326-359): ys[i] = poly_eval(polys[i], xs[i]). */
int plk_poly_eval_batch(const uint8_t *const *polys, const size_t *lens, const uint8_t *xs, int n,
                        uint8_t *ys);
/* device form: d_polys = host array of n device pointers; d_tick = plk_poly_eval_workspace(n)
 * bytes of device memory, zeroed once (every launch leaves it zeroed again). */
size_t plk_poly_eval_workspace(int n);
int plk_poly_eval_batch_dev(const uint8_t *const *d_polys, const size_t *lens, const uint8_t *xs, int n,
                            uint8_t *d_ys, void *d_tick, void *stream);

/* Replaces poly_divide (src/poly.h:124-177): num = quot * den + rem.
 *   quot: max(nl - dl + 1, 1) bytes, rem: min(dl - 1, nl) bytes (may be NULL when that is 0);
 *   *quot_len / *rem_len = lengths after the reference's trim (rem_len 0 when dl == 1).
 * Divisors x^m * lead + d0 (Z_H = x^n - 1, x - z, constants) run as parallel chain scans; any
 * other divisor, and non-canonical numerator bytes, run the reference's loop on the device.
 * A zero divisor is PLK_ERR_ARG ("Division by zero polynomial in poly_divide"); a divisor lead
 * byte >= 17 is PLK_ERR_RANGE (the reference reads hf_inverses out of bounds). */
int plk_poly_divide(const uint8_t *num, size_t nl, const uint8_t *den, size_t dl, uint8_t *quot, size_t *quot_len,
                    uint8_t *rem, size_t *rem_len);
/* device form: den stays a HOST array (classified on the host, copied into d_work when the
 * serial loop needs it); d_lens[0..1] receive the index + 1 of the last non-zero quotient /
 * remainder byte (0: all zero) over the untrimmed lengths above; d_work:
 * plk_poly_divide_workspace(nl, dl) bytes. */
size_t plk_poly_divide_workspace(size_t nl, size_t dl);
int plk_poly_divide_dev(const uint8_t *d_num, size_t nl, const uint8_t *den, size_t dl, uint8_t *d_quot,
                        uint8_t *d_rem, uint32_t *d_lens, void *d_work, void *stream);

/* Replaces matrix_mul (src/matrix.h:79-96): out[m x n] = a[m x k] b[k x n], row-major bytes,
 * sums by hf_add of hf_mul products. */
int plk_matrix_mul(const uint8_t *a, size_t m, size_t k, const uint8_t *b, size_t n, uint8_t *out);
/* Replaces matrix_inv (src/matrix.h:149-176, Gauss-Jordan src/matrix.h:100-147) as plonk_new
 * uses it for the Vandermonde inverse h_pows_inv (src/plonk.h:105-113): the same pivoting, so
 * the same bytes for singular matrices too.  Entries must be GF(17) values (< 17). */
int plk_matrix_inv(const uint8_t *mat, size_t n, uint8_t *out);
/* interpolate_at_h (src/plonk.h:162-195): out = h_pows_inv (n x n) * values, trimmed as
 * poly_new; out holds n bytes. */
int plk_interpolate(const uint8_t *h_pows_inv, const uint8_t *values, size_t n, uint8_t *out, size_t *out_len);

/* ---- device-resident prover (replaces plonk_new / plonk_prove / plonk_free,
 * src/plonk.h:53-139, 223-656, 120-139) ---------------------------------------------------
 * plk_prover_create uploads the SRS and Z_H once (the PLONK struct of plonk_new); the
 * circuit tables h, k1_h, k2_h, h_pows_inv are optional (needed only by plk_prover_prove).
 * h_pows_inv is the inverse Vandermonde matrix row-major, [r * n + c] = matrix_get(r, c).
 * A prover owns its stream and work buffers: one call at a time per plk_prover_t (distinct
 * provers may run from different threads). */
typedef struct plk_prover plk_prover_t;
typedef struct {
  size_t n;                                  /* gates = |H| */
  const uint8_t *h, *k1_h, *k2_h;            /* n each (HF values), or NULL */
  const uint8_t *h_pows_inv;                 /* n * n, or NULL */
  const uint8_t *z_h;                        /* Z_H(x) coefficients (plonk.z_h_x) */
  size_t z_h_len;
  const uint8_t *srs_g1;                     /* srs.g1s, 3 bytes per G1 */
  size_t srs_len;
} plk_plonk_desc_t;
/* CONSTRAINTS + ASSIGNMENTS (src/constraints.h:11-60); copies are (type, index) byte pairs,
 * type 0 = COPYOF_A, 1 = COPYOF_B, 2 = COPYOF_C, index 1-based (n <= 16 in GF(17)) */
typedef struct {
  const uint8_t *q_m, *q_l, *q_r, *q_o, *q_c;
  const uint8_t *copy_a, *copy_b, *copy_c;   /* 2n bytes each */
  const uint8_t *a, *b, *c;
} plk_circuit_t;
#define PLK_PROVE_STRICT 1                   /* enforce the zero-remainder asserts */
int plk_prover_create(const plk_plonk_desc_t *desc, plk_prover_t **out);
void plk_prover_destroy(plk_prover_t *p);
size_t plk_prover_device_bytes(const plk_prover_t *p);
/* plonk_prove: chal = {alpha, beta, gamma, z, v}; proof = the 34-byte PROOF struct.  Errors
 * where the reference exits or asserts (unsatisfied gate, bad copy, SRS too short, non-zero
 * remainder, t(x) too short to slice) return PLK_ERR_ARG / PLK_ERR_RANGE. */
int plk_prover_prove(plk_prover_t *p, const plk_circuit_t *circuit, const uint8_t chal[5],
                     const uint8_t rand9[9], uint8_t proof[34]);
/* rounds 1-5 of plonk_prove from device-resident interpolated polynomials (each zero padded
 * to n bytes): f_a f_b f_c q_o q_m q_l q_r q_c s_sigma_1 s_sigma_2 s_sigma_3 acc_x l_1_x.
 * Without PLK_PROVE_STRICT non-zero remainders are tolerated (synthetic inputs). */
int plk_prover_rounds_dev(plk_prover_t *p, const uint8_t *const d_polys[13], const uint8_t chal[5],
                          const uint8_t rand9[9], int flags, uint8_t proof[34]);
/* Preprocessed circuit (PLONK's preprocessed input; the reference re-derives it inside every
 * plonk_prove, src/plonk.h:386-503): the forward transforms round 3 needs of the fixed circuit
 * polynomials q_o q_m q_l q_r s_sigma_3 l_1_x (d_polys indices 3 4 5 6 10 12, device-resident,
 * zero padded to n) are computed once here.  plk_prover_rounds_dev with PLK_PROVE_PREPROCESSED
 * then uses them for the entries whose address equals the one given here; the bytes at those
 * addresses must not change while they are in use (call again after a change; d_polys = NULL
 * drops them).  Proof bytes are identical with and without. */
#define PLK_PROVE_PREPROCESSED 2
int plk_prover_preprocess(plk_prover_t *p, const uint8_t *const d_polys[13]);
/* Measurement of one proof (bench.py's C5 roofline; no reference counterpart).
 * plk_prover_profile_dev = plk_prover_rounds_dev (same bytes) with hipEvents on the prover's stream
 * around its whole launch sequence and around each of round 3's two product batches -- every NTT
 * pass kernel of the proof; ms = {launch sequence, both batches, batch 1, batch 2} in milliseconds
 * (one prover, no helpers).
 * plk_prover_launches: the kernel launches (and other graph nodes: copies, memsets) of one such
 * call, counted by capturing it as a HIP graph that is never launched (nothing runs, no state
 * changes).
 * plk_prover_alg_bytes: rounds 1-5's algorithmic bytes in SURVEY 8(d) terms over the reference's own
 * ops (src/plonk.h:277-621): 17 poly_mul at la + lb + (la + lb - 1), 9 srs_eval_at_s at 4 B per point,
 * 3 poly_divide (operands read, quotient and remainder written), 9 poly_eval (one read each). */
int plk_prover_profile_dev(plk_prover_t *p, const uint8_t *const d_polys[13], const uint8_t chal[5],
                           const uint8_t rand9[9], int flags, uint8_t proof[34], double ms[4]);
int plk_prover_launches(plk_prover_t *p, const uint8_t *const d_polys[13], const uint8_t chal[5],
                        const uint8_t rand9[9], int flags, int *kernels, int *other_nodes);
uint64_t plk_prover_alg_bytes(const plk_prover_t *p);

/* Strong-scaled proof over several GPUs (round 3's independent poly_mul jobs spread
 * across GPUs as whole jobs).  Two of round 3's product chains depend only on the proof's inputs:
 *   PLK_CHAIN_T2: t_2 = (A2 B2)(C2 z_x)            (src/plonk.h:432-434, re-associated)
 *   PLK_CHAIN_T3: t_3 = (A3 B3)(C3 z_x(omega x))   (src/plonk.h:471-473)
 * A helper GPU computes them from the same inputs as the proving GPU with plk_prover_chains_dev;
 * their bytes travel to the proving GPU (e.g. an RCCL send / receive), whose
 * plk_prover_rounds_ext_dev skips those chains and reads the bytes instead.  The proof bytes are
 * identical to plk_prover_rounds_dev's.  Buffers: plk_prover_chain_bytes(p, chain) bytes each,
 * 16-byte aligned, device memory of the prover's GPU. */
#define PLK_CHAIN_T2 1
#define PLK_CHAIN_T3 2
size_t plk_prover_chain_bytes(const plk_prover_t *p, int chain);
/* Enqueue rounds 1-3's preparation and the chains in `which` on the prover's stream, products
 * into d_t2 / d_t3; the stream `done` (NULL: the null stream) waits for them.  Returns without
 * waiting. */
int plk_prover_chains_dev(plk_prover_t *p, const uint8_t *const d_polys[13], const uint8_t chal[5],
                          const uint8_t rand9[9], int which, uint8_t *d_t2, uint8_t *d_t3, void *done);
/* plk_prover_rounds_dev with the chains in `which` read from d_t2 / d_t3, after everything
 * enqueued on stream `ready` (NULL: the null stream) at the time of the call -- e.g. their
 * receive. */
int plk_prover_rounds_ext_dev(plk_prover_t *p, const uint8_t *const d_polys[13], const uint8_t chal[5],
                              const uint8_t rand9[9], int flags, int which, const uint8_t *d_t2,
                              const uint8_t *d_t3, void *ready, uint8_t proof[34]);

/* The same split driven from C in one process, over the plk_init_devices list (no RCCL, no
 * caller-side hand-off): plk_prover_attach_helpers(p, k) creates k helper provers on list entries
 * 1..k (k = 1: t_3 on ids[1]; k = 2: t_2 on ids[1] and t_3 on ids[2]; 0 detaches; call from p's
 * device).  Afterwards plk_prover_rounds_dev and plk_prover_prove run every proof split: p's
 * stream records an event after the work already enqueued on it (the inputs); each helper's stream
 * waits for it, copies the 7 polynomials its chains read (f_a f_b f_c s_sigma_1..3 acc_x) to its
 * own GPU when that is another device (hipMemcpyPeerAsync), runs the chains, copies their products
 * into receive buffers on p's GPU (hipMemcpyPeerAsync on the helper's stream) and records an event;
 * p's stream waits for those events only before its numerator.  Ids may repeat (the one-GPU
 * rehearsal: helpers on their own streams of the same device).  Same proof bytes.
 * plk_prover_rounds_multi_dev takes the inputs already resident on every device: d_polys holds
 * ndev = 1 + k sets of 13 pointers, set 0 on p's device, set h on helper h's (no input copies). */
int plk_prover_attach_helpers(plk_prover_t *p, int k);
int plk_prover_helpers(const plk_prover_t *p);   /* the k attached (0: none) */
int plk_prover_rounds_multi_dev(plk_prover_t *p, const uint8_t *const *d_polys, int ndev, const uint8_t chal[5],
                                const uint8_t rand9[9], int flags, uint8_t proof[34]);

#ifdef __cplusplus
}
#endif
#endif /* PLONKHIP_H */
