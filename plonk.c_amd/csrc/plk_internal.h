// Internal declarations shared by the .hip translation units of libplonkhip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/plonkhip.h"

typedef plk_msm_result_t PlkMsmResult;
static_assert(sizeof(plk_msm_result_t) == 2176, "MSM result record is 2176 bytes");
static_assert(offsetof(plk_msm_result_t, log) == 8 && offsetof(plk_msm_result_t, irregular) == 12 &&
                  offsetof(plk_msm_result_t, g1) == 16 && offsetof(plk_msm_result_t, shard) == 128,
              "offsets used by plonkhip/__init__.py");
#define PLK_MSM_SHARDS 16     // ticket shards per MSM record (two per XCD)

#define PLK_NTT_SMALL_LOG 13   // universal small twiddle table covers tiles up to 2^13 rows
#define PLK_SMALL_LOG 12       // poly_mul with N <= 2^12: one workgroup does everything
#define PLK_DIRECT_MAX 32      // poly_mul with min(la, lb) <= 32: direct convolution

void plk_set_error(const char* fmt, ...);
int plk_ctx_retain(void);    // a device prover is alive (capi.hip): plk_shutdown keeps the tables
void plk_ctx_release(void);
int plk_ctx_prepare_device(int dev);   // kernel tables on a further device (helper provers)
int64_t plk_opt(int opt);    // current value of a PLK_OPT_* option (capi.hip)

#define PLK_HIP(call)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess) {                                                              \
      plk_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return PLK_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

// shards.hip: in-process multi-device plk_msm_g1 (plk_init_devices); callers hold the library lock
#define PLK_MAX_SHARDS 16
#define PLK_MAX_DEVICES 64   // device ids with their own NTT tables (ntt.hip)
int plk_cur_device(void);   // the calling thread's current HIP device (0 on error)
// host-time checkpoints (timing builds only: -DPLK_HOST_MARKS=1 records steady-clock times of
// numbered points of a proof's enqueue path and prints their deltas after each proof)
#ifndef PLK_HOST_MARKS
#define PLK_HOST_MARKS 0
#endif
void plk_host_mark(int id);
void plk_host_marks_print(void);
#define PLK_MARK(i) \
  do {                          \
    if (PLK_HOST_MARKS) plk_host_mark(i); \
  } while (0)
// lanes: the entries all name the primary device and stand for host threads of the single-device
// plk_msm_g1 (PLK_OPT_MSM_HOST_LANES), not a plk_init_devices list (plk_devices reports one device)
int plk_shards_setup(const int* ids, int n, const uint32_t* ytab, const uint8_t* exp4, const uint8_t* inv101,
                     bool lanes);
bool plk_shards_are_lanes(void);
void plk_shards_teardown(void);
int plk_shards_count(void);
int plk_shards_devices(int* ids, int cap);
int plk_shards_msm(const uint8_t* pts, const uint8_t* sc, size_t n, uint64_t* log_sum, uint64_t* irregular);

// msm.hip
int plk_msm_upload_tables(const uint32_t* ytab, const uint8_t* exp4, const uint8_t* inv101);
void plk_msm_geometry(uint64_t n, int batch, int* threads, int* blocks, int* groups_per_thread, int* copies,
                      int* half);
int plk_msm_batch_launch(const uint8_t* d_pts, uint64_t pstride, const uint8_t* d_sc, uint64_t sstride, uint64_t n,
                         int batch, PlkMsmResult* d_res, hipStream_t st);
int plk_msm_launch(const uint8_t* d_pts, const uint8_t* d_sc, uint64_t n, PlkMsmResult* d_res, hipStream_t st);
// a fixed SRS in log form (1 byte per point; *d_irregular |= 1 if any encoding is not canonical,
// and the logs are then unusable) and batch MSMs over it
// EXP words {x, y, inf, 0} of the group (uploaded with the MSM tables) on the current device
const uint32_t* plk_msm_exp_words_dev();
int plk_srs_log_launch(const uint8_t* d_pts, uint64_t n, uint8_t* d_logs, uint32_t* d_irregular, hipStream_t st);
int plk_msm_log_batch_launch(const uint8_t* d_logs, uint64_t lstride, const uint8_t* d_sc, uint64_t sstride, uint64_t n,
                             int batch, PlkMsmResult* d_res, hipStream_t st);
int plk_msm_serial_launch(const uint8_t* d_pts, const uint8_t* d_sc, uint64_t n, PlkMsmResult* d_res,
                          hipStream_t st);
int plk_msm_finalize_launch(const uint32_t* d_logs, int batch, int stride, uint8_t* d_out, hipStream_t st);
int plk_msm_combine_launch(const uint32_t* d_logs, int count, uint8_t* d_out, hipStream_t st);

// ntt.hip
struct PlkTwTables {
  const uint32_t *small_f, *small_i;   // T[2^j + r] = w_{2^(j+1)}^(+-r), 2^PLK_NTT_SMALL_LOG entries
  const uint32_t *lo_f, *hi_f;         // w_{2^27}^i = lo[i & 4095] * hi[i >> 12]
  const uint32_t *lo_i, *hi_i;         // same for the inverse root
};
PlkTwTables plk_ntt_tables(void);      // BabyBear
PlkTwTables plk_ntt_tables29(void);    // F29 (roots of order 2^26; lo/hi: w_{2^26}^i = lo[i & 4095] hi[i >> 12])
int plk_ntt_init_tables(void);
void plk_ntt_free_tables(void);
size_t plk_poly_mul_workspace_bytes(uint64_t la, uint64_t lb);
bool plk_poly_mul_is_direct(uint64_t la, uint64_t lb);
int plk_poly_mul_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, uint8_t* d_out,
                        uint32_t* d_nz, void* d_work, hipStream_t st);
int plk_ntt_launch(uint32_t* d, int k, int batch, int inverse, hipStream_t st);
int plk_ntt29_launch(uint32_t* d, int k, int batch, int inverse, hipStream_t st);
// Operand a of a product as an elementwise function of other bytes, computed by the wave
// engine's first forward pass (which also stores the bytes to a[0, la): the last inverse pass's
// top-coefficient terms read them): round 3's
//   A2 B2 = alpha (ab + gamma (a + b) + beta k1 x a + beta x b + (gamma + beta x)(gamma + beta k1 x))
// (src/plonk.h:409-434; prove.hip t2a_kernel is the same map as a launch of its own), the
// challenges read from the prover's scalar slots S at run time
struct WDerive {
  const uint8_t* ab;   // a_x b_x, [0, lab)
  const uint8_t* a;    // a_x, b_x, [0, la)
  const uint8_t* b;
  const uint8_t* S;
  uint64_t la, lab;
  int s_alpha, s_beta, s_gamma, s_bk1;   // slots of alpha, beta, gamma, beta k1 in S
};

struct PlkPolyMulJob {
  const uint8_t* a;
  uint64_t la;
  const uint8_t* b;
  uint64_t lb;
  uint8_t* out;   // la + lb - 1 bytes
  // 1: ADD this product into the preceding job's output (a sum group: the leader and up to two
  // members of one transform size, none longer than the leader's product; the members' out is
  // not written).  The sum is exact while it fits the field (the caller's bound).
  int acc = 0;
  // optional: b's forward transform computed beforehand (plk_poly_mul_pretransform with the
  // same bytes, bt_k and bt_field): used when this product runs at 2^bt_k in field bt_field,
  // which skips b's forward passes; ignored otherwise (the product is the same either way)
  const uint32_t* bt = nullptr;
  int bt_k = 0, bt_field = -1;
  // optional: a's bytes derived in the first forward pass (WDerive; wave-engine products of two
  // or more passes only, one per batch: PLK_ERR_ARG otherwise)
  const WDerive* der = nullptr;
};
int plk_poly_mul_batch_launch(const PlkPolyMulJob* jobs, int nj, void* d_work, size_t work_bytes, hipStream_t st);
bool plk_poly_mul_summable(uint64_t la, uint64_t lb);
// transform size (log2) and field (1 F29, 0 BabyBear) a wave-engine product of this shape runs
// at on its own (sum groups may force BabyBear); -1 when it does not use the wave engine
int plk_poly_mul_transform_plan(uint64_t la, uint64_t lb, int* field);
// the forward transform of b (2^k words into d_out, in the center kernel's load positions) for
// PlkPolyMulJob::bt
int plk_poly_mul_pretransform(const uint8_t* d_b, uint64_t lb, int k, int field, uint32_t* d_out, hipStream_t st);

// ntt_wave.hip (transforms of 2^13 .. 2^27 points).  One product job: u32 work arrays A, B
// (2^k each; a batch's jobs may share one when their operands are the same bytes), byte
// inputs a8[0, la), b8[0, lb), byte output out8[0, out_len + ntop).
struct WJob {
  const uint8_t* a8;
  const uint8_t* b8;
  uint64_t la, lb;
  uint8_t* out8;
  uint64_t out_len;                // outputs of the cyclic transform: min(la + lb - 1, 2^k)
  uint32_t* A;
  uint32_t* B;                     // (bfix: b's finished forward transform, plk_wave_pretransform)
  uint32_t* C = nullptr;           // center output and inverse work array (read by no other job)
  // sum groups: the leader's inverse passes add the members' center outputs (linear), the
  // members run no inverse pass of their own
  uint32_t* S1 = nullptr;
  uint32_t* S2 = nullptr;
  int skip_inv = 0;
  // wrapped products (la + lb - 1 = 2^k + ntop): the top ntop coefficients alias onto the
  // first ntop; the last inverse pass computes them from the bytes (also the sum group's
  // members' ga8/gb8) and corrects both ends
  int ntop = 0;
  int ngroup = 0;
  const uint8_t* ga8[2] = {nullptr, nullptr};
  const uint8_t* gb8[2] = {nullptr, nullptr};
  uint64_t gla[2] = {0, 0}, glb[2] = {0, 0};   // (the members' operand lengths)
  // trimmed length word (poly_new_internal's len, 0 = all zero) written by the last inverse
  // pass; the center kernel zeroes it first (nullptr: not wanted)
  uint32_t* nz = nullptr;
  int bfix = 0;                    // B holds a plk_poly_mul_pretransform result
  int afix = 0;                    // (wave engine only: A finished in the batch, see wt_fixfwd_kernel)
  // (wave engine only, set by it) a sum group whose pointwise products the leader's center item
  // adds before its inverse pass: the members (cm, their A / B / afix / bfix) have no item
  int cm[2] = {-1, -1};
  int ncm = 0;
  int cskip = 0;
  const WDerive* der = nullptr;    // (host side only: PlkPolyMulJob::der, read at launch)
};
constexpr int PLK_WAVE_MAX_JOBS = 12;   // jobs per launch of the wave engine (larger batches run in chunks)
bool plk_wave_ntt_supported(int k);
// field 0 = BabyBear, 1 = F29 (lazy; only when every job's min(la, lb) * 256 < f29::P);
// ninv = 2^-k mod p in normal form for that field
int plk_wave_poly_mul_batch_launch(const WJob* jobs, int nj, int k, int field, uint32_t ninv, hipStream_t st);
int plk_wave_ntt_launch(uint32_t* d, int k, int batch, int inverse, int field, hipStream_t st);   // field 0 BabyBear, 1 F29
int plk_wave_pretransform(const uint8_t* b8, uint64_t lb, int k, int field, uint32_t* d_out, hipStream_t st);
int plk_wave_init_coltabs(void);    // after plk_ntt_init_tables' root tables
void plk_wave_free_coltabs(void);

// polyops.hip: poly_eval / poly_divide / matrix ops
#define PLK_EVAL_MAX_JOBS 32
int plk_poly_eval_batch_launch(const uint8_t* const* polys, const uint64_t* lens, const uint8_t* xs, int nj,
                               uint8_t* d_y, void* d_tick, hipStream_t st);
size_t plk_poly_divide_workspace_bytes(uint64_t nl, uint64_t dl);
int plk_poly_divide_launch(const uint8_t* d_num, uint64_t nl, const uint8_t* den, uint64_t dl, uint8_t* d_q,
                           uint8_t* d_rem, uint32_t* d_lens, void* d_work, hipStream_t st);
int plk_matrix_mul_launch(const uint8_t* d_a, uint64_t m, uint64_t k, const uint8_t* d_b, uint64_t n, uint8_t* d_out,
                          hipStream_t st);
int plk_matrix_inv_launch(const uint8_t* d_mat, uint64_t n, uint8_t* d_aug, uint8_t* d_out, hipStream_t st);
// ntt.hip: index + 1 of the last non-zero byte of d[0, len) (0 if none) into *d_nz
int plk_trim_launch(const uint8_t* d, uint64_t len, uint32_t* d_nz, hipStream_t st);
