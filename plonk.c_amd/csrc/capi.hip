// C ABI of libplonkhip (include/plonkhip.h): context, device buffers, host-buffer wrappers
// around the gfx950 kernels in msm.hip and ntt.hip.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "plk_device.h"
#include "plk_internal.h"

namespace {

thread_local char g_err[512] = "";

struct Ctx {
  std::mutex mu;            // guards everything below; never destroyed (plk_shutdown resets fields)
  bool ready = false;
  int device = -1;
  int live_provers = 0;     // plk_prover_t objects alive: they use the NTT tables
  hipStream_t st = nullptr;
  uint8_t gen[3] = {0, 0, 0};
  // MSM staging (host-buffer plk_msm_g1)
  uint8_t* d_pts = nullptr;
  size_t cap_pts = 0;
  uint8_t* d_sc = nullptr;
  size_t cap_sc = 0;
  PlkMsmResult* d_res = nullptr;
  // SRS upload cache (layer 4): the device copy of the last point array, keyed by the
  // caller's pointer; reused when the first 3n bytes still equal the host mirror (memcmp: exact,
  // no hash collisions).  srs_eval_at_s passes the same srs->g1s on every commitment of a proof
  // (src/plonk.h:299-301, 379, 522-524, 620-621) with vs->len <= srs->len points.
  const uint8_t* srs_key = nullptr;
  size_t srs_cached = 0;    // bytes valid in d_pts / h_srs
  uint8_t* h_srs = nullptr; // host mirror of the cached bytes
  size_t cap_h_srs = 0;
  // pinned staging for host -> device copies
  uint8_t* h_stage = nullptr;
  size_t cap_stage = 0;
  bool stage_busy = false;  // staged copies of a call may still be in flight (see Stage)
  // toy-size calls (the reference's own 4-gate prove makes ~100 of them): inputs and outputs in
  // mapped, coherent pinned memory the kernels read and write directly (no runtime blit copies),
  // and evaluation tick words that stay zeroed between calls (the kernel re-arms them)
  uint8_t* h_tiny = nullptr;
  uint8_t* d_tiny = nullptr;  // its device address
  uint8_t* d_tick0 = nullptr;
  size_t cap_tick0 = 0;
  // poly_mul staging
  uint8_t* d_a = nullptr;
  size_t cap_a = 0;
  uint8_t* d_b = nullptr;
  size_t cap_b = 0;
  uint8_t* d_out = nullptr;
  size_t cap_out = 0;
  uint32_t* d_nz = nullptr;
  void* d_work = nullptr;
  size_t cap_work = 0;
  // small-op staging (poly_divide / poly_eval / interpolate): one device arena
  uint8_t* d_ops = nullptr;
  size_t cap_ops = 0;
  // further devices holding the kernel tables (helper provers, plk_ctx_prepare_device)
  bool dev_tables[PLK_MAX_DEVICES] = {};
} g;

// the initialised device, published after init_locked (-1: not initialised), so that device
// entry points take no lock once the library is up: a host-buffer call holding g.mu for its
// uploads or a serial fold does not stall another thread's kernel launches
std::atomic<int> g_live_dev{-1};

// ---- E(F101) tables, built from the group law on canonical points ----------------------
struct HP { int x, y, inf; };

int md(int v) { v %= PLK_GF_P; return v < 0 ? v + PLK_GF_P : v; }
int inv101(int a) {  // a^99 mod 101 (Fermat, 0 -> 0), same as the reference gf_inv
  int r = 1, b = md(a), e = PLK_GF_P - 2;
  while (e) { if (e & 1) r = r * b % PLK_GF_P; b = b * b % PLK_GF_P; e >>= 1; }
  return r;
}
HP hp_add(HP a, HP b) {
  if (a.inf) return b;
  if (b.inf) return a;
  int m;
  if (a.x == b.x) {
    if (md(a.y + b.y) == 0) return HP{0, 0, 1};
    m = md(3 * a.x * a.x) * inv101(md(2 * a.y)) % PLK_GF_P;
  } else {
    m = md(b.y - a.y) * inv101(md(b.x - a.x)) % PLK_GF_P;
  }
  const int xr = md(m * m - a.x - b.x);
  const int yr = md(m * (a.x - xr) - a.y);
  return HP{xr, yr, 0};
}

// the kernel tables as built (uploaded again to every further device of plk_init_devices)
uint32_t s_ytab[512];
uint8_t s_exp4[PLK_GROUP_ORDER * 4];
uint8_t s_inv[PLK_GF_P];

int build_group_tables(uint8_t gen_out[3]) {
  std::vector<HP> pts;
  for (int x = 0; x < PLK_GF_P; x++)
    for (int y = 0; y < PLK_GF_P; y++)
      if (y * y % PLK_GF_P == (x * x * x + 3) % PLK_GF_P) pts.push_back(HP{x, y, 0});
  if (pts.size() + 1 != PLK_GROUP_ORDER) {
    plk_set_error("E(F101) has %zu points, expected 102", pts.size() + 1);
    return PLK_ERR_ARG;
  }
  HP g0{0, 0, 1};
  for (const HP& p : pts) {  // first (x, y) point of order 102
    HP q = p;
    int ord = 1;
    while (!q.inf && ord <= PLK_GROUP_ORDER) { q = hp_add(q, p); ord++; }
    if (ord == PLK_GROUP_ORDER) { g0 = p; break; }
  }
  if (g0.inf) {
    plk_set_error("no generator of order 102 found");
    return PLK_ERR_ARG;
  }
  static int logt[PLK_GF_P][PLK_GF_P];
  for (auto& row : logt)
    for (int& v : row) v = -1;
  uint8_t exp4[PLK_GROUP_ORDER * 4];
  HP q{0, 0, 1};
  for (int k = 0; k < PLK_GROUP_ORDER; k++) {
    exp4[4 * k + 0] = (uint8_t)q.x;
    exp4[4 * k + 1] = (uint8_t)q.y;
    exp4[4 * k + 2] = (uint8_t)q.inf;
    exp4[4 * k + 3] = 0;
    if (!q.inf) logt[q.x][q.y] = k;
    q = hp_add(q, g0);
  }
  // Lookup table of the MSM kernel (msm.hip): cubing is a bijection of GF(101), so each y
  // has exactly one x on the curve.  Index y | (inf & 1) << 8; a point encoded as
  // k = x << 8 | y << 16 | inf << 24 is canonical iff E[idx] - k < 256, and then that
  // difference is its log.  Entries that must never match get a wrong y byte.
  uint32_t ytab[512];
  for (int i = 0; i < 512; i++) ytab[i] = (uint32_t)((i & 0xFF) ^ 1) << 16;
  for (int x = 0; x < PLK_GF_P; x++)
    for (int y = 0; y < PLK_GF_P; y++)
      if (logt[x][y] >= 0) ytab[y] = (uint32_t)x << 8 | (uint32_t)y << 16 | (uint32_t)logt[x][y];
  ytab[256] = 1u << 24;  // identity {0, 0, 1}: log 0
  for (int y = 0; y < PLK_GF_P; y++)
    if ((ytab[y] >> 16 & 0xFF) != (uint32_t)y) {
      plk_set_error("E(F101): no point with y = %d", y);
      return PLK_ERR_ARG;
    }
  uint8_t inv[PLK_GF_P];
  for (int a = 0; a < PLK_GF_P; a++) inv[a] = (uint8_t)inv101(a);
  gen_out[0] = (uint8_t)g0.x;
  gen_out[1] = (uint8_t)g0.y;
  gen_out[2] = 0;
  memcpy(s_ytab, ytab, sizeof s_ytab);
  memcpy(s_exp4, exp4, sizeof s_exp4);
  memcpy(s_inv, inv, sizeof s_inv);
  return plk_msm_upload_tables(ytab, exp4, inv);
}

template <class T>
int grow(T** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return PLK_OK;
  size_t n = *cap ? *cap : 4096;
  while (n < need) n *= 2;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipMalloc((void**)p, n);
  if (e != hipSuccess) {
    plk_set_error("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    return PLK_ERR_NOMEM;
  }
  *cap = n;
  return PLK_OK;
}

int grow_host(uint8_t** p, size_t* cap, size_t need, bool pinned) {
  if (*cap >= need && *p) return PLK_OK;
  size_t n = *cap ? *cap : 4096;
  while (n < need) n *= 2;
  if (*p) {
    if (pinned) (void)hipHostFree(*p);
    else free(*p);
  }
  *p = nullptr;
  *cap = 0;
  if (pinned) {
    if (hipHostMalloc((void**)p, n, hipHostMallocDefault) != hipSuccess) *p = nullptr;
  } else {
    *p = (uint8_t*)malloc(n);
  }
  if (!*p) {
    plk_set_error("host allocation of %zu bytes failed", n);
    return PLK_ERR_NOMEM;
  }
  *cap = n;
  return PLK_OK;
}

// Host -> device through the pinned staging buffer in chunks (the caller's pageable memory is
// copied into pinned memory while the previous chunk's DMA runs).  Synchronous on g.st.
constexpr size_t STAGE_CHUNK = 4u << 20;
int upload(uint8_t* dst, const uint8_t* src, size_t bytes) {
  constexpr size_t CHUNK = STAGE_CHUNK;
  if (!bytes) return PLK_OK;
  int rc = grow_host(&g.h_stage, &g.cap_stage, 2 * CHUNK, true);
  if (rc) return rc;
  if (g.stage_busy) {
    PLK_HIP(hipStreamSynchronize(g.st));
    g.stage_busy = false;
  }
  hipEvent_t done[2] = {nullptr, nullptr};
  PLK_HIP(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
  PLK_HIP(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
  for (size_t off = 0, k = 0; off < bytes; off += CHUNK, k ^= 1) {
    const size_t len = bytes - off < CHUNK ? bytes - off : CHUNK;
    uint8_t* h = g.h_stage + k * CHUNK;
    if (off >= 2 * CHUNK) PLK_HIP(hipEventSynchronize(done[k]));   // this half's previous DMA
    memcpy(h, src + off, len);
    PLK_HIP(hipMemcpyAsync(dst + off, h, len, hipMemcpyHostToDevice, g.st));
    PLK_HIP(hipEventRecord(done[k], g.st));
  }
  PLK_HIP(hipStreamSynchronize(g.st));
  (void)hipEventDestroy(done[0]);
  (void)hipEventDestroy(done[1]);
  return PLK_OK;
}

// The small copies of one host-buffer call without a synchronisation per copy (the drop-in makes
// many calls of a few bytes each: a stream synchronize per upload cost ~20 us apiece): uploads are
// copied into the pinned staging buffer and enqueued, downloads land in staging and are copied out
// after the call's ONE stream synchronize (finish).  A copy that does not fit takes the chunked
// upload() / a direct copy.  Staging is reused by the next call only after that synchronize
// (stage_busy guards calls that returned early on an error).
struct Stage {
  struct Down {
    uint8_t* dst;
    size_t off, n;
  };
  size_t used = 0;
  Down downs[8];
  int nd = 0;
  int begin() {
    int rc = grow_host(&g.h_stage, &g.cap_stage, 2 * STAGE_CHUNK, true);
    if (rc) return rc;
    if (g.stage_busy) {
      PLK_HIP(hipStreamSynchronize(g.st));
      g.stage_busy = false;
    }
    return PLK_OK;
  }
  bool fits(size_t n) const { return used + ((n + 255) & ~(size_t)255) <= 2 * STAGE_CHUNK; }
  int up(uint8_t* d, const uint8_t* h, size_t n) {
    if (!n) return PLK_OK;
    if (!fits(n)) return upload(d, h, n);   // (synchronises: earlier staged copies are done)
    memcpy(g.h_stage + used, h, n);
    PLK_HIP(hipMemcpyAsync(d, g.h_stage + used, n, hipMemcpyHostToDevice, g.st));
    g.stage_busy = true;
    used += (n + 255) & ~(size_t)255;
    return PLK_OK;
  }
  int down(uint8_t* h, const uint8_t* d, size_t n) {
    if (!n) return PLK_OK;
    if (!fits(n) || nd == 8) {
      PLK_HIP(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, g.st));
      return PLK_OK;
    }
    PLK_HIP(hipMemcpyAsync(g.h_stage + used, d, n, hipMemcpyDeviceToHost, g.st));
    g.stage_busy = true;
    downs[nd++] = Down{h, used, n};
    used += (n + 255) & ~(size_t)255;
    return PLK_OK;
  }
  int finish() {
    PLK_HIP(hipStreamSynchronize(g.st));
    g.stage_busy = false;
    for (int i = 0; i < nd; i++) memcpy(downs[i].dst, g.h_stage + downs[i].off, downs[i].n);
    nd = 0;
    used = 0;
    return PLK_OK;
  }
};

// Toy-size calls: TINY_BYTES of mapped coherent pinned memory (h_tiny / d_tiny).  Only for
// kernels that read their inputs and plain-store their outputs there (no atomics on host memory);
// PLK_OPT_TINY_CALLS = 0 sends every call through the staged device copies instead.
constexpr size_t TINY_BYTES = 16u << 10;
bool tiny_ok(size_t bytes) {
  if (!plk_opt(PLK_OPT_TINY_CALLS) || bytes > TINY_BYTES) return false;
  if (!g.h_tiny) {
    if (hipHostMalloc((void**)&g.h_tiny, TINY_BYTES, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      g.h_tiny = nullptr;
      return false;
    }
    if (hipHostGetDevicePointer((void**)&g.d_tiny, g.h_tiny, 0) != hipSuccess) {
      (void)hipHostFree(g.h_tiny);
      g.h_tiny = g.d_tiny = nullptr;
      return false;
    }
  }
  return true;
}
// zeroed evaluation tick words for n jobs (the kernel leaves them zero again)
int tick0(int n, uint8_t** out) {
  const size_t need = plk_poly_eval_workspace(n);
  if (g.cap_tick0 < need) {
    (void)hipFree(g.d_tick0);
    g.d_tick0 = nullptr;
    g.cap_tick0 = 0;
    PLK_HIP(hipMalloc((void**)&g.d_tick0, need));
    PLK_HIP(hipMemsetAsync(g.d_tick0, 0, need, g.st));
    g.cap_tick0 = need;
  }
  *out = g.d_tick0;
  return PLK_OK;
}

// "a,b,c" -> device ids (at most PLK_MAX_SHARDS); returns the count, 0 if malformed
int parse_devices(const char* e, int* ids) {
  int n = 0;
  const char* p = e;
  while (*p && n < PLK_MAX_SHARDS) {
    char* end = nullptr;
    const long v = strtol(p, &end, 10);
    if (end == p || v < 0 || v > 4095) return 0;
    ids[n++] = (int)v;
    p = end;
    while (*p == ' ') p++;
    if (*p == ',') p++;
    else if (*p) return 0;
  }
  return n;
}

// the single-device plk_msm_g1's host lanes: PLK_OPT_MSM_HOST_LANES shards of `device`
int setup_lanes(int device) {
  const int nl = (int)std::min<int64_t>(plk_opt(PLK_OPT_MSM_HOST_LANES), PLK_MAX_SHARDS);
  int ids[PLK_MAX_SHARDS];
  for (int i = 0; i < nl; i++) ids[i] = device;
  return plk_shards_setup(ids, nl, s_ytab, s_exp4, s_inv, true);
}

int init_locked(int device) {
  if (g.ready) {
    if (device >= 0 && device != g.device) {
      plk_set_error("libplonkhip is initialised on device %d; plk_init(%d) refused (plk_shutdown first)",
                    g.device, device);
      return PLK_ERR_ARG;
    }
    return PLK_OK;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    plk_set_error("no HIP device available (libplonkhip has no CPU fallback)");
    return PLK_ERR_NODEV;
  }
  int list[PLK_MAX_SHARDS], nlist = 0;
  if (device < 0) {   // implicit: $PLK_DEVICE ("2", or a list "0,1,2,3" of shards), else the current device
    const char* e = getenv("PLK_DEVICE");
    if (e) {
      nlist = parse_devices(e, list);
      if (!nlist) {
        plk_set_error("PLK_DEVICE=\"%s\": expected a device id or a comma list of ids", e);
        return PLK_ERR_ARG;
      }
      device = list[0];
    } else if (hipGetDevice(&device) != hipSuccess) {
      device = 0;
    }
  }
  for (int i = 0; i < (nlist ? nlist : 1); i++)
    if ((nlist ? list[i] : device) >= count) {
      plk_set_error("device %d out of range (%d devices)", nlist ? list[i] : device, count);
      return PLK_ERR_NODEV;
    }
  PLK_HIP(hipSetDevice(device));
  PLK_HIP(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
  int rc = build_group_tables(g.gen);
  if (rc) return rc;
  if ((rc = plk_ntt_init_tables())) return rc;
  PLK_HIP(hipMalloc((void**)&g.d_res, sizeof(PlkMsmResult)));
  PLK_HIP(hipMemset(g.d_res, 0, sizeof(PlkMsmResult)));
  PLK_HIP(hipMalloc((void**)&g.d_nz, 16));
  if (nlist > 1 || plk_opt(PLK_OPT_MSM_HOST_LANES) > 1) {
    // the shards first: a failure leaves the library uninitialised (every later call retries
    // and reports it) instead of published and quietly running on one device.  One device:
    // host lanes of it (PLK_OPT_MSM_HOST_LANES), so that plk_msm_g1's memcmp and staging run
    // on several host threads
    rc = nlist > 1 ? plk_shards_setup(list, nlist, s_ytab, s_exp4, s_inv, false) : setup_lanes(device);
    (void)hipSetDevice(device);
    if (rc && nlist <= 1) {
      // host lanes are an optimisation of the one-device call: if they cannot be set up (e.g. the
      // pinned staging is refused) the library runs without them instead of failing;
      // the reason stays readable through plk_last_error until the next error
      const std::string why = g_err;
      plk_shards_teardown();
      plk_set_error("plk_init: host lanes unavailable, single-lane plk_msm_g1 (%s)", why.c_str());
      rc = PLK_OK;
    }
    if (rc) {
      const std::string why = g_err;
      plk_shards_teardown();
      (void)hipFree(g.d_res);
      (void)hipFree(g.d_nz);
      g.d_res = nullptr;
      g.d_nz = nullptr;
      plk_ntt_free_tables();
      (void)hipStreamDestroy(g.st);
      g.st = nullptr;
      plk_set_error("%s", why.c_str());
      return rc;
    }
  }
  g.device = device;
  g.ready = true;
  g_live_dev.store(device, std::memory_order_release);
  return PLK_OK;
}

// Host-buffer entry points hold g.mu for the whole call and run on g.device (set for the
// call's thread).  Device entry points take the lock only to initialise, and then require
// the calling thread's current device to be the library's: their stream and buffers belong to
// that device, and the tables (dlog, NTT twiddles) exist only there.
int ensure_locked(void) {
  int rc = init_locked(-1);
  if (rc) return rc;
  return hipSetDevice(g.device) == hipSuccess ? PLK_OK : PLK_ERR_HIP;
}

int ensure_dev(void) {
  int dev = g_live_dev.load(std::memory_order_acquire);
  if (dev < 0) {
    std::lock_guard<std::mutex> lk(g.mu);
    int rc = init_locked(-1);
    if (rc) return rc;
    dev = g.device;
  }
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return PLK_ERR_HIP;
  if (cur != dev) {
    plk_set_error("libplonkhip runs on device %d but the calling thread's current device is %d", dev, cur);
    return PLK_ERR_ARG;
  }
  return PLK_OK;
}

// ---- options (include/plonkhip.h PLK_OPT_*): the library's only switches besides the
// device selection; atomics so that a launch reads a consistent value without the lock
struct OptDef {
  int64_t def, lo, hi;
  bool init_only;
};
const OptDef kOpt[PLK_OPT_COUNT] = {
    {0, 0, 0, false},                          // (0: unused)
    {1, 0, 1, false},                          // TINY_CALLS
    {0, 0, 1, false},                          // PROVE_SYNC
    {0, 0, (1ll << 26) - 3670016 + 1, false},  // POLY_BLOCK_L
    {0, 0, 3670016, false},                    // POLY_BLOCK_S
    {1, 0, 1, false},                          // NTT_F29
    {1, 0, 1, false},                          // NTT_SHARE
    {1, 0, 2, false},                          // NTT_SHARED_FIX
    {21, 13, 28, true},                        // NTT_T13_MIN_K (the column tables depend on it)
    {0, 0, 1 << 20, false},                    // NTT_CENTER_BLOCKS
    {0, 0, 1024, false},                       // MSM_THREADS
    {0, 0, 8 * 65535, false},                  // MSM_MAX_BLOCKS
    {0, 0, 4, false},                          // MSM_GROUPS
    {0, 0, 8, false},                          // MSM_COPIES
    {1, 0, 1, false},                          // MSM_HALF
    {1 << 16, 1, 1ll << 40, false},            // MSM_SHARD_MIN
    {1, 0, 1, false},                          // NTT_CENTER_SUM
    {4, 1, PLK_MAX_SHARDS, false},             // MSM_HOST_LANES (read at plk_init / plk_init_devices)
    {2, 0, 2, false},                          // PROVE_DERIVE_T2A (2: in the t_2 product's first pass)
    {1, 0, 1, false},                          // NTT_TABLE_SHARE
    {0, 0, 1, false},                          // NTT_LAUNCH_LOG
    {0, 0, 1, false},                          // PROVE_FUSE_DIV (measured slower)
    {1, 0, 1, false},                          // PROVE_SRS_LOGS
    {1, 0, 1, false},                          // PROVE_PACK_FUSE
    {1, 0, 2, false},                          // PROVE_EARLY_COMMITS (2: in round 4's evaluation launch)
    {0, 0, 1, false},                          // PROVE_HELPER_COPY (tests: the distinct-device input path on one GPU)
    {1, 0, 1, false},                          // PROVE_EVAL_AGG
    {0, 0, 1, false},                          // PROVE_GRAPH
    {32768, 0, 1ll << 40, false},              // DROPIN_HOST_WORK (read by include/plk_host.h only)
};
struct Opts {
  std::atomic<int64_t> v[PLK_OPT_COUNT];
  Opts() {
    for (int i = 0; i < PLK_OPT_COUNT; i++) v[i].store(kOpt[i].def);
  }
} g_opt;

// Bump-carves the small-op device arena (poly_eval / poly_divide / matrix host calls).
struct Arena {
  size_t off = 0;
  size_t take(size_t b) {
    const size_t o = off;
    off += (b + 255) & ~(size_t)255;
    return o;
  }
};

// Device entry points run on exactly the stream they are given; NULL is HIP's null stream
// (torch's default stream also has handle 0).  g.st is used only by the host-buffer calls.
hipStream_t pick(void* s) { return (hipStream_t)s; }

}  // namespace

void plk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

int64_t plk_opt(int opt) {
  return opt > 0 && opt < PLK_OPT_COUNT ? g_opt.v[opt].load(std::memory_order_relaxed) : -1;
}

// device provers (prove.hip) hold the context: plk_shutdown keeps the tables while any is alive
int plk_ctx_retain(void) {
  int rc = ensure_dev();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g.mu);
  g.live_provers++;
  return PLK_OK;
}

void plk_ctx_release(void) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (g.live_provers > 0) g.live_provers--;
}

// A further device runs the library's kernels (a helper prover of plk_prover_attach_helpers):
// its NTT root / column tables and the MSM __constant__ tables are built there once.  Returns
// with the calling thread's current device unchanged.
int plk_ctx_prepare_device(int dev) {
  int rc = ensure_dev();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g.mu);
  if (dev < 0 || dev >= PLK_MAX_DEVICES || dev >= plk_device_count()) {
    plk_set_error("device %d out of range", dev);
    return PLK_ERR_NODEV;
  }
  if (dev == g.device || g.dev_tables[dev]) return PLK_OK;
  const int prev = plk_cur_device();
  PLK_HIP(hipSetDevice(dev));
  rc = plk_ntt_init_tables();
  if (!rc) rc = plk_msm_upload_tables(s_ytab, s_exp4, s_inv);
  (void)hipSetDevice(prev);
  if (!rc) g.dev_tables[dev] = true;
  return rc;
}

extern "C" {

const char* plk_last_error(void) { return g_err; }

int plk_set_option(int opt, int64_t value) {
  if (opt <= 0 || opt >= PLK_OPT_COUNT) {
    plk_set_error("plk_set_option: unknown option %d", opt);
    return PLK_ERR_ARG;
  }
  const OptDef& d = kOpt[opt];
  if (value < d.lo || value > d.hi) {
    plk_set_error("plk_set_option(%d): %lld outside [%lld, %lld]", opt, (long long)value, (long long)d.lo,
                  (long long)d.hi);
    return PLK_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g.mu);
  if (d.init_only && g.ready && g_opt.v[opt].load() != value) {
    plk_set_error("plk_set_option(%d) shapes the tables plk_init builds: set it before plk_init", opt);
    return PLK_ERR_ARG;
  }
  g_opt.v[opt].store(value);
  return PLK_OK;
}

int64_t plk_get_option(int opt) { return plk_opt(opt); }
const char* plk_version(void) { return "libplonkhip 0.1 gfx950"; }

int plk_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int plk_init(int device) {
  std::lock_guard<std::mutex> lk(g.mu);
  return init_locked(device);
}

int plk_init_devices(const int* ids, int n) {
  if (!ids || n < 1 || n > PLK_MAX_SHARDS) {
    plk_set_error("plk_init_devices: %d devices (1..%d)", n, PLK_MAX_SHARDS);
    return PLK_ERR_ARG;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    plk_set_error("no HIP device available (libplonkhip has no CPU fallback)");
    return PLK_ERR_NODEV;
  }
  for (int i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= count) {
      plk_set_error("plk_init_devices: device %d out of range (%d devices)", ids[i], count);
      return PLK_ERR_NODEV;
    }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = init_locked(ids[0]);   // the primary: tables, NTT, prover, every non-MSM call
  if (rc) return rc;
  rc = n > 1 ? plk_shards_setup(ids, n, s_ytab, s_exp4, s_inv, false) : setup_lanes(g.device);
  (void)hipSetDevice(g.device);
  return rc;
}

int plk_devices(int* ids, int cap) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.ready) return 0;
  const int ns = plk_shards_count();
  if (ns > 1 && !plk_shards_are_lanes()) return plk_shards_devices(ids, cap);
  if (ids && cap > 0) ids[0] = g.device;
  return 1;
}

void plk_shutdown(void) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.ready) return;
  if (g.live_provers > 0) {   // their kernels read the NTT tables: keep everything
    plk_set_error("plk_shutdown: %d prover(s) still alive; nothing released", g.live_provers);
    return;
  }
  g_live_dev.store(-1, std::memory_order_release);
  plk_shards_teardown();
  (void)hipSetDevice(g.device);
  (void)hipStreamSynchronize(g.st);
  (void)hipFree(g.d_pts); (void)hipFree(g.d_sc); (void)hipFree(g.d_res);
  (void)hipFree(g.d_a); (void)hipFree(g.d_b); (void)hipFree(g.d_out); (void)hipFree(g.d_nz); (void)hipFree(g.d_work);
  (void)hipFree(g.d_ops);
  if (g.h_stage) (void)hipHostFree(g.h_stage);
  if (g.h_tiny) (void)hipHostFree(g.h_tiny);
  (void)hipFree(g.d_tick0);
  free(g.h_srs);
  plk_ntt_free_tables();   // (every device's)
  for (bool& b : g.dev_tables) b = false;
  (void)hipSetDevice(g.device);
  (void)hipStreamDestroy(g.st);
  // reset field by field: the mutex (held here) stays as it is
  g.ready = false;
  g.device = -1;
  g.st = nullptr;
  g.d_pts = g.d_sc = g.d_a = g.d_b = g.d_out = g.d_ops = nullptr;
  g.cap_pts = g.cap_sc = g.cap_a = g.cap_b = g.cap_out = g.cap_work = g.cap_ops = 0;
  g.d_res = nullptr;
  g.d_nz = nullptr;
  g.d_work = nullptr;
  g.srs_key = nullptr;
  g.srs_cached = 0;
  g.h_srs = nullptr;
  g.cap_h_srs = 0;
  g.h_stage = nullptr;
  g.cap_stage = 0;
  g.h_tiny = g.d_tiny = g.d_tick0 = nullptr;
  g.cap_tick0 = 0;
}

int plk_dlog_generator(uint8_t out[3]) {
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  memcpy(out, g.gen, 3);
  return PLK_OK;
}

}  // extern "C"

namespace {
// plk_msm_g1 on the primary device alone (g.mu held): the cached SRS upload, one launch, and the
// reference's raw fold on the device when an input is not a canonical group element
int msm_single_locked(const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t out[3]) {
  int rc;
  if ((rc = grow(&g.d_sc, &g.cap_sc, n + 16))) return rc;
  const size_t pb = 3 * n;
  const bool hit = n && points == g.srs_key && pb <= g.srs_cached && memcmp(points, g.h_srs, pb) == 0;
  if (!hit && n) {
    // keep the device copy of the longer of (cached, new) when the new bytes extend it
    if (pb > g.cap_pts) {
      g.srs_key = nullptr;
      g.srs_cached = 0;
      if ((rc = grow(&g.d_pts, &g.cap_pts, pb + 16))) return rc;
    }
    if ((rc = grow_host(&g.h_srs, &g.cap_h_srs, pb + 16, false))) return rc;
    g.srs_key = nullptr;   // invalid until the upload completed
  }
  Stage S;
  if ((rc = S.begin())) return rc;
  if (!hit && n) {
    if ((rc = S.up(g.d_pts, points, pb))) return rc;   // (ordered before the kernel on g.st)
    memcpy(g.h_srs, points, pb);
    g.srs_key = points;
    g.srs_cached = pb;
  }
  if ((rc = S.up(g.d_sc, scalars, n))) return rc;
  if ((rc = plk_msm_launch(g.d_pts, g.d_sc, n, g.d_res, g.st))) return rc;
  PlkMsmResult h;
  if ((rc = S.down((uint8_t*)&h, (const uint8_t*)g.d_res, 32)) || (rc = S.finish())) return rc;   // log, irregular, g1
  if (h.irregular) {
    if ((rc = plk_msm_serial_launch(g.d_pts, g.d_sc, n, g.d_res, g.st))) return rc;
    PLK_HIP(hipMemcpyAsync(&h, g.d_res, sizeof h, hipMemcpyDeviceToHost, g.st));
    PLK_HIP(hipStreamSynchronize(g.st));
  }
  memcpy(out, h.g1, 3);
  return PLK_OK;
}
}  // namespace

extern "C" {

int plk_msm_g1(const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t out[3]) {
  if ((!points || !scalars) && n) { plk_set_error("plk_msm_g1: NULL input"); return PLK_ERR_ARG; }
  if (!out) { plk_set_error("plk_msm_g1: NULL out"); return PLK_ERR_ARG; }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  if (plk_shards_count() > 1 && n >= (size_t)plk_opt(PLK_OPT_MSM_SHARD_MIN)) {
    // point-range shards on the plk_init_devices list; the exchange is a host sum of their
    // partial logs.  An irregular encoding anywhere: the reference's raw fold is serial and
    // order-dependent, so the whole input is folded on the primary device instead
    uint64_t ls = 0, irr = 0;
    if ((rc = plk_shards_msm(points, scalars, n, &ls, &irr))) return rc;
    PLK_HIP(hipSetDevice(g.device));
    if (irr) return msm_single_locked(points, scalars, n, out);
    memcpy(out, s_exp4 + 4 * (ls % PLK_GROUP_ORDER), 3);
    return PLK_OK;
  }
  return msm_single_locked(points, scalars, n, out);
}

int plk_poly_mul(const uint8_t* a, size_t la, const uint8_t* b, size_t lb, uint8_t* out, size_t* out_len) {
  if (!out_len) { plk_set_error("plk_poly_mul: NULL out_len"); return PLK_ERR_ARG; }
  if (la == 0 || lb == 0) {
    // reference: calloc(la+lb-1) of zeros, poly_new trims to one zero (or keeps length 0)
    const size_t rl = la + lb - 1;
    if (la + lb == 0) { plk_set_error("plk_poly_mul: both polynomials empty"); return PLK_ERR_ARG; }
    if (rl && out) out[0] = 0;
    *out_len = rl ? 1 : 0;
    return PLK_OK;
  }
  if (!a || !b || !out) { plk_set_error("plk_poly_mul: NULL buffer"); return PLK_ERR_ARG; }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  const size_t rl = la + lb - 1;
  if (plk_poly_mul_is_direct(la, lb) && tiny_ok(la + lb + rl + 128)) {   // toy sizes: no copies
    if (g.stage_busy) {
      PLK_HIP(hipStreamSynchronize(g.st));
      g.stage_busy = false;
    }
    const size_t o_b = (la + 31) & ~(size_t)15, o_o = o_b + ((lb + 31) & ~(size_t)15);
    const size_t o_nz = (o_o + rl + 31) & ~(size_t)15;
    memcpy(g.h_tiny, a, la);
    memcpy(g.h_tiny + o_b, b, lb);
    if ((rc = plk_poly_mul_launch(g.d_tiny, la, g.d_tiny + o_b, lb, g.d_tiny + o_o, (uint32_t*)(g.d_tiny + o_nz),
                                  nullptr, g.st)))
      return rc;
    PLK_HIP(hipStreamSynchronize(g.st));
    uint32_t nz;
    memcpy(&nz, g.h_tiny + o_nz, 4);
    memcpy(out, g.h_tiny + o_o, rl);
    *out_len = nz ? nz : 1;
    return PLK_OK;
  }
  const size_t ws = plk_poly_mul_workspace_bytes(la, lb);
  if ((rc = grow(&g.d_a, &g.cap_a, la + 16)) || (rc = grow(&g.d_b, &g.cap_b, lb + 16)) ||
      (rc = grow(&g.d_out, &g.cap_out, rl + 16)))
    return rc;
  if (ws && (rc = grow((uint8_t**)&g.d_work, &g.cap_work, ws))) return rc;
  Stage S;
  if ((rc = S.begin()) || (rc = S.up(g.d_a, a, la)) || (rc = S.up(g.d_b, b, lb))) return rc;
  if ((rc = plk_poly_mul_launch(g.d_a, la, g.d_b, lb, g.d_out, g.d_nz, g.d_work, g.st))) return rc;
  uint32_t nz = 0;
  if ((rc = S.down(out, g.d_out, rl)) || (rc = S.down((uint8_t*)&nz, (const uint8_t*)g.d_nz, 4)) ||
      (rc = S.finish()))
    return rc;
  *out_len = nz ? nz : 1;
  return PLK_OK;
}

// ---- device-resident ------------------------------------------------------------------
int plk_msm_result_init(plk_msm_result_t* d_res, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  PLK_HIP(hipMemsetAsync(d_res, 0, sizeof(plk_msm_result_t), pick(stream)));
  return PLK_OK;
}

int plk_msm_g1_dev(const uint8_t* d_points, const uint8_t* d_scalars, size_t n, plk_msm_result_t* d_res,
                   void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_msm_launch(d_points, d_scalars, n, d_res, pick(stream));
}

int plk_msm_g1_batch_dev(const uint8_t* d_points, size_t points_stride, const uint8_t* d_scalars,
                         size_t scalars_stride, size_t n, int batch, plk_msm_result_t* d_res, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_msm_batch_launch(d_points, points_stride, d_scalars, scalars_stride, n, batch, d_res, pick(stream));
}

int plk_msm_g1_serial_dev(const uint8_t* d_points, const uint8_t* d_scalars, size_t n, plk_msm_result_t* d_res,
                          void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_msm_serial_launch(d_points, d_scalars, n, d_res, pick(stream));
}

int plk_msm_combine_dev(const uint32_t* d_logs, int count, uint8_t* d_out3, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_msm_combine_launch(d_logs, count, d_out3, pick(stream));
}

int plk_msm_finalize_dev(const uint32_t* d_logs, int batch, int stride, uint8_t* d_out4, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_msm_finalize_launch(d_logs, batch, stride, d_out4, pick(stream));
}

size_t plk_poly_mul_workspace(size_t la, size_t lb) { return plk_poly_mul_workspace_bytes(la, lb); }

int plk_poly_mul_dev(const uint8_t* d_a, size_t la, const uint8_t* d_b, size_t lb, uint8_t* d_out,
                     uint32_t* d_out_nz, void* d_work, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_poly_mul_launch(d_a, la, d_b, lb, d_out, d_out_nz, d_work, pick(stream));
}

size_t plk_poly_mul_batch_workspace(const plk_polymul_job_t* jobs, int n) {
  // the size groups run one after another on the stream and reuse the workspace: the largest
  // group's need (jobs of one size 2^k take 2^(k+3) bytes each)
  size_t per_k[64] = {0}, best = 0;
  for (int i = 0; jobs && i < n; i++) {
    const size_t w = plk_poly_mul_workspace_bytes(jobs[i].la, jobs[i].lb);
    if (!w) continue;
    int k = 0;
    while (((size_t)8 << k) < w) k++;
    per_k[k] += w;
    best = per_k[k] > best ? per_k[k] : best;
  }
  return best;
}

int plk_poly_mul_batch_dev(const plk_polymul_job_t* jobs, int n, void* d_work, size_t work_bytes, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  if (!jobs || n < 1 || n > 64) {
    plk_set_error("plk_poly_mul_batch_dev: %d jobs (1..64)", n);
    return PLK_ERR_ARG;
  }
  PlkPolyMulJob js[64];
  for (int i = 0; i < n; i++) {
    if (!jobs[i].a || !jobs[i].b || !jobs[i].out) {
      plk_set_error("plk_poly_mul_batch_dev: null buffer in job %d", i);
      return PLK_ERR_ARG;
    }
    js[i] = PlkPolyMulJob{jobs[i].a, jobs[i].la, jobs[i].b, jobs[i].lb, jobs[i].out, jobs[i].acc ? 1 : 0};
  }
  return plk_poly_mul_batch_launch(js, n, d_work, work_bytes, pick(stream));
}

int plk_ntt_dev(uint32_t* d_data, int log_n, int inverse, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_ntt_launch(d_data, log_n, 1, inverse, pick(stream));
}

int plk_ntt_batch_dev(uint32_t* d_data, int log_n, int batch, int inverse, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  if (!d_data || batch < 1) {
    plk_set_error("plk_ntt_batch_dev: null data or batch %d", batch);
    return PLK_ERR_ARG;
  }
  return plk_ntt_launch(d_data, log_n, batch, inverse, pick(stream));
}

int plk_ntt29_dev(uint32_t* d_data, int log_n, int inverse, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  return plk_ntt29_launch(d_data, log_n, 1, inverse, pick(stream));
}

int plk_ntt29_batch_dev(uint32_t* d_data, int log_n, int batch, int inverse, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  if (!d_data || batch < 1) {
    plk_set_error("plk_ntt29_batch_dev: null data or batch %d", batch);
    return PLK_ERR_ARG;
  }
  return plk_ntt29_launch(d_data, log_n, batch, inverse, pick(stream));
}

// ---- the ops around the hot path -----------------------------------------
size_t plk_poly_eval_workspace(int n) { return (size_t)128 * (n > 0 ? n : 1); }

int plk_poly_eval_batch_dev(const uint8_t* const* d_polys, const size_t* lens, const uint8_t* xs, int n,
                            uint8_t* d_ys, void* d_tick, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  if (!d_polys || !lens || !xs || !d_ys || !d_tick || n < 1) {
    plk_set_error("plk_poly_eval_batch_dev: NULL argument or n = %d", n);
    return PLK_ERR_ARG;
  }
  for (int b = 0; b < n; b += PLK_EVAL_MAX_JOBS) {
    const int m = n - b < PLK_EVAL_MAX_JOBS ? n - b : PLK_EVAL_MAX_JOBS;
    uint64_t l64[PLK_EVAL_MAX_JOBS];
    for (int i = 0; i < m; i++) l64[i] = lens[b + i];
    if ((rc = plk_poly_eval_batch_launch(d_polys + b, l64, xs + b, m, d_ys + b,
                                         (uint8_t*)d_tick + (size_t)128 * b, pick(stream))))
      return rc;
  }
  return PLK_OK;
}

int plk_poly_eval_batch(const uint8_t* const* polys, const size_t* lens, const uint8_t* xs, int n, uint8_t* ys) {
  if (!polys || !lens || !xs || !ys || n < 1) {
    plk_set_error("plk_poly_eval_batch: NULL argument or n = %d", n);
    return PLK_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  Arena A;
  std::vector<size_t> off(n);
  for (int i = 0; i < n; i++) off[i] = A.take(lens[i] + 16);
  const size_t o_y = A.take(n);
  for (int i = 0; i < n; i++)
    if (lens[i] && !polys[i]) {
      plk_set_error("plk_poly_eval_batch: NULL polynomial %d", i);
      return PLK_ERR_ARG;
    }
  if (tiny_ok(A.off)) {   // toy sizes: no copies, one launch per 12 evaluations, one synchronize
    if (g.stage_busy) {
      PLK_HIP(hipStreamSynchronize(g.st));
      g.stage_busy = false;
    }
    uint8_t* tk;
    if ((rc = tick0(n, &tk))) return rc;
    std::vector<const uint8_t*> dp(n);
    for (int i = 0; i < n; i++) {
      if (lens[i]) memcpy(g.h_tiny + off[i], polys[i], lens[i]);
      dp[i] = g.d_tiny + off[i];
    }
    for (int b = 0; b < n; b += PLK_EVAL_MAX_JOBS) {
      const int m = n - b < PLK_EVAL_MAX_JOBS ? n - b : PLK_EVAL_MAX_JOBS;
      uint64_t l64[PLK_EVAL_MAX_JOBS];
      for (int i = 0; i < m; i++) l64[i] = lens[b + i];
      if ((rc = plk_poly_eval_batch_launch(dp.data() + b, l64, xs + b, m, g.d_tiny + o_y + b, tk + (size_t)128 * b,
                                           g.st)))
        return rc;
    }
    PLK_HIP(hipStreamSynchronize(g.st));
    memcpy(ys, g.h_tiny + o_y, n);
    return PLK_OK;
  }
  const size_t o_tick = A.take(plk_poly_eval_workspace(n));
  if ((rc = grow(&g.d_ops, &g.cap_ops, A.off))) return rc;
  std::vector<const uint8_t*> dp(n);
  Stage S;
  if ((rc = S.begin())) return rc;
  for (int i = 0; i < n; i++) {
    if (lens[i] && (rc = S.up(g.d_ops + off[i], polys[i], lens[i]))) return rc;
    dp[i] = g.d_ops + off[i];
  }
  PLK_HIP(hipMemsetAsync(g.d_ops + o_tick, 0, plk_poly_eval_workspace(n), g.st));
  for (int b = 0; b < n; b += PLK_EVAL_MAX_JOBS) {
    const int m = n - b < PLK_EVAL_MAX_JOBS ? n - b : PLK_EVAL_MAX_JOBS;
    uint64_t l64[PLK_EVAL_MAX_JOBS];
    for (int i = 0; i < m; i++) l64[i] = lens[b + i];
    if ((rc = plk_poly_eval_batch_launch(dp.data() + b, l64, xs + b, m, g.d_ops + o_y + b,
                                         g.d_ops + o_tick + (size_t)128 * b, g.st)))
      return rc;
  }
  if ((rc = S.down(ys, g.d_ops + o_y, n)) || (rc = S.finish())) return rc;
  return PLK_OK;
}

int plk_poly_eval(const uint8_t* p, size_t len, uint8_t x, uint8_t* y) {
  const uint8_t* ps[1] = {p};
  const size_t ls[1] = {len};
  return plk_poly_eval_batch(ps, ls, &x, 1, y);
}

size_t plk_poly_divide_workspace(size_t nl, size_t dl) { return plk_poly_divide_workspace_bytes(nl, dl); }

int plk_poly_divide_dev(const uint8_t* d_num, size_t nl, const uint8_t* den, size_t dl, uint8_t* d_quot,
                        uint8_t* d_rem, uint32_t* d_lens, void* d_work, void* stream) {
  int rc = ensure_dev();
  if (rc) return rc;
  if (!d_quot || !d_lens || !d_work || (dl > 1 && nl && !d_rem)) {
    plk_set_error("plk_poly_divide_dev: NULL buffer");
    return PLK_ERR_ARG;
  }
  return plk_poly_divide_launch(d_num, nl, den, dl, d_quot, d_rem, d_lens, d_work, pick(stream));
}

int plk_poly_divide(const uint8_t* num, size_t nl, const uint8_t* den, size_t dl, uint8_t* quot, size_t* quot_len,
                    uint8_t* rem, size_t* rem_len) {
  if (!quot || !quot_len || !rem_len || (nl && !num)) {
    plk_set_error("plk_poly_divide: NULL argument");
    return PLK_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  const size_t ql = nl >= dl ? nl - dl + 1 : 1;
  const size_t rl = dl ? (dl - 1 < nl ? dl - 1 : nl) : 0;
  if (rl && !rem) {
    plk_set_error("plk_poly_divide: NULL remainder buffer");
    return PLK_ERR_ARG;
  }
  Arena A;
  const size_t o_num = A.take(nl + 16), o_q = A.take(nl + 16), o_r = A.take(nl + 16), o_len = A.take(16),
               o_w = A.take(plk_poly_divide_workspace_bytes(nl, dl));
  if ((rc = grow(&g.d_ops, &g.cap_ops, A.off))) return rc;
  uint8_t* d = g.d_ops;
  Stage S;
  if ((rc = S.begin()) || (rc = S.up(d + o_num, num, nl))) return rc;
  if ((rc = plk_poly_divide_launch(d + o_num, nl, den, dl, d + o_q, d + o_r, (uint32_t*)(d + o_len), d + o_w, g.st)))
    return rc;
  uint32_t lens[2] = {0, 0};
  if ((rc = S.down(quot, d + o_q, ql)) || (rc = S.down(rem, d + o_r, rl)) ||
      (rc = S.down((uint8_t*)lens, d + o_len, 8)) || (rc = S.finish()))
    return rc;
  // poly_new's trim keeps one coefficient (src/poly.h:21-24); a zero-length remainder stays empty
  *quot_len = lens[0] ? lens[0] : 1;
  *rem_len = rl ? (lens[1] ? lens[1] : 1) : 0;
  return PLK_OK;
}

int plk_matrix_mul(const uint8_t* a, size_t m, size_t k, const uint8_t* b, size_t n, uint8_t* out) {
  if ((m * k && !a) || (k * n && !b) || (m * n && !out)) {
    plk_set_error("plk_matrix_mul: NULL argument");
    return PLK_ERR_ARG;
  }
  if (!m || !n) return PLK_OK;
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  Arena A;
  const size_t o_a = A.take(m * k), o_b = A.take(k * n), o_o = A.take(m * n);
  if ((rc = grow(&g.d_ops, &g.cap_ops, A.off))) return rc;
  uint8_t* d = g.d_ops;
  Stage S;
  if ((rc = S.begin()) || (rc = S.up(d + o_a, a, m * k)) || (rc = S.up(d + o_b, b, k * n))) return rc;
  if ((rc = plk_matrix_mul_launch(d + o_a, m, k, d + o_b, n, d + o_o, g.st))) return rc;
  if ((rc = S.down(out, d + o_o, m * n)) || (rc = S.finish())) return rc;
  return PLK_OK;
}

int plk_matrix_inv(const uint8_t* mat, size_t n, uint8_t* out) {
  if (n && (!mat || !out)) {
    plk_set_error("plk_matrix_inv: NULL argument");
    return PLK_ERR_ARG;
  }
  for (size_t i = 0; i < n * n; i++)
    if (mat[i] >= 17) {   // hf_div of a raw pivot reads hf_inverses out of bounds in the reference
      plk_set_error("plk_matrix_inv: entry %zu = %u is not a GF(17) value (reference behaviour undefined)", i,
                    (unsigned)mat[i]);
      return PLK_ERR_RANGE;
    }
  if (!n) return PLK_OK;
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  Arena A;
  const size_t o_m = A.take(n * n), o_aug = A.take(2 * n * n), o_o = A.take(n * n);
  if ((rc = grow(&g.d_ops, &g.cap_ops, A.off))) return rc;
  uint8_t* d = g.d_ops;
  Stage S;
  if ((rc = S.begin()) || (rc = S.up(d + o_m, mat, n * n))) return rc;
  if ((rc = plk_matrix_inv_launch(d + o_m, n, d + o_aug, d + o_o, g.st))) return rc;
  if ((rc = S.down(out, d + o_o, n * n)) || (rc = S.finish())) return rc;
  return PLK_OK;
}

int plk_interpolate(const uint8_t* h_pows_inv, const uint8_t* values, size_t n, uint8_t* out, size_t* out_len) {
  if (!out_len || (n && (!h_pows_inv || !values || !out))) {
    plk_set_error("plk_interpolate: NULL argument");
    return PLK_ERR_ARG;
  }
  if (!n) {
    *out_len = 0;
    return PLK_OK;
  }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure_locked();
  if (rc) return rc;
  Arena A;
  const size_t o_m = A.take(n * n), o_v = A.take(n), o_o = A.take(n), o_len = A.take(16);
  if ((rc = grow(&g.d_ops, &g.cap_ops, A.off))) return rc;
  uint8_t* d = g.d_ops;
  Stage S;
  if ((rc = S.begin()) || (rc = S.up(d + o_m, h_pows_inv, n * n)) || (rc = S.up(d + o_v, values, n))) return rc;
  if ((rc = plk_matrix_mul_launch(d + o_m, n, n, d + o_v, 1, d + o_o, g.st))) return rc;
  if ((rc = plk_trim_launch(d + o_o, n, (uint32_t*)(d + o_len), g.st))) return rc;
  uint32_t nz = 0;
  if ((rc = S.down(out, d + o_o, n)) || (rc = S.down((uint8_t*)&nz, d + o_len, 4)) || (rc = S.finish())) return rc;
  *out_len = nz ? nz : 1;
  return PLK_OK;
}

}  // extern "C"
