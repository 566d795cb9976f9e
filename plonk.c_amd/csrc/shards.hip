// In-process multi-device MSM for the host-buffer entry point plk_msm_g1 (SURVEY 8(b)
// plk_init(n_gpus), 8(e) point-range sharding; the reference caller is srs_eval_at_s,
// src/srs.h:53-68, reached from plonk_prove at src/plonk.h:299-301, 379, 522-524, 620-621).
//
// plk_init_devices(ids, n) gives the library a list of shards, one per entry (a device may
// appear more than once: several shards on one GPU, which is how a one-GPU box rehearses the
// N-device path).  An MSM of n points is split into contiguous point ranges (the same
// shard_range as plonkhip/dist.py); shard s uploads its range over its own device's PCIe link
// from its own host thread, runs the single-pass dlog kernel on its own stream and returns
// (partial log, irregular count).  The exchange is the SUM of those N 4-byte partials mod 102,
// done on the host: the result goes to the host anyway (plk_msm_g1 returns 3 bytes), every
// shard's record is already read back with its own stream's synchronize, and a collective (a
// single-process RCCL communicator) would add a launch and a second synchronisation per device
// for 4 bytes -- and RCCL refuses a communicator that names one GPU twice, which the rehearsal
// needs.  The device-resident multi-GPU path (one process per GPU, plonkhip/dist.py) keeps its
// RCCL all-reduce.
//
// Each shard caches the SRS points it has uploaded, keyed by the caller's pointer: a device
// copy and a host mirror indexed by absolute point position, valid over [c_lo, c_hi).  A later
// call whose range overlaps or touches that interval re-uses it after an exact memcmp of the
// overlap, uploading only the missing ends -- the 9 commitments of a proof have lengths n+2 /
// n+3 whose shard boundaries differ by a point or two.
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "plk_device.h"
#include "plk_internal.h"

namespace {

constexpr size_t CHUNK = 4u << 20;   // pinned staging: two halves of this size per shard

struct Shard {
  int dev = -1;
  hipStream_t st = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool busy[2] = {false, false};   // a staged copy out of that half may still be in flight
  int next = 0;                    // the half the next staged copy uses
  uint8_t* d_pts = nullptr;     // absolute layout: point i at 3 i
  size_t cap_pts = 0;
  uint8_t* mirror = nullptr;    // host copy of the cached bytes, same layout
  size_t cap_mirror = 0;
  const uint8_t* key = nullptr;
  size_t c_lo = 0, c_hi = 0;    // cached point interval
  uint8_t* d_sc = nullptr;
  size_t cap_sc = 0;
  PlkMsmResult* d_res = nullptr;
  uint8_t* h_stage = nullptr;   // pinned, 2 * CHUNK
  PlkMsmResult* h_res = nullptr;  // pinned
  // this call's job and answer
  size_t lo = 0, hi = 0;
  int rc = 0;
  std::string err;
  uint32_t log = 0, irregular = 0;
};

struct Pool {
  std::vector<Shard> sh;
  std::vector<std::thread> th;   // th[s - 1] runs shard s; the caller's thread runs shard 0
  std::mutex m;
  std::condition_variable go, done;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
  const uint8_t* pts = nullptr;
  const uint8_t* sc = nullptr;
  bool lanes = false;   // host lanes of the one primary device (not a plk_init_devices list)
  // a program that exits without plk_shutdown (the reference's own test programs through the
  // drop-in): the idle workers are released and joined here -- no HIP call, the runtime may be
  // gone already -- instead of std::thread's terminate on a joinable thread
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
    }
    go.notify_all();
    for (auto& t : th)
      if (t.joinable()) t.join();
  }
} P;

int dgrow(uint8_t** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return PLK_OK;
  size_t n = *cap ? *cap : 65536;
  while (n < need) n *= 2;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  PLK_HIP(hipMalloc((void**)p, n));
  *cap = n;
  return PLK_OK;
}

// host -> device through this shard's two pinned halves (alternating across calls, each
// refilled only after its previous copy completed); ordered on the shard's stream
int up(Shard& s, uint8_t* dst, const uint8_t* src, size_t bytes) {
  for (size_t off = 0; off < bytes; off += CHUNK) {
    const size_t len = bytes - off < CHUNK ? bytes - off : CHUNK;
    const int k = s.next;
    s.next ^= 1;
    if (s.busy[k]) PLK_HIP(hipEventSynchronize(s.ev[k]));
    memcpy(s.h_stage + k * CHUNK, src + off, len);
    PLK_HIP(hipMemcpyAsync(dst + off, s.h_stage + k * CHUNK, len, hipMemcpyHostToDevice, s.st));
    PLK_HIP(hipEventRecord(s.ev[k], s.st));
    s.busy[k] = true;
  }
  return PLK_OK;
}

// the points [lo, hi) resident on the shard's device (cache, see the header)
int ensure_points(Shard& s, const uint8_t* pts, size_t lo, size_t hi) {
  const bool same = s.key == pts && s.c_hi > s.c_lo && lo <= s.c_hi && hi >= s.c_lo;
  if (same) {
    const size_t ol = lo > s.c_lo ? lo : s.c_lo, oh = hi < s.c_hi ? hi : s.c_hi;
    if (memcmp(pts + 3 * ol, s.mirror + 3 * ol, 3 * (oh - ol)) == 0 && 3 * hi <= s.cap_pts &&
        3 * hi <= s.cap_mirror) {
      int rc;
      if (lo < s.c_lo) {
        if ((rc = up(s, s.d_pts + 3 * lo, pts + 3 * lo, 3 * (s.c_lo - lo)))) return rc;
        memcpy(s.mirror + 3 * lo, pts + 3 * lo, 3 * (s.c_lo - lo));
        s.c_lo = lo;
      }
      if (hi > s.c_hi) {
        if ((rc = up(s, s.d_pts + 3 * s.c_hi, pts + 3 * s.c_hi, 3 * (hi - s.c_hi)))) return rc;
        memcpy(s.mirror + 3 * s.c_hi, pts + 3 * s.c_hi, 3 * (hi - s.c_hi));
        s.c_hi = hi;
      }
      return PLK_OK;
    }
  }
  s.key = nullptr;   // invalid until this upload is enqueued
  s.c_lo = s.c_hi = 0;
  int rc = dgrow(&s.d_pts, &s.cap_pts, 3 * hi + 16);
  if (rc) return rc;
  if (s.cap_mirror < 3 * hi) {
    free(s.mirror);
    s.cap_mirror = 3 * hi + (3 * hi >> 3);
    s.mirror = (uint8_t*)malloc(s.cap_mirror);
    if (!s.mirror) {
      s.cap_mirror = 0;
      plk_set_error("shard mirror: host allocation of %zu bytes failed", 3 * hi);
      return PLK_ERR_NOMEM;
    }
  }
  if ((rc = up(s, s.d_pts + 3 * lo, pts + 3 * lo, 3 * (hi - lo)))) return rc;
  memcpy(s.mirror + 3 * lo, pts + 3 * lo, 3 * (hi - lo));
  s.key = pts;
  s.c_lo = lo;
  s.c_hi = hi;
  return PLK_OK;
}

int run_shard_body(Shard& s, const uint8_t* pts, const uint8_t* sc) {
  PLK_HIP(hipSetDevice(s.dev));
  const size_t m = s.hi - s.lo;
  int rc;
  if ((rc = ensure_points(s, pts, s.lo, s.hi))) return rc;
  if ((rc = dgrow(&s.d_sc, &s.cap_sc, m + 16))) return rc;
  if ((rc = up(s, s.d_sc, sc + s.lo, m))) return rc;
  if ((rc = plk_msm_launch(s.d_pts + 3 * s.lo, s.d_sc, m, s.d_res, s.st))) return rc;
  PLK_HIP(hipMemcpyAsync(s.h_res, s.d_res, 32, hipMemcpyDeviceToHost, s.st));
  PLK_HIP(hipStreamSynchronize(s.st));
  s.busy[0] = s.busy[1] = false;
  s.log = s.h_res->log;
  s.irregular = s.h_res->irregular;
  return PLK_OK;
}

void run_shard(Shard& s, const uint8_t* pts, const uint8_t* sc) {
  s.log = s.irregular = 0;
  s.err.clear();
  s.rc = s.hi > s.lo ? run_shard_body(s, pts, sc) : PLK_OK;
  if (s.rc) {
    s.err = plk_last_error();   // (the error text is thread-local)
    if (s.st) (void)hipStreamSynchronize(s.st);   // nothing of this call left in flight
    s.busy[0] = s.busy[1] = false;
    s.key = nullptr;                              // the cache state is unknown after a failure
    s.c_lo = s.c_hi = 0;
  }
}

void worker(int idx) {
  uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(P.m);
      P.go.wait(lk, [&] { return P.stop || P.gen != seen; });
      if (P.stop) return;
      seen = P.gen;
    }
    run_shard(P.sh[idx], P.pts, P.sc);
    std::lock_guard<std::mutex> lk(P.m);
    if (--P.pending == 0) P.done.notify_one();
  }
}

void free_shard(Shard& s) {
  if (s.dev >= 0) {
    (void)hipSetDevice(s.dev);
    if (s.st) (void)hipStreamSynchronize(s.st);
  }
  (void)hipFree(s.d_pts);
  (void)hipFree(s.d_sc);
  (void)hipFree(s.d_res);
  if (s.h_stage) (void)hipHostFree(s.h_stage);
  if (s.h_res) (void)hipHostFree(s.h_res);
  for (hipEvent_t e : s.ev)
    if (e) (void)hipEventDestroy(e);
  if (s.st) (void)hipStreamDestroy(s.st);
  free(s.mirror);
  s = Shard{};
}

}  // namespace

// caller holds the library lock; tables = the dlog / EXP / inverse tables plk_init built
void plk_shards_teardown(void) {
  {
    std::lock_guard<std::mutex> lk(P.m);
    P.stop = true;
  }
  P.go.notify_all();
  for (auto& t : P.th) t.join();
  P.th.clear();
  for (auto& s : P.sh) free_shard(s);
  P.sh.clear();
  P.stop = false;
  P.pending = 0;
  P.lanes = false;
}

int plk_shards_setup(const int* ids, int n, const uint32_t* ytab, const uint8_t* exp4, const uint8_t* inv101,
                     bool lanes) {
  plk_shards_teardown();
  P.lanes = false;
  if (n <= 1) return PLK_OK;   // one device: the single-device path, no shards
  int prev = -1;
  (void)hipGetDevice(&prev);
  std::vector<int> loaded;
  P.sh.resize(n);
  int rc = PLK_OK;
  for (int i = 0; i < n && !rc; i++) {
    Shard& s = P.sh[i];
    s.dev = ids[i];
    auto fail = [&](hipError_t e, const char* what) {
      plk_set_error("shard %d (device %d): %s: %s", i, s.dev, what, hipGetErrorString(e));
      return PLK_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(s.dev)) != hipSuccess) { rc = fail(e, "hipSetDevice"); break; }
    bool have = false;
    for (int d : loaded) have |= d == s.dev;
    if (!have) {   // the kernels' __constant__ tables exist per device
      if ((rc = plk_msm_upload_tables(ytab, exp4, inv101))) break;
      loaded.push_back(s.dev);
    }
    if ((e = hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking)) != hipSuccess) { rc = fail(e, "stream"); break; }
    for (hipEvent_t& ev : s.ev)
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) { rc = fail(e, "event"); break; }
    if (rc) break;
    if ((e = hipMalloc((void**)&s.d_res, sizeof(PlkMsmResult))) != hipSuccess ||
        (e = hipMemset(s.d_res, 0, sizeof(PlkMsmResult))) != hipSuccess) { rc = fail(e, "result record"); break; }
    if ((e = hipHostMalloc((void**)&s.h_stage, 2 * CHUNK, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_res, sizeof(PlkMsmResult), hipHostMallocDefault)) != hipSuccess) {
      rc = fail(e, "pinned staging");
      break;
    }
  }
  if (!rc) {
    P.gen = 0;
    P.lanes = lanes;
    for (int i = 1; i < n; i++) P.th.emplace_back(worker, i);
  } else {
    for (auto& s : P.sh) free_shard(s);
    P.sh.clear();
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return rc;
}

int plk_shards_count(void) { return (int)P.sh.size(); }
bool plk_shards_are_lanes(void) { return P.lanes; }

int plk_shards_devices(int* ids, int cap) {
  const int n = (int)P.sh.size();
  for (int i = 0; i < n && i < cap; i++) ids[i] = P.sh[i].dev;
  return n;
}

// One MSM over the shards: *log_sum = sum of the partial logs (not reduced), *irregular = sum
// of the irregular counts.  Caller holds the library lock (one call at a time).
int plk_shards_msm(const uint8_t* pts, const uint8_t* sc, size_t n, uint64_t* log_sum, uint64_t* irregular) {
  const int ns = (int)P.sh.size();
  if (ns < 2) {
    plk_set_error("plk_shards_msm: no shards");
    return PLK_ERR_ARG;
  }
  const size_t base = n / ns, extra = n % ns;
  for (int i = 0; i < ns; i++) {   // shard_range (plonkhip/dist.py)
    P.sh[i].lo = i * base + (i < (int)extra ? i : extra);
    P.sh[i].hi = P.sh[i].lo + base + (i < (int)extra ? 1 : 0);
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  {
    std::lock_guard<std::mutex> lk(P.m);
    P.pts = pts;
    P.sc = sc;
    P.pending = ns - 1;
    P.gen++;
  }
  P.go.notify_all();
  run_shard(P.sh[0], pts, sc);
  {
    std::unique_lock<std::mutex> lk(P.m);
    P.done.wait(lk, [] { return P.pending == 0; });
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  uint64_t ls = 0, irr = 0;
  for (int i = 0; i < ns; i++) {
    const Shard& s = P.sh[i];
    if (s.rc) {
      plk_set_error("shard %d (device %d): %s", i, s.dev, s.err.c_str());
      return s.rc;
    }
    ls += s.log;
    irr += s.irregular;
  }
  *log_sum = ls;
  *irregular = irr;
  return PLK_OK;
}
