// The ticketed in-launch finish shared by the MSM kernels (msm.hip) and the prover's fused
// commitment kernel (prove.hip).
#pragma once
#include "plk_device.h"
#include "plk_internal.h"

#ifndef PLK_MSM_DIAG
#define PLK_MSM_DIAG 0
#endif

// Finish of one block of an MSM launch (msm_dlog_kernel, msm_log_kernel, the prover's
// commit_pack_kernel): the block's log sum and irregular flag go to record res with the ticketed
// atomics described at msm_dlog_kernel.  true for the one thread that completed the record.
// (x, X, y: the block's index among the record's X blocks and the record's index, which spread the
// shard words; a kernel whose grid is one MSM per row passes blockIdx.x, gridDim.x, blockIdx.y)
template <int NT>
__device__ __forceinline__ bool msm_finish_xy(uint32_t acc, bool bad, PlkMsmResult* res, uint32_t* wsum,
                                              uint32_t* wbad, const uint32_t* etab, uint32_t x, uint32_t X,
                                              uint32_t y) {
  const uint32_t wave = threadIdx.x / PLK_WAVE;
  const uint32_t s = plk_wave_sum(acc);
  const uint64_t anybad = __ballot(bad);
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) {
    wsum[wave] = s;
    wbad[wave] = anybad != 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return false;
  uint32_t bs = 0, bb_ = 0;
#pragma unroll
  for (int k = 0; k < NT / PLK_WAVE; k++) {
    bs += wsum[k];
    bb_ |= wbad[k];
  }
  if (PLK_MSM_DIAG & 2) {
    res->pad[blockIdx.x % 11] = bs + bb_;
    return false;
  }
  unsigned long long add =
      (unsigned long long)(bs % PLK_GROUP_ORDER) | (1ull << 32) | ((unsigned long long)(bb_ != 0) << 48);
  {
    const uint32_t lin = y * X + x;
    const uint32_t sh = lin % PLK_MSM_SHARDS;
    // blocks of this MSM in shard sh: x in [0, X) with (y X + x) = sh (mod PLK_MSM_SHARDS)
    const uint32_t r = (sh + PLK_MSM_SHARDS - (y * X) % PLK_MSM_SHARDS) % PLK_MSM_SHARDS;
    const uint32_t in_shard = r < X ? (X - r + PLK_MSM_SHARDS - 1) / PLK_MSM_SHARDS : 0u;
    unsigned long long* word = reinterpret_cast<unsigned long long*>(&res->shard[sh][0]);
    const unsigned long long old = atomicAdd(word, add);
    if (((old >> 32) & 0xFFFFull) != in_shard - 1) return false;
    const unsigned long long tot = old + add;
    atomicExch(word, 0ull);
    add = (unsigned long long)((uint32_t)(tot & 0xFFFFFFFFull) % PLK_GROUP_ORDER) | (1ull << 32) |
          ((unsigned long long)((tot >> 48) != 0) << 48);
  }
  const uint32_t arrivals = X < PLK_MSM_SHARDS ? X : PLK_MSM_SHARDS;   // shards with blocks
  const unsigned long long old = atomicAdd(&res->top, add);
  if (((old >> 32) & 0xFFFFull) != arrivals - 1) return false;
  const unsigned long long tot = old + add;
  const uint32_t lg = (uint32_t)(tot & 0xFFFFFFFFull) % PLK_GROUP_ORDER;
  res->log = lg;
  res->irregular = (uint32_t)(tot >> 48);
  *reinterpret_cast<uint32_t*>(res->g1) = etab[lg];
  atomicExch(&res->top, 0ull);
  return true;
}
template <int NT>
__device__ __forceinline__ bool msm_finish(uint32_t acc, bool bad, PlkMsmResult* res, uint32_t* wsum, uint32_t* wbad,
                                           const uint32_t* etab) {
  return msm_finish_xy<NT>(acc, bad, res, wsum, wbad, etab, blockIdx.x, gridDim.x, blockIdx.y);
}

// Block x of X of a log-form MSM over n points (logs: one byte per point, msm.hip's srs_log_kernel;
// sc: the scalars; both 16-byte aligned), record res, row index y (shard spread): 16-point groups
// with the stride X NT, the n mod 16 tail in block 0, then the ticketed finish.  etab (LDS, 102
// words) is staged here; wsum / wbad are the finish's LDS words.  true for the thread that
// completed the record.
template <int NT>
__device__ __forceinline__ bool msm_log_block(const uint8_t* logs, const uint8_t* sc, uint64_t n, uint32_t x,
                                              uint32_t X, uint32_t y, PlkMsmResult* res, const uint32_t* exp_words,
                                              uint32_t* etab, uint32_t* wsum, uint32_t* wbad) {
  if (threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = exp_words[threadIdx.x];
  const uint64_t stride = (uint64_t)X * NT;
  const uint64_t ngroups = n >> 4;
  const uint4* l4 = reinterpret_cast<const uint4*>(logs);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  uint32_t acc = 0;
  for (uint64_t g = (uint64_t)x * NT + threadIdx.x; g < ngroups; g += stride) {
    const uint4 l = l4[g], s = s4[g];
    uint32_t t = __builtin_amdgcn_udot4(l.x, s.x, 0u, false);   // 16 x 101 x 255 < 2^19
    t = __builtin_amdgcn_udot4(l.y, s.y, t, false);
    t = __builtin_amdgcn_udot4(l.z, s.z, t, false);
    t = __builtin_amdgcn_udot4(l.w, s.w, t, false);
    acc += t % PLK_GROUP_ORDER;
  }
  const uint64_t base = ngroups << 4;
  if (x == 0 && base + threadIdx.x < n) acc += (uint32_t)logs[base + threadIdx.x] * sc[base + threadIdx.x];
  return msm_finish_xy<NT>(acc % PLK_GROUP_ORDER, false, res, wsum, wbad, etab, x, X, y);
}
