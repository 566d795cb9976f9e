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
template <int NT>
__device__ __forceinline__ bool msm_finish(uint32_t acc, bool bad, PlkMsmResult* res, uint32_t* wsum, uint32_t* wbad,
                                           const uint32_t* etab) {
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
  const uint32_t X = gridDim.x;
  unsigned long long add =
      (unsigned long long)(bs % PLK_GROUP_ORDER) | (1ull << 32) | ((unsigned long long)(bb_ != 0) << 48);
  {
    const uint32_t lin = blockIdx.y * X + blockIdx.x;
    const uint32_t sh = lin % PLK_MSM_SHARDS;
    // blocks of this MSM in shard sh: x in [0, X) with (y X + x) = sh (mod 8)
    const uint32_t r = (sh + PLK_MSM_SHARDS - (blockIdx.y * X) % PLK_MSM_SHARDS) % PLK_MSM_SHARDS;
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
