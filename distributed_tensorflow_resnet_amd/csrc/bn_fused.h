// In-kernel BatchNorm finalize by the last-arriving workgroup.
//
// A conv (STATS) or dgrad (BNB) launch writes per-tile partials; instead of a
// separate finalize launch, every workgroup of one column tile announces its
// partial with write-through (sc1) stores, drains them (s_waitcnt vmcnt(0) in
// every storing wave, then a workgroup barrier) and takes a relaxed agent-scope
// atomic ticket -- no release fence: an agent release is `buffer_wbl2`, which
// writes back the whole XCD L2 including the conv tile just stored (measured:
// 35 % slower CIFAR step).  cdna_hip_programming.md §6 Guideline 16, R1 with a
// counter as the flag.  The workgroup that draws
// the last ticket acquires, combines all tiles in a fixed order (bitwise
// deterministic: placement changes only WHO combines, not the order) and
// writes the BN outputs.  It then resets the counter for the next launch
// (counters start zeroed at allocation).
#pragma once
#include "common.h"

namespace dtr {

// Partial tiles per combining thread in the last arriver (the host enables the
// fused finalize only when ceil(tiles / (256 / BN)) <= FIN_UNROLL, so every
// partial is loaded in one round trip).
constexpr int FIN_UNROLL = 8;

// Write-through (sc1) store of one handed-off float.
__device__ __forceinline__ void publish_f32(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Returns (block-uniformly) whether this workgroup is the last of `total`
// arrivals on *cnt.  Call after this workgroup's partial stores.
__device__ __forceinline__ bool last_arriver(unsigned* cnt, unsigned total, int* smem_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {   // partials were stored sc1 and drained: no release fence
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    *smem_flag = (prev == total - 1) ? 1 : 0;
  }
  __syncthreads();
  const bool last = *smem_flag != 0;
  if (last) {
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  return last;
}

__device__ __forceinline__ void reset_counter(unsigned* cnt) {
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dtr
