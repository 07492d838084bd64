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
#include "kernels.h"

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

// Consumer-side finalize (BnPreFin, kernels.h): all 256 threads combine the
// producer's partials for C channels (C a power of two <= 256; thread = (channel
// c = tid % C, slice q = tid / C), items q, q + G, ... with G = 256 / C, at most
// FIN_UNROLL each -- one round of loads), fold the G slices in fixed order and
// write the BN scale/shift table sc_s/sh_s (LDS).  Block (0,0) also writes the
// global mean/rstd/scale/shift and the moving averages.  `scratch` = 768 LDS
// floats.  Ends with a barrier (the table is ready for every thread).
__device__ __forceinline__ void bn_prefin_table(const BnPreFin& P, int C, float* sc_s,
                                                float* sh_s, float* scratch) {
  const int tid = threadIdx.x;
  const int G = 256 / C;
  const int c = tid % C, q = tid / C;
  // Division-free parallel combine about a common centre (Chan et al.): for items
  // (n_i, mean_i, M2_i): N = sum n_i, mean = sum n_i mean_i / N,
  // M2 = sum M2_i + sum n_i (mean_i - mean)^2 -- two passes over the registers
  // instead of one dependent division per item (sequential Welford).
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (q < G) {
    float mv[FIN_UNROLL], qv[FIN_UNROLL], nv[FIN_UNROLL];
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const int t = q + u * G;
      const bool ok = t < P.cnt;
      mv[u] = ok ? P.part[(long)t * 2 * C + c] : 0.f;
      qv[u] = ok ? P.part[(long)t * 2 * C + C + c] : 0.f;
      nv[u] = ok ? (float)min(P.rows_per, P.M - t * P.rows_per) : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      n += nv[u];
      s += nv[u] * mv[u];
    }
    mu = n > 0.f ? s / n : 0.f;
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const float d = mv[u] - mu;
      m2 += qv[u] + nv[u] * d * d;
    }
    scratch[tid] = n;
    scratch[256 + tid] = mu;
    scratch[512 + tid] = m2;
  }
  __syncthreads();
  if (q == 0) {
    float fn_ = 0.f, s = 0.f;
    for (int k = 0; k < G; ++k) {
      fn_ += scratch[k * C + c];
      s += scratch[k * C + c] * scratch[256 + k * C + c];
    }
    const float fmu = s / fn_;
    float fm2 = 0.f;
    for (int k = 0; k < G; ++k) {
      const float d = scratch[256 + k * C + c] - fmu;
      fm2 += scratch[512 + k * C + c] + scratch[k * C + c] * d * d;
    }
    const float rs = rsqrtf(fm2 / fn_ + P.eps);
    const float sc = P.gamma[c] * rs;
    const float sh = P.beta[c] - fmu * sc;
    sc_s[c] = sc;
    sh_s[c] = sh;
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      P.mean[c] = fmu;
      P.rstd[c] = rs;
      P.scale[c] = sc;
      P.shift[c] = sh;
      if (P.update_moving) {
        const float uvar = fn_ > 1.f ? fm2 / (fn_ - 1.f) : fm2;
        P.mmean[c] -= (1.f - P.momentum) * (P.mmean[c] - fmu);
        P.mvar[c] -= (1.f - P.momentum) * (P.mvar[c] - uvar);
      }
    }
  }
  __syncthreads();
}

}  // namespace dtr
