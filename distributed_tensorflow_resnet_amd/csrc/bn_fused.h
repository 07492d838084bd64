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

// Consumer-side finalize (BnPreFin, kernels.h): the 256 threads of the BN's first
// consuming conv combine the producer's per-tile partials [cnt][2][C] (mean, M2)
// themselves -- no finalize launch between the two convs.  Thread = (channel
// group of 4 = one 16-B load, tile slice q); slice q holds tiles q, q + G, ...
// (G = 1024 / C), PFIN_ITEMS per round with all loads of a round in flight.
// Per round a division-free Chan fold about the round mean, then pairwise Chan
// combines: xor-shuffles across the slices inside a wave, one fixed-order LDS
// pass across the 4 waves -- bitwise deterministic.  Writes the BN scale/shift
// table sc_s/sh_s (LDS); block (0,0) also writes the global mean/rstd/scale/
// shift and the moving averages.  `scratch` >= 12*C LDS floats (>= 768 for
// C <= 64).  C: multiple of 4 with C/4 a power of two <= 64.  Ends with a barrier.
constexpr int PFIN_ITEMS = 8;
constexpr int PFIN_ROUNDS = 2;   // the host keeps cnt <= PFIN_ITEMS*PFIN_ROUNDS*1024/C

__device__ __forceinline__ void chan_merge(float& n, float& mu, float& m2, float nb, float mub,
                                           float m2b) {
  const float nn = n + nb;
  if (nn <= 0.f) return;
  const float d = mub - mu, fb = nb / nn;
  mu += d * fb;
  m2 += m2b + d * d * n * fb;
  n = nn;
}

// fp64 accumulator replicas [BN_ACC_REP][2][C] -> the channel's two sums, replicas
// added in a fixed order (the per-replica atomic sums of fp32 tile partials are
// exact in fp64 while the partials' magnitudes stay within ~2^20 of each other).
__device__ __forceinline__ void bn_acc_sums(const double* __restrict__ acc, int C, int c,
                                            double& s1, double& s2) {
  double a[BN_ACC_REP], b[BN_ACC_REP];
#pragma unroll
  for (int r = 0; r < BN_ACC_REP; ++r) {
    a[r] = acc[(long)r * 2 * C + c];
    b[r] = acc[(long)r * 2 * C + C + c];
  }
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll
  for (int r = 0; r < BN_ACC_REP; ++r) {
    s1 += a[r];
    s2 += b[r];
  }
}

// Adds one tile's per-column sums to its replica (memory-side fp64 atomics, no return).
__device__ __forceinline__ void bn_acc_add(double* acc, int C, int col, double v1, double v2) {
  double* p = acc + (long)(blockIdx.x % BN_ACC_REP) * 2 * C + col;
  unsafeAtomicAdd(p, v1);
  unsafeAtomicAdd(p + C, v2);
}

__device__ __forceinline__ void bn_prefin_table(const BnPreFin& P, int C, float* sc_s,
                                                float* sh_s, float* scratch) {
  const int tid = threadIdx.x;
  if (P.acc != nullptr) {   // accumulator mode: sum y, sum y^2 of all M rows (any C)
    for (int c = tid; c < C; c += blockDim.x) {
      const float gam = P.gamma[c], bet = P.beta[c];
      double s1, s2;
      bn_acc_sums(P.acc, C, c, s1, s2);
      const double dm = s1 / (double)P.M;
      const double var = fmax(s2 / (double)P.M - dm * dm, 0.0);
      const float fmu = (float)dm, fvar = (float)var;
      const float rs = rsqrtf(fvar + P.eps);
      const float sc = gam * rs;
      const float sh = bet - fmu * sc;
      sc_s[c] = sc;
      sh_s[c] = sh;
      if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
        P.mean[c] = fmu;
        P.rstd[c] = rs;
        P.scale[c] = sc;
        P.shift[c] = sh;
        if (P.update_moving) {
          const float uvar = P.M > 1 ? (float)(var * P.M / (P.M - 1.0)) : fvar;
          const float mmv = P.mmean[c], mvv = P.mvar[c];
          P.mmean[c] = mmv - (1.f - P.momentum) * (mmv - fmu);
          P.mvar[c] = mvv - (1.f - P.momentum) * (mvv - uvar);
        }
      }
    }
    __syncthreads();
    return;
  }
  const int CG = C >> 2, cg = tid & (CG - 1), q = tid / CG, G = 256 / CG;
  float gam = 0.f, bet = 0.f, mmv = 0.f, mvv = 0.f;   // issued ahead of the partials
  if (tid < C) {
    gam = P.gamma[tid];
    bet = P.beta[tid];
    if (P.update_moving && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      mmv = P.mmean[tid];
      mvv = P.mvar[tid];
    }
  }
  float n = 0.f, mu[4] = {0.f, 0.f, 0.f, 0.f}, m2[4] = {0.f, 0.f, 0.f, 0.f};
  for (int base = q; base < P.cnt; base += PFIN_ITEMS * G) {
    f32x4 mv[PFIN_ITEMS], qv[PFIN_ITEMS];
    float nv[PFIN_ITEMS];
#pragma unroll
    for (int u = 0; u < PFIN_ITEMS; ++u) {
      const int t = base + u * G;
      const bool ok = t < P.cnt;
      const float* row = P.part + (long)t * 2 * C + 4 * cg;
      mv[u] = ok ? *reinterpret_cast<const f32x4*>(row) : f32x4{0.f, 0.f, 0.f, 0.f};
      qv[u] = ok ? *reinterpret_cast<const f32x4*>(row + C) : f32x4{0.f, 0.f, 0.f, 0.f};
      nv[u] = ok ? (float)min(P.rows_per, P.M - t * P.rows_per) : 0.f;
    }
    float nr = 0.f;
#pragma unroll
    for (int u = 0; u < PFIN_ITEMS; ++u) nr += nv[u];
    const float inv = nr > 0.f ? 1.f / nr : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sx = 0.f;
#pragma unroll
      for (int u = 0; u < PFIN_ITEMS; ++u) sx += nv[u] * mv[u][j];
      const float mr = sx * inv;
      float q2 = 0.f;
#pragma unroll
      for (int u = 0; u < PFIN_ITEMS; ++u) {
        const float d = mv[u][j] - mr;
        q2 += qv[u][j] + nv[u] * d * d;
      }
      float nn = n;
      chan_merge(nn, mu[j], m2[j], nr, mr, q2);
      if (j == 3) n = nn;
    }
  }
  // slices inside the wave (lanes cg + CG*k), then across the 4 waves
  for (int o = CG; o < 64; o <<= 1) {
    const float nb = __shfl_xor(n, o, 64);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float mub = __shfl_xor(mu[j], o, 64), m2b = __shfl_xor(m2[j], o, 64);
      float nn = n;
      chan_merge(nn, mu[j], m2[j], nb, mub, m2b);
      if (j == 3) n = nn;
    }
  }
  const int wave = tid >> 6, lane = tid & 63;
  if (lane < CG) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      scratch[(wave * 3 + 0) * C + 4 * lane + j] = n;
      scratch[(wave * 3 + 1) * C + 4 * lane + j] = mu[j];
      scratch[(wave * 3 + 2) * C + 4 * lane + j] = m2[j];
    }
  }
  __syncthreads();
  if (tid < C) {
    const int c = tid;
    float fn_ = scratch[c], fmu = scratch[C + c], fm2 = scratch[2 * C + c];
    for (int k = 1; k < 4; ++k)
      chan_merge(fn_, fmu, fm2, scratch[(k * 3) * C + c], scratch[(k * 3 + 1) * C + c],
                 scratch[(k * 3 + 2) * C + c]);
    const float rs = rsqrtf(fm2 / fn_ + P.eps);
    const float sc = gam * rs;
    const float sh = bet - fmu * sc;
    sc_s[c] = sc;
    sh_s[c] = sh;
    if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      P.mean[c] = fmu;
      P.rstd[c] = rs;
      P.scale[c] = sc;
      P.shift[c] = sh;
      if (P.update_moving) {
        const float uvar = fn_ > 1.f ? fm2 / (fn_ - 1.f) : fm2;
        P.mmean[c] = mmv - (1.f - P.momentum) * (mmv - fmu);
        P.mvar[c] = mvv - (1.f - P.momentum) * (mvv - uvar);
      }
    }
  }
  __syncthreads();
}

// The BN-backward counterpart (BnBwdPre, the direct dgrad's ABWD prologue): sums
// sum g, sum g*xhat over the producer's [cnt][2][C] partials with the same
// thread layout, shuffles and fixed-order cross-wave pass.  Returns in out1/out2
// (valid for tid < C).  `scratch` >= 8*C floats.
__device__ __forceinline__ void bn_prefin_sums(const float* __restrict__ part, int cnt, int C,
                                               float* scratch, float& out1, float& out2) {
  const int tid = threadIdx.x;
  const int CG = C >> 2, cg = tid & (CG - 1), q = tid / CG, G = 256 / CG;
  f32x4 a1 = {0.f, 0.f, 0.f, 0.f}, a2 = {0.f, 0.f, 0.f, 0.f};
  for (int base = q; base < cnt; base += PFIN_ITEMS * G) {
    f32x4 v1[PFIN_ITEMS], v2[PFIN_ITEMS];
#pragma unroll
    for (int u = 0; u < PFIN_ITEMS; ++u) {
      const int t = base + u * G;
      const bool ok = t < cnt;
      const float* row = part + (long)t * 2 * C + 4 * cg;
      v1[u] = ok ? *reinterpret_cast<const f32x4*>(row) : f32x4{0.f, 0.f, 0.f, 0.f};
      v2[u] = ok ? *reinterpret_cast<const f32x4*>(row + C) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < PFIN_ITEMS; ++u) {
      a1 += v1[u];
      a2 += v2[u];
    }
  }
  for (int o = CG; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a1[j] += __shfl_xor(a1[j], o, 64);
      a2[j] += __shfl_xor(a2[j], o, 64);
    }
  }
  const int wave = tid >> 6, lane = tid & 63;
  if (lane < CG) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      scratch[(wave * 2) * C + 4 * lane + j] = a1[j];
      scratch[(wave * 2 + 1) * C + 4 * lane + j] = a2[j];
    }
  }
  __syncthreads();
  out1 = out2 = 0.f;
  if (tid < C) {
    out1 = (scratch[tid] + scratch[2 * C + tid]) + (scratch[4 * C + tid] + scratch[6 * C + tid]);
    out2 = (scratch[C + tid] + scratch[3 * C + tid]) + (scratch[5 * C + tid] + scratch[7 * C + tid]);
  }
}

}  // namespace dtr
