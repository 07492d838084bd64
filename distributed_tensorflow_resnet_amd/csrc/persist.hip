// Persistent multi-layer prototype for the small-batch CIFAR stage 3 ("weak"
// item 1): L consecutive 3x3 / stride-1 64 -> 64 convolutions on 8x8 maps -- the
// residual chain of ResNet-50 v2 stage 3, resnet_model_official.py:80-91 + the
// building_block of :120-160 (x + conv2(relu(bn2(conv1(relu(bn1(x))))))) -- in ONE
// launch, a grid barrier between dependent layers instead of a kernel boundary.
//
// Per layer, every workgroup (one image x 32 of the 64 output channels, 4 waves):
//   1. waits at the grid barrier for layer l-1 (its weights for layer l were prefetched
//      into LDS before the wait, so the weight staging hides behind the barrier);
//   2. finalizes the input BatchNorm from layer l-1's batch sums (training-mode
//      statistics, every workgroup redundantly: 64 channels), applies BN+ReLU while
//      staging the 10x10x64 halo (zero padding stays zero) into LDS;
//   3. 18 k-steps of v_mfma_f32_16x16x32_bf16 (k = tap x channel) per 16x16 fragment;
//   4. epilogue: + block input (odd layers: the conv2 of a building block), ONE bf16
//      rounding, 16-B stores, the output's per-channel sum / sum of squares into the
//      layer's fp32 accumulators (memory-side atomics), then arrives at the barrier.
//
// Hand-offs between workgroups follow the measured "sc1" recipe of MI355X_MICROARCH.md
// (Valid forms, row 1): every store of a hand-off byte is a write-through sc1 buffer
// store, every storing wave drains (vmcnt(0)) before its workgroup's lane 0 adds to
// the barrier counter, the consumer polls that counter with relaxed agent-scope loads
// and then reads the bytes with sc1 loads only -- no release / acquire fences.  Every
// spin is bounded (wall clock): a timed-out barrier sets *err and the kernel drains.
//
// Scope: a measurement prototype (scripts/persist_probe.py), not wired into the engine.
// BN sums are fp32 atomics (order-dependent in the last bits, unlike the engine's
// fixed-order combines); stage 3 only (C = 64, 8x8).  The grid (2 workgroups per image)
// must be co-resident: the host caps it at 256 (one per CU).
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace dtr {

namespace {

constexpr int PC = 64;                // channels
constexpr int PH = 8;                 // map side
constexpr int PK = 9 * PC;            // reduction depth (tap, channel)
constexpr int WROW = PK + 8;          // LDS weight row (bf16), padded 16 B
constexpr int CO_WG = 32;             // output channels per workgroup
constexpr int HALO = (PH + 2) * (PH + 2);
constexpr long long kBarrierTicks = 200000000;   // 2 s at 100 MHz

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 ld_sc1(const __amdgpu_buffer_rsrc_t& rs, int byte_off) {
  return __builtin_bit_cast(bf16x8, (u32x4)__builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16));
}

__device__ __forceinline__ float ld_sc1_f(const __amdgpu_buffer_rsrc_t& rs, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, byte_off, 0, 16));
}

}  // namespace

__global__ void __launch_bounds__(256)
persist_stage_fwd_kernel(PersistArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* wl = reinterpret_cast<bf16*>(smem);                        // [CO_WG][WROW]
  bf16* halo = wl + CO_WG * WROW;                                  // [HALO][PC] swizzled
  float* bn_s = reinterpret_cast<float*>(halo + HALO * PC);        // [2][PC] scale, shift
  float* ct = bn_s + 2 * PC;                                       // [64 px][CO_WG] fp32
  float* red = ct + 64 * CO_WG;                                    // [2][4 quarters][CO_WG]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int img = blockIdx.x >> 1, co0 = (blockIdx.x & 1) * CO_WG;
  const int G = gridDim.x;
  const long act = (long)p.N * PH * PH * PC;                        // elements per activation
  const auto rs_y = __builtin_amdgcn_make_buffer_rsrc(p.y, 0, 0x7fffffff, 0x00020000);
  const auto rs_st = __builtin_amdgcn_make_buffer_rsrc(p.stats, 0, 0x7fffffff, 0x00020000);

  // weight slice of layer l -> registers (9 x 16 B per thread), stored to LDS later
  bf16x8 wv[9];
  auto load_w = [&](int l) {
    const bf16* wsrc = p.w + (long)l * PC * PK;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int q = tid + i * 256;                 // 2304 = 32 rows x 72 units
      const int row = q / (PK / 8), u = q - row * (PK / 8);
      wv[i] = *reinterpret_cast<const bf16x8*>(wsrc + (long)(co0 + row) * PK + u * 8);
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int q = tid + i * 256;
      const int row = q / (PK / 8), u = q - row * (PK / 8);
      *reinterpret_cast<bf16x8*>(wl + row * WROW + u * 8) = wv[i];
    }
  };

  load_w(0);
  for (int l = 0; l < p.L; ++l) {
    // ---- 1. barrier: layer l-1 complete everywhere ----
    if (l > 0) {
      if (tid == 0) {
        const unsigned target = (unsigned)(l * G);
        const long long t0 = wall_clock64();
        while (__hip_atomic_load(p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kBarrierTicks) {
            __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __syncthreads();
      if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
    // ---- 2. input BN table, halo (BN+ReLU), weights to LDS ----
    const bool first = l == 0;
    const long in_off = first ? 0 : (long)(l - 1) * act;
    // halo loads first (one round trip), then the BN table from the batch sums
    bf16x8 hv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + i * 256;                 // 512 units = 64 px x 8
      const int px = q >> 3, u = q & 7;
      const long e = ((long)img * 64 + px) * PC + u * 8;
      hv[i] = first ? *reinterpret_cast<const bf16x8*>(p.x0 + e)
                    : ld_sc1(rs_y, (int)((in_off + e) * 2));
    }
    bf16x8 rv[1];                                  // residual rows for the epilogue
    const bool resid = (l & 1) != 0;
    {
      const int px = tid >> 2, u = tid & 3;        // epilogue chunk of this thread
      const long e = ((long)img * 64 + px) * PC + co0 + u * 8;
      if (resid) rv[0] = l == 1 ? *reinterpret_cast<const bf16x8*>(p.x0 + e)
                                : ld_sc1(rs_y, (int)(((long)(l - 2) * act + e) * 2));
    }
    if (tid < PC) {
      float sc, sh;
      if (first) {
        sc = p.bn0_scale[tid];
        sh = p.bn0_shift[tid];
      } else {
        const float cnt = (float)(p.N * PH * PH);
        const float s1 = ld_sc1_f(rs_st, ((l - 1) * 2 * PC + tid) * 4);
        const float s2 = ld_sc1_f(rs_st, ((l - 1) * 2 * PC + PC + tid) * 4);
        const float mean = s1 / cnt, var = fmaxf(s2 / cnt - mean * mean, 0.f);
        sc = p.gamma[(l - 1) * PC + tid] * rsqrtf(var + p.eps);
        sh = p.beta[(l - 1) * PC + tid] - mean * sc;
      }
      bn_s[tid] = sc;
      bn_s[PC + tid] = sh;
    }
    // zero the halo border (padding), store the weights (wl is free: the previous
    // layer's MFMAs ended with a barrier)
    for (int q = tid; q < HALO * 8; q += 256) {
      const int hp = q >> 3, hr = hp / (PH + 2), hc = hp - hr * (PH + 2);
      if (hr == 0 || hc == 0 || hr == PH + 1 || hc == PH + 1)
        *reinterpret_cast<bf16x8*>(halo + (hp * 8 + ((q & 7) ^ (hp & 7))) * 8) = bf16x8{};
    }
    store_w();
    __syncthreads();                               // BN table visible
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + i * 256;
      const int px = q >> 3, u = q & 7;
      const int hp = ((px >> 3) + 1) * (PH + 2) + (px & 7) + 1;
      const bf16x8 v = affine_relu8(hv[i], bn_s + u * 8, bn_s + PC + u * 8);
      *reinterpret_cast<bf16x8*>(halo + (hp * 8 + (u ^ (hp & 7))) * 8) = v;
    }
    __syncthreads();
    // the next layer's weights: in flight across this layer's MFMAs, epilogue and barrier
    if (l + 1 < p.L) load_w(l + 1);

    // ---- 3. MFMA: wave = 16 pixels (2 image rows) x 32 channels ----
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int pxa = wave * 16 + fr;                // this lane's A row (output pixel)
    const int ar = pxa >> 3, ac = pxa & 7;
#pragma unroll
    for (int s = 0; s < PK / 32; ++s) {
      const int k = s * 32 + fq * 8;
      const int tap = k / PC, u = (k - tap * PC) >> 3;
      const int dy = tap / 3, dx = tap - dy * 3;
      const int hp = (ar + dy) * (PH + 2) + ac + dx;
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(halo + (hp * 8 + (u ^ (hp & 7))) * 8);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(wl + (nb * 16 + fr) * WROW + k);
        acc[nb] = mfma16(af, bfr, acc[nb]);
      }
    }
    // ---- 4. epilogue: fp32 tile -> LDS -> 16-B rows (+ residual), stats, arrive ----
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) ct[(wave * 16 + fq * 4 + i) * CO_WG + nb * 16 + fr] = acc[nb][i];
    __syncthreads();
    const int px = tid >> 2, u = tid & 3;
    bf16x8 ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = ct[px * CO_WG + u * 8 + j];
      if (resid) v += (float)rv[0][j];
      ob[j] = (bf16)v;
    }
    const long e = (long)l * act + ((long)img * 64 + px) * PC + co0 + u * 8;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ob), rs_y, (int)(e * 2), 0, 16);
    // BN sums of the rounded outputs: write them back over this thread's own fp32 slots,
    // then thread (which, quarter, c) sums 16 pixels of channel c, 64 threads finish
#pragma unroll
    for (int j = 0; j < 8; ++j) ct[px * CO_WG + u * 8 + j] = (float)ob[j];
    __syncthreads();
    {
      const int c = tid & 31, qtr = (tid >> 5) & 3, which = tid >> 7;
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = ct[(qtr * 16 + r) * CO_WG + c];
        t += which ? v * v : v;
      }
      red[(which * 4 + qtr) * CO_WG + c] = t;
    }
    __syncthreads();
    if (tid < 2 * CO_WG) {
      const int which = tid / CO_WG, c = tid - which * CO_WG;
      const float t = red[(which * 4) * CO_WG + c] + red[(which * 4 + 1) * CO_WG + c] +
                      red[(which * 4 + 2) * CO_WG + c] + red[(which * 4 + 3) * CO_WG + c];
      __hip_atomic_fetch_add(p.stats + (l * 2 + which) * PC + co0 + c, t, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores and atomics
    __syncthreads();
    if (tid == 0)
      __hip_atomic_fetch_add(p.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

void persist_stage_fwd(const PersistArgs& a, hipStream_t s) {
  if (a.N < 1 || 2 * a.N > 256 || a.L < 1 || a.L > 64)
    throw std::invalid_argument("persist_stage_fwd: 1 <= N <= 128 images, 1 <= L <= 64 layers");
  const size_t lds = (size_t)CO_WG * WROW * 2 + (size_t)HALO * PC * 2 + 2 * PC * 4 +
                     64 * CO_WG * 4 + 4 * 2 * CO_WG * 4;
  hipLaunchKernelGGL(persist_stage_fwd_kernel, dim3(2 * a.N), dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
