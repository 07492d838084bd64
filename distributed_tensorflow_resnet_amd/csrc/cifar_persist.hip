// Persistent small-batch CIFAR step: the whole forward in one launch, the whole
// backward (with its weight gradients) in one more.
//
// Why: at the per-rank batches of the strong-scaling headline config (global batch 128
// over 4-8 GPUs = 16-32 images per rank) every CIFAR conv is a few MFMA microseconds
// wrapped in a ~1.5 us kernel boundary plus a global-memory round trip of its operands
// (profiles/cifar_direct_conv_phases.md); ~110 dependent launches set the step time.
// Here each image is split into P row slices and one 512-thread workgroup owns one slice
// for the whole network (resnet_model_official.py:217-278, building_block :94-130):
//   * the slice's activations stay on-chip between layers: a conv's fp32 accumulators
//     are rounded to bf16 in registers, the next BatchNorm + ReLU is applied from the
//     registers straight into an LDS halo, and the next conv reads its B operand there;
//   * a 3x3 conv needs one halo row from each neighbouring slice: the forward reads it
//     from the tensor the neighbour publishes anyway (the activations saved for the
//     backward, stored write-through before the barrier) and applies BN + ReLU itself;
//     the backward recomputes the neighbour's BN-backward output rows from what the
//     neighbour published before the barrier (its dgrad output) plus saved tensors;
//   * BatchNorm's batch statistics are the only cross-slice dependency: each workgroup
//     adds its slice's per-channel sums into fp64 replicas with memory-side atomics
//     (exact: fp32 partials summed in fp64, so the result does not depend on the order),
//     one grid barrier, then every workgroup reads the sums -- one round trip;
//   * the next layer's weights are prefetched into registers by waves 1-7 between the
//     barrier's arrive and its wait (wave 0 polls), then stored to LDS;
//   * MFMA orientation D[channel][pixel] = W[channel][k] x Act[k][pixel]
//     (v_mfma_f32_16x16x32_bf16): a lane's accumulator holds 4 consecutive channels of
//     one pixel, i.e. one 8-byte NHWC store / LDS write after the bf16 rounding;
//   * pixels are kept in a "canonical" order per slice: parity-class-major on the 32x32
//     and 16x16 maps, so every stride-2 dgrad tile (sub-pixel decomposition: 1, 2, 2 or
//     4 taps per output parity class) is made of pixels of one class.
// In the backward launch the workgroups beyond the N x P slices compute the 52 weight
// gradients (dW = sum_p dy x im2col(relu(bn(x)))) per image group into fp32 slabs: they
// take items from one queue in readiness order (the slices join once their dgrad chain
// is done), each as soon as the readiness count says its dy is published; the existing
// deterministic grouped reduce sums the slabs afterwards (which workgroup ran an item
// does not change its slab: bitwise deterministic).
//
// Hand-off protocol (MI355X_MICROARCH.md, "Valid forms" row 1): every byte another
// workgroup reads inside the launch (published tensors) is stored write-through (sc1),
// every wave drains (s_waitcnt vmcnt(0)) before its workgroup's lane 0 adds to the
// barrier counter, consumers poll the counter with relaxed agent loads and read the bytes
// with sc1 loads.  BN sums are memory-side atomics, read with sc1 loads after the
// barrier.  Every spin is bounded (2 s of wall clock): a timed-out wait sets *err and the
// workgroup exits.  The grid must be co-resident: one workgroup per CU, grid <= CUs.
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace dtr {

namespace {

constexpr int PT = PRN_THREADS;
constexpr int NW = PT / 64;                  // waves per workgroup
constexpr long long kSpinTicks = 200000000;  // 2 s at 100 MHz

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ---- geometry ---------------------------------------------------------------------
template <int S, int P>
struct Stg {                                  // stage S: R x R maps, C channels, P slices
  static constexpr int R = 32 >> S, C = 16 << S, U = C / 8, W2 = R + 2;
  static constexpr int RS = R / P, HR = RS + 2;          // rows per slice, halo rows
  static constexpr int NPX = R * RS;                     // pixels per slice
  static constexpr int NPB = NPX / 16, NCB = C / 16;     // 16-pixel / 16-channel blocks
  static constexpr int WPB = NPB >= NW ? 1 : NW / NPB;   // waves per pixel block
  static constexpr int PBW = NPB >= NW ? NPB / NW : 1;   // pixel blocks per wave
  static constexpr int CBW = NCB / WPB > 0 ? NCB / WPB : 1;   // channel blocks per wave
  static constexpr int TPW = PBW * CBW;                  // 16x16 tiles per wave
  static constexpr int NT = NPB * NCB;                   // 16x16 output tiles
  static constexpr bool ALL = NT >= NW;                  // every wave holds tiles
  static constexpr bool CLS = R > 8;                     // parity-class-major pixel order
  static_assert(RS >= 2 && (!CLS || RS % 2 == 0) && NPX % 16 == 0 && TPW <= 8, "slices");
  static_assert(!CLS || (NPB / 4) % PBW == 0, "a wave's pixel blocks lie in one class");
};

// slice k's canonical pixel p -> image (h, w): parity-class-major on 32x32 / 16x16
// (class, class row, class column), row-major on 8x8
template <int S, int P>
__device__ __forceinline__ void canon(int k, int p, int& h, int& w) {
  using G = Stg<S, P>;
  if constexpr (G::CLS) {
    constexpr int Q = G::NPX / 4, H2 = G::R / 2;
    const int cls = p / Q, idx = p - cls * Q, il = idx / H2;
    h = k * G::RS + 2 * il + (cls >> 1);
    w = 2 * (idx - il * H2) + (cls & 1);
  } else {
    h = k * G::RS + p / G::R;
    w = p % G::R;
  }
}

// this wave's tile t -> (pixel block, channel block); a wave is idle (no tiles) when the
// slice has fewer tiles than waves and its channel block is past the last
template <int S, int P>
__device__ __forceinline__ void tile_of(int wave, int t, int& pb, int& cb) {
  using G = Stg<S, P>;
  pb = (wave / G::WPB) * G::PBW + t / G::CBW;
  cb = (wave % G::WPB) * G::CBW + t % G::CBW;
}
template <int S, int P>
__device__ __forceinline__ bool wave_active(int wave) {
  using G = Stg<S, P>;
  return G::ALL || (wave % G::WPB) * G::CBW < G::NCB;
}

// LDS halo element offset: local pixel `pix` (row-major in the HR x W2 slice halo,
// column lc), channel c (multiple of 4) of a U-unit (8 channels per 16-B unit) image;
// units XOR-swizzled by the column so a fragment's 16 pixel lanes spread over banks
// (Not on the 32x32 map, U = 2: its fragments are parity-class-major, so their 16 lanes
// share the column parity and the swizzle bit -- it moved no lane to another bank, and
// without it a halo read is one add on a per-pixel-block base instead of five VALU ops.)
template <int U>
__device__ __forceinline__ int haddr(int pix, int lc, int c) {
  if constexpr (U == 2) return pix * 16 + c;
  return (pix * U + ((c >> 3) ^ (lc & (U - 1)))) * 8 + (c & 7);
}

// Descriptor tables (blocks, BatchNorms, weight-gradient items) are read-only for the
// whole launch: read them through the constant address space, i.e. scalar loads into
// SGPRs via the scalar cache.  Through a generic pointer the compiler issues vector
// loads, waits a full memory round trip for each pointer it needs and then builds
// buffer descriptors from VGPRs in readfirstlane loops.
#define DTR_CONST_AS __attribute__((address_space(4)))
template <typename T>
__device__ __forceinline__ T ld_const(const T* p) {
#if __HIP_DEVICE_COMPILE__
  return *(const DTR_CONST_AS T*)p;
#else
  return *p;   // (host pass: never called)
#endif
}

// Global loads / stores through pointers read from the descriptor tables: the compiler
// cannot infer their address space and emits flat instructions, which also count in
// lgkmcnt -- every LDS barrier (s_waitcnt lgkmcnt(0)) after one then waits for a memory
// round trip.  These casts make them global_load / global_store.
template <typename T>
__device__ __forceinline__ T ldg(const T* p) {
#if __HIP_DEVICE_COMPILE__
  return *(const __attribute__((address_space(1))) T*)p;
#else
  return *p;
#endif
}
template <typename T>
__device__ __forceinline__ void stg(T* p, T v) {
#if __HIP_DEVICE_COMPILE__
  *(__attribute__((address_space(1))) T*)p = v;
#else
  *p = v;
#endif
}

// 4-byte write-through store (global_store_dword ... sc1): read by another agent-scope
// consumer before this kernel ends (overlap mode)
__device__ __forceinline__ void st_sc1_f32(float* p, float v) {
#if __HIP_DEVICE_COMPILE__
  __hip_atomic_store((__attribute__((address_space(1))) float*)p, v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = v;
#endif
}

__device__ __forceinline__ bf16x8 lds16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ double ld_sc1_d(const double* p) {
#if __HIP_DEVICE_COMPILE__
  return __hip_atomic_load((const __attribute__((address_space(1))) double*)p, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#else
  return *p;
#endif
}
// memory-side fp64 add (global_atomic_add_f64, no return)
__device__ __forceinline__ void atomic_add_g(double* p, double v) {
#if __HIP_DEVICE_COMPILE__
  __builtin_amdgcn_global_atomic_fadd_f64((__attribute__((address_space(1))) double*)p, v);
#else
  *p += v;
#endif
}
// a wave-uniform pointer, stated as such (SGPRs): a buffer descriptor built from VGPRs
// costs a readfirstlane waterfall loop around every buffer instruction
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}

// 8-byte write-through store of 4 bf16 / 16-byte sc1 load (buffer ops with the sc1 bit);
// `base` is wave-uniform
__device__ __forceinline__ void st_sc1_b64(bf16* base, long elem, bf16x4 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, (int)(elem * 2), 0, 16);
}
// the same store without sc1 (write-back L2): tensors only a later launch reads
__device__ __forceinline__ void st_wb_b64(bf16* base, long elem, bf16x4 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, (int)(elem * 2), 0, 0);
}
__device__ __forceinline__ void st_sc1_b128(bf16* base, long elem, bf16x8 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, (int)(elem * 2), 0, 16);
}
__device__ __forceinline__ bf16x8 ld_sc1_b128(const bf16* base, long elem) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(const_cast<bf16*>(base)), 0,
                                                    0x7fffffff, 0x00020000);
  return __builtin_bit_cast(bf16x8, (u32x4)__builtin_amdgcn_raw_buffer_load_b128(rs, (int)(elem * 2), 0, 16));
}

// Opaque copies of the lane / wave ids: every per-tile address is derived from them
// inside each phase instead of being hoisted to the kernel entry and kept live across
// the whole network (which spilled hundreds of registers).
__device__ __forceinline__ int opaque_v(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ int opaque_s(int v) {
  asm volatile("" : "+s"(v));
  return v;
}

// ---- grid barrier ---------------------------------------------------------------------
// Arrival counters sharded over up to PRN_SHARDS cache lines: workgroup b adds to line
// b % shards (8 or 64, prn_shards; with 8, one XCD per line under round-robin placement),
// and the waiters poll all lines with ONE load, one lane per line.  One shared counter serialises its arrivals at the memory side (~12 ns
// each) and its pollers contend with them: microbench/bn_barrier.hip, profiles/bn_barrier.md
// -- a BN barrier (sums, drain, arrive, wait, sums read) at 128 workgroups 3.94 -> 2.72 us,
// at 256 8.85 -> 4.86 us, at 64 2.31 -> 2.07 us.
constexpr int PRN_SHARDS = 64, PRN_LINE = 32;   // (max shards) 32 words = one 128-B line per shard
// bar layout (words): forward shards at PRN_FWD + 32 s, backward shards at PRN_BWD + 32 s,
// the backward readiness count at PRN_READY, the weight-gradient item queue at PRN_QUEUE
// (each on its own line; PRN_BAR_WORDS in all, zeroed every step)
constexpr int PRN_FWD = 0, PRN_BWD = PRN_SHARDS * PRN_LINE, PRN_READY = 2 * PRN_SHARDS * PRN_LINE,
              PRN_QUEUE = PRN_READY + PRN_LINE, PRN_BUCKET = PRN_QUEUE + PRN_LINE,
              PRN_NBUCKET = 3, PRN_BAR_WORDS = PRN_BUCKET + PRN_NBUCKET * PRN_LINE;
constexpr unsigned PRN_BUCKET_RELEASED = 0x40000000u;   // a timed-out launch releases the waiters

// a timed-out wait: flag the error and release the comm stream's bucket waiters (they
// would otherwise wait for counts the exiting workgroups never reach)
__device__ __forceinline__ void prn_fail(unsigned* bar, int* err) {
  __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int b = 0; b < PRN_NBUCKET; ++b)
    __hip_atomic_store(bar + PRN_BUCKET + b * PRN_LINE, PRN_BUCKET_RELEASED, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Every wave drains its stores / atomics, then lane 0 arrives on its shard.  The caller
// issues its prefetches (waves 1-7) and waits (grid_wait).
__device__ __forceinline__ void grid_arrive(unsigned* bar, int shards) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(bar + (blockIdx.x % shards) * PRN_LINE, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until barrier k (1-based) of `nsl` arriving workgroups is complete: shard s holds
// k x (the arrivers b < nsl with b % 8 == s).  Lanes 0-7 of wave 0 poll their shard every
// 64 clocks.  Returns false when the wait timed out (*err set): the caller exits.
__device__ __forceinline__ bool grid_wait(unsigned* base, int off, unsigned k, unsigned nsl,
                                          int shards, int* err, int* flag) {
  unsigned* bar = base + off;
  if ((int)threadIdx.x < shards) {
    const unsigned sh = threadIdx.x;
    const unsigned target = k * ((nsl + shards - 1 - sh) >> __builtin_ctz(shards));   // (1 or 8)
    const unsigned* p = bar + sh * PRN_LINE;
    const long long t0 = wall_clock64();
    int ok = 1;
    for (;;) {
      const bool done = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (__builtin_amdgcn_ballot_w64(!done) == 0) break;   // every shard complete
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > kSpinTicks) {
        if (sh == 0) prn_fail(base, err);
        ok = 0;
        break;
      }
    }
    if (sh == 0) *flag = ok;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*flag) != 0;   // uniform: no divergent region after
}

// Wait until the single counter `ctr` reaches `target` (the weight-gradient workgroups on
// the readiness line; they poll 8x less often: ~190 pollers on one line slow its writer).
template <int SLEEP = 8>
__device__ __forceinline__ bool count_wait(unsigned* base, int off, unsigned target, int* err,
                                           int* flag) {
  if (threadIdx.x == 0) {
    const unsigned* ctr = base + off;
    const long long t0 = wall_clock64();
    int ok = 1;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(SLEEP);
      if (wall_clock64() - t0 > kSpinTicks) {
        prn_fail(base, err);
        ok = 0;
        break;
      }
    }
    *flag = ok;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*flag) != 0;
}

// ---- weights: global -> registers (waves 1-7) -> LDS -----------------------------------
struct WLoad {
  const bf16* src;
  int rows, K, KP;      // LDS rows x K (padded row KP; columns [K, KP - 8) zero)
  int dgrad, cin, cout; // dgrad: rows = ci of HWIO [tap][ci][co], k = tap * cout + co
  // unit u -> (row, 16-B column j) without integer division (the shapes are runtime
  // values -- the next block's -- and a 32-bit division by one is ~20 VALU per unit,
  // ~40 % of the forward's VALU): row = (u + 1/2) x (8 / K) in fp32 (exact: u < 2^13 and
  // the quotient's fraction is >= 1/144 away from an integer); cout / 8 is a power of 2
  float inv_upr;
  int cu_shift, ci_shift;   // log2(cout / 8), log2(cin): the dgrad's HWIO offsets as shifts
};
__device__ __forceinline__ int wl_row(const WLoad& L, int u) {
  return (int)(((float)u + 0.5f) * L.inv_upr);
}

// (the thread id is taken opaque in both: otherwise each stage loop hoists the per-thread
// addresses of every weight unit out of its loop and keeps them live across the blocks --
// the backward kernels' VGPR spills)
template <int NR>
__device__ __forceinline__ void w_prefetch(const WLoad& L, bf16x8 (&r)[NR]) {
  const int t = opaque_v((int)threadIdx.x) - 64;
  if (t < 0 || L.src == nullptr) return;
  const int upr = L.K / 8, units = L.rows * upr;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int u = t + i * (PT - 64);
    if (u < units) {
      int off;   // (< 2^31: weights of <= 64 x 576)
      if (L.dgrad) {   // HWIO [tap][ci = row][co]: ((tap * cin + row) * cout + co
        const int row = wl_row(L, u), j = u - __umul24(row, upr);
        const int tap = j >> L.cu_shift;
        off = ((((tap << L.ci_shift) + row) << L.cu_shift) + (j - (tap << L.cu_shift))) * 8;
      } else {         // rows of K contiguous: unit u is at u x 8
        off = u * 8;
      }
      r[i] = ldg(reinterpret_cast<const bf16x8*>(L.src + off));
    }
  }
}

template <int NR>
__device__ __forceinline__ void w_store(const WLoad& L, const bf16x8 (&r)[NR], bf16* wl) {
  if (L.src == nullptr) return;
  const int tid = opaque_v((int)threadIdx.x), t = tid - 64;
  const int upr = L.K / 8, units = L.rows * upr;
  if (t >= 0) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int u = t + i * (PT - 64);
      if (u < units) {   // row * KP + j * 8 = u * 8 + row * (KP - K)
        const int row = wl_row(L, u);
        *reinterpret_cast<bf16x8*>(wl + u * 8 + __umul24(row, L.KP - L.K)) = r[i];
      }
    }
  }
  const int pad = (L.KP - 8 - L.K) / 8;   // zero columns up to the last k-step (0-3)
  for (int q = tid; q < L.rows * pad; q += PT) {
    const int row = pad == 1 ? q : pad == 2 ? q >> 1 : q / pad, j = upr + (q - row * pad);
    *reinterpret_cast<bf16x8*>(wl + row * L.KP + j * 8) = bf16x8{};
  }
}

// 16-B weight units of a conv, and the prefetch registers waves 1-7 need for them
__host__ __device__ constexpr int conv_units(int co, int ci, int ks) { return co * ks * ks * ci / 8; }
__host__ __device__ constexpr int nreg(int units) { return (units + PT - 65) / (PT - 64); }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

__host__ __device__ constexpr int kpad_of(int K) { return ((K + 31) / 32) * 32 + 8; }

__device__ __forceinline__ WLoad wl_fwd(const bf16* src, int co, int ci, int ks) {
  const int K = ks * ks * ci;
  return WLoad{src, co, K, kpad_of(K), 0, ci, co, __frcp_rn((float)(K / 8)), __builtin_ctz(co / 8),
               __builtin_ctz(ci)};
}
__device__ __forceinline__ WLoad wl_dgrad(const bf16* src, int co, int ci, int ks) {
  const int K = ks * ks * co;
  return WLoad{src, ci, K, kpad_of(K), 1, ci, co, __frcp_rn((float)(K / 8)), __builtin_ctz(co / 8),
               __builtin_ctz(ci)};
}

// ---- convolutions on the LDS halo ------------------------------------------------------
// acc[t] += sum_k W[channel][k] * Act[k][pixel] over this wave's tiles of output stage SO,
// slice k.  The input halo (CI channels, resolution R_SO * STR, slice rows RS_SO * STR
// plus one halo row above and below) holds image row hi at local row hi - k*RSI + 1.
// Forward (FLIP = false): tap (r, s) of output pixel (h, w) reads input (h*STR + r - PAD,
// w*STR + s - PAD), PAD = 1 for 3x3 (TF fixed padding), 0 for 1x1.
// Stride-1 dgrad (FLIP = true, 3x3): input (h + 1 - r, w + 1 - s) of the output gradient.
// Weights in LDS: [channel][k = tap * CI + ci] rows of KP.
// When the slice has fewer output tiles than waves (stage 3 at 4 slices: 4 tiles), the
// idle waves take half of each tile's k-steps (SPLIT) and their partial sums are added
// through the LDS scratch `xred` (two barriers; every wave calls this function).
template <int SO, int P, int CI, int KSZ, int STR, bool FLIP>
__device__ __forceinline__ void conv_acc(f32x4 (&acc)[8], const bf16* hal, const bf16* wl,
                                         int kslice, int wave, int lane, float* xred) {
  using G = Stg<SO, P>;
  lane = opaque_v(lane);
  constexpr int RI = G::R * STR, RSI = G::RS * STR, W2I = RI + 2, UI = CI >= 8 ? CI / 8 : 1;
  constexpr int K = KSZ * KSZ * CI, KS = (K + 31) / 32, KP = kpad_of(K);
  constexpr int PAD = KSZ == 3 ? 1 : 0;
  constexpr bool SPLIT = !G::ALL && KS >= 4 && NW % G::NT == 0;
  constexpr int WPT = SPLIT ? NW / G::NT : 1;   // waves per tile
  static_assert(!SPLIT || (G::TPW == 1 && G::NT * 256 * (WPT - 1) <= 8 * 128), "split scratch");
  int kh = 0;
  if constexpr (SPLIT) {
    kh = wave / G::NT;
    wave = wave % G::NT;
  } else if (!wave_active<SO, P>(wave)) {
    return;
  }
  const int fr = lane & 15, fq = lane >> 4;
  int hb[G::PBW], hcb[G::PBW];
#pragma unroll
  for (int i = 0; i < G::PBW; ++i) {
    int pb, cb, h, w;
    tile_of<SO, P>(wave, i * G::CBW, pb, cb);
    canon<SO, P>(kslice, pb * 16 + fr, h, w);
    const int lr = FLIP ? h - kslice * RSI + 2 : h * STR - PAD - kslice * RSI + 1;
    hcb[i] = FLIP ? w + 2 : w * STR - PAD + 1;
    hb[i] = lr * W2I + hcb[i];
  }
  int cb0, pb0;
  tile_of<SO, P>(wave, 0, pb0, cb0);
#pragma unroll
  for (int ks = kh; ks < KS; ks += WPT) {
    const int k = ks * 32 + fq * 8;
    int tap = k / CI;
    const int c = k - tap * CI;
    tap = tap < KSZ * KSZ ? tap : KSZ * KSZ - 1;   // padded k: zero weights
    const int tr = FLIP ? -(tap / KSZ) : tap / KSZ;
    const int ts = FLIP ? -(tap % KSZ) : tap % KSZ;
    bf16x8 a[G::CBW];
#pragma unroll
    for (int j = 0; j < G::CBW; ++j) a[j] = lds16(wl + ((cb0 + j) * 16 + fr) * KP + k);
#pragma unroll
    for (int i = 0; i < G::PBW; ++i) {
      const bf16x8 b = lds16(hal + haddr<UI>(hb[i] + tr * W2I + ts, hcb[i] + ts, c));
#pragma unroll
      for (int j = 0; j < G::CBW; ++j) acc[i * G::CBW + j] = mfma16(a[j], b, acc[i * G::CBW + j]);
    }
  }
  if constexpr (SPLIT) {   // partial sums of waves kh > 0 -> the tile's kh = 0 wave
    if (kh > 0) *reinterpret_cast<f32x4*>(xred + ((kh - 1) * G::NT + wave) * 256 + lane * 4) = acc[0];
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int j = 1; j < WPT; ++j)
        acc[0] += *reinterpret_cast<const f32x4*>(xred + ((j - 1) * G::NT + wave) * 256 + lane * 4);
    }
    __syncthreads();   // (xred is the BN sums' scratch next)
  }
}

// Stride-2 dgrad into output stage SO (high resolution, parity-class-major pixels), slice
// k, from the output gradient of CO channels at resolution R_SO / 2 in the halo `hal`
// (slice rows RS_SO / 2 + 2 halo rows):
//   3x3 (PROJ = false): dx(2i+a, 2j+b) = sum over taps r = a+1 (mod 2), s = b+1 (mod 2)
//     of dy(i + di, j + dj) W[r][s], di = (a + 1 - r) / 2 -- 1, 2, 2 or 4 taps per class;
//   1x1 (PROJ): dx(2i, 2j) = dy(i, j) Wp (class 0 only).
// Weights [ci][k = tap * CO + co].  A wave's pixel blocks all lie in one class.
template <int SO, int P, int CO, bool PROJ>
__device__ __forceinline__ void dgrad_s2_acc(f32x4 (&acc)[8], const bf16* hal, const bf16* wl,
                                             int kslice, int wave, int lane) {
  using G = Stg<SO, P>;
  lane = opaque_v(lane);
  static_assert(G::CLS, "class-major output");
  if (!wave_active<SO, P>(wave)) return;
  constexpr int RL = G::R / 2, RSL = G::RS / 2, W2L = RL + 2, UL = CO / 8;
  constexpr int KP = kpad_of(PROJ ? CO : 9 * CO);
  const int fr = lane & 15, fq = lane >> 4;
  int pb0, cb0;
  tile_of<SO, P>(wave, 0, pb0, cb0);
  const int cls = (pb0 * 16) / (G::NPX / 4);
  const int ca = cls >> 1, cbit = cls & 1;
  if (PROJ && cls != 0) return;
  int il[G::PBW], jl[G::PBW];
#pragma unroll
  for (int i = 0; i < G::PBW; ++i) {
    int pb, cb, h, w;
    tile_of<SO, P>(wave, i * G::CBW, pb, cb);
    canon<SO, P>(kslice, pb * 16 + fr, h, w);
    il[i] = (h >> 1) - kslice * RSL + 1;   // local halo row of dy(i, .)
    jl[i] = (w >> 1) + 1;
  }
  const int nr = PROJ ? 1 : (ca ? 2 : 1), ns = PROJ ? 1 : (cbit ? 2 : 1);
  for (int ri = 0; ri < nr; ++ri) {
    const int r = PROJ ? 0 : (ca ? 2 * ri : 1), di = PROJ ? 0 : (ca ? 1 - ri : 0);
    for (int si = 0; si < ns; ++si) {
      const int s = PROJ ? 0 : (cbit ? 2 * si : 1), dj = PROJ ? 0 : (cbit ? 1 - si : 0);
      const int tap = PROJ ? 0 : r * 3 + s;
#pragma unroll
      for (int kk = 0; kk < CO / 32; ++kk) {
        const int c = kk * 32 + fq * 8;
        const int k = tap * CO + c;
        bf16x8 av[G::CBW];
#pragma unroll
        for (int j = 0; j < G::CBW; ++j) av[j] = lds16(wl + ((cb0 + j) * 16 + fr) * KP + k);
#pragma unroll
        for (int i = 0; i < G::PBW; ++i) {
          const int hr = il[i] + di, hc = jl[i] + dj;
          const bf16x8 b = lds16(hal + haddr<UL>(hr * W2L + hc, hc, c));
#pragma unroll
          for (int j = 0; j < G::CBW; ++j) acc[i * G::CBW + j] = mfma16(av[j], b, acc[i * G::CBW + j]);
        }
      }
    }
  }
}

// ---- register tensors (bf16x4 per tile: 4 channels of one pixel) ------------------------
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[8]) {
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// image NHWC element offset of this lane's tile-t values
template <int S, int P>
__device__ __forceinline__ int gofs(int kslice, int wave, int lane, int t) {
  using G = Stg<S, P>;
  int pb, cb, h, w;
  tile_of<S, P>(wave, t, pb, cb);
  canon<S, P>(kslice, pb * 16 + (lane & 15), h, w);
  return (h * G::R + w) * G::C + cb * 16 + 4 * (lane >> 4);
}

template <int S, int P>
__device__ __forceinline__ void load_regs(bf16x4 (&v)[8], const bf16* img_base, int kslice,
                                          int wave, int lane) {
  lane = opaque_v(lane);
  if (!wave_active<S, P>(wave)) return;
#pragma unroll
  for (int t = 0; t < Stg<S, P>::TPW; ++t)
    v[t] = ldg(reinterpret_cast<const bf16x4*>(img_base + gofs<S, P>(kslice, wave, lane, t)));
}

// write-through (sc1) stores: these tensors are read by other workgroups in the launch.
// ROWS 1: only the slice's first and last rows (what the neighbouring slices read inside
// the launch), 2: only the rows between them, 0: all.  WB: write-back stores instead (the
// forward's saved tensors past the border rows: only the backward launch reads them).
template <int S, int P, int ROWS = 0, bool WB = false>
__device__ __forceinline__ void publish(const bf16x4 (&v)[8], bf16* img_base, int kslice,
                                        int wave, int lane) {
  using G = Stg<S, P>;
  lane = opaque_v(lane);
  if (!wave_active<S, P>(wave)) return;
#pragma unroll
  for (int t = 0; t < G::TPW; ++t) {
    int pb, cb, h, w;
    tile_of<S, P>(wave, t, pb, cb);
    canon<S, P>(kslice, pb * 16 + (lane & 15), h, w);
    const int lr = h - kslice * G::RS;
    const bool border = lr == 0 || lr == G::RS - 1;
    if (ROWS == 0 || (ROWS == 1) == border) {
      if constexpr (WB) st_wb_b64(img_base, (h * G::R + w) * G::C + cb * 16 + 4 * (lane >> 4), v[t]);
      else st_sc1_b64(img_base, (h * G::R + w) * G::C + cb * 16 + 4 * (lane >> 4), v[t]);
    }
  }
}

// The slice's own rows of a halo (rows 1..RS) -> the image tensor (write-through 16-B
// stores): publishes a tensor some time after it was staged, from LDS, without holding
// its registers live in between.
template <int S, int P>
__device__ __forceinline__ void halo_to_global(const bf16* hal, bf16* img_base, int kslice) {
  using G = Stg<S, P>;
  constexpr int UNITS = G::RS * G::R * G::U;
  for (int q = threadIdx.x; q < UNITS; q += PT) {
    const int row = q / (G::R * G::U), rem = q - row * G::R * G::U;
    const int col = rem / G::U, u = rem - col * G::U;
    const int lr = row + 1, lc = col + 1;
    st_sc1_b128(img_base, ((long)(kslice * G::RS + row) * G::R + col) * G::C + u * 8,
                lds16(hal + haddr<G::U>(lr * G::W2 + lc, lc, u * 8)));
  }
}

// ---- halos -------------------------------------------------------------------------------
// Neighbour halo rows: 2 rows x R pixels x U units (always 128 units) -- thread t < 128
// handles unit t: row sel = t / (R U) (0: image row k*RS - 1, 1: row (k+1)*RS), column,
// unit.  `ok` is false outside the image (the conv's zero padding).
template <int S, int P>
struct Nbr {
  static constexpr int UNITS = 2 * Stg<S, P>::R * Stg<S, P>::U;
  static_assert(UNITS <= PT, "neighbour units");
  int sel, col, u, gofs;   // gofs: image element offset of the unit
  bool ok;
  __device__ __forceinline__ Nbr(int kslice) {
    using G = Stg<S, P>;
    const int t = threadIdx.x;
    sel = t / (G::R * G::U);
    const int rem = t - sel * G::R * G::U;
    col = rem / G::U;
    u = rem - col * G::U;
    const int gr = sel ? (kslice + 1) * G::RS : kslice * G::RS - 1;
    ok = t < UNITS && gr >= 0 && gr < G::R;
    gofs = (gr * G::R + col) * G::C + u * 8;
  }
};

// own values (this wave's tiles; MODE 1: BN + ReLU with the LDS table sc/sh, 0: as is)
// -> halo rows 1..RS; the neighbour units `nv` (already transformed; zero where !ok)
// -> rows 0 and RS + 1; the left / right border columns -> zero
template <int S, int P, int MODE>
__device__ __forceinline__ void to_halo(bf16* hal, const bf16x4 (&v)[8], const float* sc,
                                        const float* sh, const Nbr<S, P>& nb, bf16x8 nv,
                                        int kslice, int wave, int lane) {
  using G = Stg<S, P>;
  lane = opaque_v(lane);
  const int fr = lane & 15, fq = lane >> 4;
  if (wave_active<S, P>(wave)) {
    // (MODE 1) this lane's 4 channels of each of the wave's channel blocks, read once: the
    // halo stores below may alias the table for the compiler, which re-read it per tile
    f32x4 scv[G::CBW], shv[G::CBW];
    if constexpr (MODE == 1) {
#pragma unroll
      for (int j = 0; j < G::CBW; ++j) {
        int pb, cb;
        tile_of<S, P>(wave, j, pb, cb);
        scv[j] = *reinterpret_cast<const f32x4*>(sc + cb * 16 + 4 * fq);
        shv[j] = *reinterpret_cast<const f32x4*>(sh + cb * 16 + 4 * fq);
      }
    }
#pragma unroll
    for (int t = 0; t < G::TPW; ++t) {
      int pb, cb, h, w;
      tile_of<S, P>(wave, t, pb, cb);
      canon<S, P>(kslice, pb * 16 + fr, h, w);
      const int c0 = cb * 16 + 4 * fq;
      bf16x4 o = v[t];
      if constexpr (MODE == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[r] = (bf16)fmaxf((float)v[t][r] * scv[t % G::CBW][r] + shv[t % G::CBW][r], 0.f);
      }
      const int lr = h - kslice * G::RS + 1;
      *reinterpret_cast<bf16x4*>(hal + haddr<G::U>(lr * G::W2 + w + 1, w + 1, c0)) = o;
    }
  }
  if ((int)threadIdx.x < Nbr<S, P>::UNITS) {
    const int lr = nb.sel ? G::RS + 1 : 0, lc = nb.col + 1;
    *reinterpret_cast<bf16x8*>(hal + haddr<G::U>(lr * G::W2 + lc, lc, nb.u * 8)) = nb.ok ? nv : bf16x8{};
  }
  // left / right border columns of every halo row
  for (int q = threadIdx.x; q < 2 * G::HR * G::U; q += PT) {
    const int b = q / G::U, u = q - b * G::U;
    const int lr = b >> 1, lc = (b & 1) ? G::R + 1 : 0;
    *reinterpret_cast<bf16x8*>(hal + haddr<G::U>(lr * G::W2 + lc, lc, u * 8)) = bf16x8{};
  }
}

// Sum over the 16 lanes of a DPP row (the 16 pixel lanes of an MFMA fragment): quad
// swaps, then the half-row and row mirrors -- VALU-latency DPP moves instead of the
// LDS-latency ds_bpermute chain __shfl_xor compiles to.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
  return v;
}

// fp64 accumulator replicas per BatchNorm of the persistent kernels (the per-layer
// kernels use BN_ACC_REP; the engine sizes every BN's block for the larger count).  Each
// workgroup adds into replica blockIdx % REP; after the barrier every workgroup reads all
// REP replicas of its channels.  Same-box A/B, step ms bs128 / bs16
// (profiles/cifar_persist_variants.md): 1 replica 1.058 / 0.657 (same-address atomics
// serialise), 2: 0.887 / 0.594, 4: 0.850 / 0.595, 8: 0.862 / 0.597, 16: 0.879 / 0.627
// (the combine's reads grow).
constexpr int PRN_ACC_REP = 4;

// Per-channel sums over this slice of two per-value quantities f(t, r, x1, x2), added to
// a BN's fp64 accumulator replicas acc [PRN_ACC_REP][2][C] (memory-side atomics; exact, so
// order-independent).  Folding: xor-shuffles over the 16 pixel lanes, then the waves that
// hold each channel through LDS `red` [8 waves][128] in a fixed order.
template <int S, int P, typename F>
__device__ __forceinline__ void bn_sums(F f, float* red, double* acc, int wave, int lane) {
  using G = Stg<S, P>;
  lane = opaque_v(lane);
  const int fr = lane & 15, fq = lane >> 4;
  if (wave_active<S, P>(wave)) {
    float s1[G::CBW][4], s2[G::CBW][4];
#pragma unroll
    for (int j = 0; j < G::CBW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
#pragma unroll
    for (int t = 0; t < G::TPW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a, b;
        f(t, r, a, b);
        s1[t % G::CBW][r] += a;
        s2[t % G::CBW][r] += b;
      }
#pragma unroll
    for (int j = 0; j < G::CBW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] = row16_sum(s1[j][r]);
        s2[j][r] = row16_sum(s2[j][r]);
      }
    if (fr == 0) {
      int pb, cb0;
      tile_of<S, P>(wave, 0, pb, cb0);
#pragma unroll
      for (int j = 0; j < G::CBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = (cb0 + j) * 16 + 4 * fq + r;
          red[wave * 128 + c] = s1[j][r];
          red[wave * 128 + 64 + c] = s2[j][r];
        }
    }
  }
  __syncthreads();
  if (threadIdx.x < G::C) {
    const int c = threadIdx.x;
    const int grp = (c / 16) / G::CBW;   // waves w with w % WPB == grp hold channel c
    float v1 = 0.f, v2 = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (w % G::WPB == grp) {
        v1 += red[w * 128 + c];
        v2 += red[w * 128 + 64 + c];
      }
    double* p = acc + (long)(blockIdx.x % PRN_ACC_REP) * 2 * G::C + c;
    atomic_add_g(p, (double)v1);
    atomic_add_g(p + G::C, (double)v2);
  }
}

// After the barrier: the channel's two sums from the PRN_ACC_REP replicas (sc1 loads,
// replicas added in a fixed order)
__device__ __forceinline__ void acc_read(const double* acc, int C, int c, double& s1, double& s2) {
  double a[PRN_ACC_REP], b[PRN_ACC_REP];
#pragma unroll
  for (int r = 0; r < PRN_ACC_REP; ++r) {
    a[r] = ld_sc1_d(acc + (long)r * 2 * C + c);
    b[r] = ld_sc1_d(acc + (long)r * 2 * C + C + c);
  }
  s1 = s2 = 0.0;
#pragma unroll
  for (int r = 0; r < PRN_ACC_REP; ++r) {
    s1 += a[r];
    s2 += b[r];
  }
}

// BN parameters prefetched into registers (thread c < C) before a barrier wait
struct BnRegs {
  float g, b, mean, rstd, scale, shift, mm, mv;
};
// (workgroup 0 also updates the moving averages: their old values are prefetched too,
// or its read-modify-write would put a memory round trip in front of its next arrive --
// and every workgroup waits for that one)
__device__ __forceinline__ void bn_prefetch_fwd(const PrnBn& bn, int C, BnRegs& r) {
  const int c = threadIdx.x;
  if (c < C) {
    r.g = ldg(bn.gamma + c);
    r.b = ldg(bn.beta + c);
    if (blockIdx.x == 0) {
      r.mm = ldg(bn.mmean + c);
      r.mv = ldg(bn.mvar + c);
    }
  }
}
__device__ __forceinline__ void bn_prefetch_bwd(const PrnBn& bn, int C, BnRegs& r) {
  const int c = threadIdx.x;
  if (c < C) {
    r.g = ldg(bn.gamma + c);
    r.mean = ldg(bn.mean + c);
    r.rstd = ldg(bn.rstd + c);
    r.scale = ldg(bn.scale + c);
    r.shift = ldg(bn.shift + c);
  }
}

// the forward table (scale, shift, mean, rstd) of a BN the forward launch finalized,
// into registers before a wait / from registers into LDS [4][64] as (scale, shift,
// -mean*rstd, rstd): the backward's xhat = x*rstd + (-mean*rstd), one fma
__device__ __forceinline__ void bn_prefetch_tab(const PrnBn& bn, int C, BnRegs& r) {
  const int c = threadIdx.x;
  if (c < C) {
    r.scale = ldg(bn.scale + c);
    r.shift = ldg(bn.shift + c);
    r.mean = ldg(bn.mean + c);
    r.rstd = ldg(bn.rstd + c);
  }
}
__device__ __forceinline__ void tab_store(const BnRegs& r, int C, float* tbl) {
  const int c = threadIdx.x;
  if (c < C) {
    tbl[c] = r.scale;
    tbl[64 + c] = r.shift;
    tbl[128 + c] = -r.mean * r.rstd;
    tbl[192 + c] = r.rstd;
  }
}

// forward BN: sums -> scale/shift/mean/rstd table [4][64] in LDS; workgroup 0 publishes the
// batch statistics and updates the moving averages (TF FusedBatchNorm, bn_fused.h).
// Ends with a barrier.
__device__ __forceinline__ void bn_fwd_table(const PrnBn& bn, const BnRegs& pr, int C, double M,
                                             float eps, float momentum, int update_moving,
                                             float* tbl) {
  const int c = threadIdx.x;
  if (c < C) {
    double s1, s2;
    acc_read(bn.acc, C, c, s1, s2);
    const double dm = s1 / M;
    const double var = fmax(s2 / M - dm * dm, 0.0);
    const float fmu = (float)dm, fvar = (float)var;
    const float rs = rsqrtf(fvar + eps);
    const float sc = pr.g * rs;
    const float sh = pr.b - fmu * sc;
    tbl[c] = sc;
    tbl[64 + c] = sh;
    tbl[128 + c] = fmu;
    tbl[192 + c] = rs;
    if (blockIdx.x == 0) {
      stg(bn.mean + c, fmu);
      stg(bn.rstd + c, rs);
      stg(bn.scale + c, sc);
      stg(bn.shift + c, sh);
      if (update_moving) {
        const float uvar = M > 1.0 ? (float)(var * M / (M - 1.0)) : fvar;
        const float mm = pr.mm, mv = pr.mv;
        stg(bn.mmean + c, mm - (1.f - momentum) * (mm - fmu));
        stg(bn.mvar + c, mv - (1.f - momentum) * (mv - uvar));
      }
    }
  }
  __syncthreads();
}

// backward BN: sums (sum g, sum g*xhat) -> coefficient table [a, k0, k1, scale, shift] x 64
// with dh = a g - b - c xhat (bn_bwd_apply's formula) refactored as a g + k0 + k1 x:
// k1 = -c rstd, k0 = c mean rstd - b (two fmas per element); workgroup 0 writes
// dgamma / dbeta.  Ends with a barrier.
__device__ __forceinline__ void bn_bwd_table(const PrnBn& bn, const BnRegs& pr, int C, float M,
                                             float* tbl) {
  const int c = threadIdx.x;
  if (c < C) {
    double d1, d2;
    acc_read(bn.bacc, C, c, d1, d2);
    const float sg = (float)d1, sgx = (float)d2;
    const float a = pr.g * pr.rstd;
    const float b = a * sg / M, cc = a * sgx / M;
    tbl[c] = a;
    tbl[64 + c] = cc * pr.mean * pr.rstd - b;
    tbl[128 + c] = -cc * pr.rstd;
    tbl[192 + c] = pr.scale;
    tbl[256 + c] = pr.shift;
    if (blockIdx.x == 0) {   // (write-through: the overlap mode's comm stream reads them
      st_sc1_f32(bn.dbeta + c, sg);   //  while this launch still runs)
      st_sc1_f32(bn.dgamma + c, sgx);
    }
  }
  __syncthreads();
}

// the forward table of a BN the forward launch finalized (backward launch: read back)
__device__ __forceinline__ void bn_load_table(const PrnBn& bn, int C, float* tbl) {
  const int c = threadIdx.x;
  if (c < C) {
    const float rs = ldg(bn.rstd + c);
    tbl[c] = ldg(bn.scale + c);
    tbl[64 + c] = ldg(bn.shift + c);
    tbl[128 + c] = -ldg(bn.mean + c) * rs;   // (tab_store's layout)
    tbl[192 + c] = rs;
  }
}

// one value of the BN-backward output a g + k0 + k1 x, g = da [x*scale+shift > 0]
// (bn_bwd_table's coefficients cf)
__device__ __forceinline__ float bwd1(float da, float xf, const float* cf, int c) {
  const float gg = fmaf(xf, cf[192 + c], cf[256 + c]) > 0.f ? da : 0.f;
  return fmaf(cf[128 + c], xf, fmaf(cf[c], gg, cf[64 + c]));
}
// 8 values (+ add)
__device__ __forceinline__ bf16x8 bwd8(bf16x8 da, bf16x8 x, bf16x8 add, bool has_add,
                                       const float* cf, int c0) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float r = bwd1((float)da[j], (float)x[j], cf, c0 + j);
    if (has_add) r += (float)add[j];
    o[j] = (bf16)r;
  }
  return o;
}

// ---- LDS carve-up (bytes) ------------------------------------------------------------
constexpr int HALO_B = (32 + 2) * 34 * 16 * 2;            // P = 1: the whole 32x32x16 map
constexpr int W1_B = 64 * kpad_of(576) * 2;               // 64 rows x 9*64 (+pad)
constexpr int W2_B = 64 * kpad_of(32) * 2;                // projection (64 x 32 fwd / 32 x 64 dgrad)
constexpr int TBL_B = 7 * 64 * 4;
constexpr int RED_B = 8 * 128 * 4;
constexpr int MISC_B = 256;
constexpr int OFF_HA = 0, OFF_HB = OFF_HA + HALO_B, OFF_W1 = OFF_HB + HALO_B,
              OFF_W2 = OFF_W1 + W1_B, OFF_TBL = OFF_W2 + W2_B, OFF_TBL2 = OFF_TBL + TBL_B,
              OFF_RED = OFF_TBL2 + TBL_B, OFF_MISC = OFF_RED + RED_B,
              LDS_TOTAL = OFF_MISC + MISC_B;
static_assert(LDS_TOTAL <= 163840, "LDS");

struct Smem {
  bf16 *ha, *hb, *w1, *w2;
  float *tbl, *tbl2, *red;
  int* flag;
};
__device__ __forceinline__ Smem carve(char* s) {
  Smem m;
  m.ha = reinterpret_cast<bf16*>(s + OFF_HA);
  m.hb = reinterpret_cast<bf16*>(s + OFF_HB);
  m.w1 = reinterpret_cast<bf16*>(s + OFF_W1);
  m.w2 = reinterpret_cast<bf16*>(s + OFF_W2);
  m.tbl = reinterpret_cast<float*>(s + OFF_TBL);
  m.tbl2 = reinterpret_cast<float*>(s + OFF_TBL2);
  m.red = reinterpret_cast<float*>(s + OFF_RED);
  m.flag = reinterpret_cast<int*>(s + OFF_MISC);
  return m;
}

// round accumulators (+ optional bf16 residual) to bf16 registers
template <int S, int P, bool RES>
__device__ __forceinline__ void round_acc(bf16x4 (&o)[8], const f32x4 (&acc)[8], const bf16x4 (&res)[8]) {
#pragma unroll
  for (int t = 0; t < Stg<S, P>::TPW; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) o[t][r] = (bf16)(RES ? acc[t][r] + (float)res[t][r] : acc[t][r]);
}

template <int S_, int STR_, bool PROJ_>
struct BlkTag {
  static constexpr int S = S_, STR = STR_;
  static constexpr bool PROJ = PROJ_;
};

struct Ctx {
  const PrnArgs* a;
  Smem m;
  int img, kslice, wave, lane;
  unsigned nbar;     // barriers passed
  unsigned slices;   // barrier arrivals per barrier (N x P)
  int pc;            // probe stamps written
  BnRegs bnr;        // prefetched BN parameters of the next combine
  BnRegs ftr;        // backward: prefetched forward table of the next BN-backward sums
  unsigned* mark;    // overlap mode, workgroup 0: bucket line its next arrive counts on
};

// diagnostics: workgroup 0's lane 0 records (tag, wall clock) pairs (prn_set_probe)
__device__ __forceinline__ void probe(Ctx& x, int tag) {
  if (x.a->probe != nullptr) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      x.a->probe[2 * x.pc] = tag;
      x.a->probe[2 * x.pc + 1] = wall_clock64();
    }
    ++x.pc;
  }
}

__device__ __forceinline__ bool wait_fwd(Ctx& x) {
  ++x.nbar;
  if (x.a->fault_bar == (int)x.nbar && blockIdx.x == 0) {   // tests: a lost workgroup
    if (threadIdx.x == 0) __hip_atomic_store(x.a->err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return grid_wait(x.a->bar, PRN_FWD, x.nbar, x.slices, x.a->shards, x.a->err, x.m.flag);
}
// Backward: slice workgroup 0 republishes every completed barrier as a count on its own
// line (bar + PRN_READY): the ~190 weight-gradient workgroups poll that line instead of
// the arrival shards the slices' atomics go to.
// backward arrive; workgroup 0 then also counts a finished bucket of BatchNorm gradients
// (x.mark), ordered after the arrive's drain of its write-through dgamma / dbeta stores
__device__ __forceinline__ void arrive_bwd(Ctx& x) {
  grid_arrive(x.a->bar + PRN_BWD, x.a->shards);
  if (x.mark != nullptr) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(x.mark, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x.mark = nullptr;
  }
}
__device__ __forceinline__ bool wait_bwd(Ctx& x) {
  ++x.nbar;
  const bool ok = grid_wait(x.a->bar, PRN_BWD, x.nbar, x.slices, x.a->shards, x.a->err, x.m.flag);
  if (ok && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(x.a->bar + PRN_READY, x.nbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ok;
}

// =====================================================================================
// forward
// =====================================================================================
template <int S, int P>
__device__ __forceinline__ void fwd_sums(Ctx& x, const bf16x4 (&v)[8], int bi, int wave, int lane) {
  bn_sums<S, P>([&](int t, int r, float& s1, float& s2) {
    const float f = (float)v[t][r];
    s1 = f;
    s2 = f * f;
  }, x.m.red, ld_const(x.a->bns + (bi)).acc, wave, lane);
}

// prefetch registers for the next block's conv1 after a stage-S block (stage S or S+1)
template <int S>
__host__ __device__ constexpr int nreg_next_fwd() {
  return S < 2 ? cmax(nreg(conv_units(16 << S, 16 << S, 3)), nreg(conv_units(32 << S, 16 << S, 3)))
               : nreg(conv_units(64, 64, 3));
}

// BN + ReLU of the published raw tensor `src` (stage S, this image) into halo `hal`: own
// values from registers, neighbour rows from src (sc1 loads issued first), table from
// the BN's accumulators (bnr prefetched).  Ends with a barrier.
template <int S, int P>
__device__ __forceinline__ void fwd_bn_halo(Ctx& x, bf16* hal, const bf16x4 (&v)[8],
                                            const bf16* src, int bi, int wave, int lane) {
  using G = Stg<S, P>;
  const PrnArgs& a = *x.a;
  const Nbr<S, P> nb(x.kslice);
  bf16x8 nv = {};
  if ((int)threadIdx.x < Nbr<S, P>::UNITS && nb.ok) nv = ld_sc1_b128(src, nb.gofs);
  bn_fwd_table(ld_const(a.bns + (bi)), x.bnr, G::C, (double)a.N * G::R * G::R, a.eps, a.momentum,
               a.update_moving, x.m.tbl);
  if ((int)threadIdx.x < Nbr<S, P>::UNITS && nb.ok)
    nv = affine_relu8(nv, x.m.tbl + nb.u * 8, x.m.tbl + 64 + nb.u * 8);
  to_halo<S, P, 1>(hal, v, x.m.tbl, x.m.tbl + 64, nb, nv, x.kslice, wave, lane);
}

// One building block, output stage S; STR 2: transition (input stage S-1, projection);
// PROJ with STR 1: stage-0 block 0 (1x1 stride-1 projection).  On entry W1 (W2) hold
// conv1's (the projection's) weights and x.bnr the block's BN1 parameters; on exit the
// next block's.
template <int S, int STR, bool PROJ, int P>
__device__ __forceinline__ bool block_fwd(Ctx& x, bf16x4 (&xr)[8], int bi_next,
                                          const WLoad& next_w1, const WLoad& next_wp,
                                          const PrnBlock& B) {
  constexpr int SI = STR == 2 ? S - 1 : S;
  using GI = Stg<SI, P>;
  using G = Stg<S, P>;
  const PrnArgs& a = *x.a;
  const int wave = opaque_s(x.wave), lane = opaque_v(x.lane);
  const long img_o = (long)x.img * G::R * G::R * G::C;
  const long img_i = (long)x.img * GI::R * GI::R * GI::C;
  probe(x, 100 + S);
  // BN1 + ReLU of the block input -> halo A (input stage)
  fwd_bn_halo<SI, P>(x, x.m.ha, xr, B.x + img_i, B.bn1, wave, lane);
  probe(x, 1);
  __syncthreads();
  probe(x, 2);
  bf16x4 pr[8], hr[8];
  f32x4 acc[8];
  if constexpr (PROJ) {
    zero_acc(acc);
    conv_acc<S, P, GI::C, 1, STR, false>(acc, x.m.ha, x.m.w2, x.kslice, wave, lane, x.m.red);
    round_acc<S, P, false>(pr, acc, pr);
  }
  zero_acc(acc);
  conv_acc<S, P, GI::C, 3, STR, false>(acc, x.m.ha, x.m.w1, x.kslice, wave, lane, x.m.red);
  round_acc<S, P, false>(hr, acc, hr);
  probe(x, 3);
  // Inside this launch only the neighbouring slices read the saved tensor, and only its
  // border rows: those are published before the arrive; the rest (read by the backward
  // launch) is stored after it, its drain overlapping the barrier wait.
  if constexpr (P > 1) publish<S, P, 1>(hr, B.h1 + img_o, x.kslice, wave, lane);
  fwd_sums<S, P>(x, hr, B.bn2, wave, lane);
  probe(x, 4);
  grid_arrive(a.bar + PRN_FWD, a.shards);
  publish<S, P, P == 1 ? 0 : 2, true>(hr, B.h1 + img_o, x.kslice, wave, lane);
  probe(x, 5);
  {
    bf16x8 w2r[nreg(conv_units(G::C, G::C, 3))];
    const WLoad L2 = wl_fwd(B.w2f, G::C, G::C, 3);
    w_prefetch(L2, w2r);
    bn_prefetch_fwd(ld_const(a.bns + (B.bn2)), G::C, x.bnr);
    if (!wait_fwd(x)) return false;
    probe(x, 6);
    // BN2 + ReLU -> halo A, conv2 (+ residual)
    fwd_bn_halo<S, P>(x, x.m.ha, hr, B.h1 + img_o, B.bn2, wave, lane);
    w_store(L2, w2r, x.m.w1);
  }
  __syncthreads();
  probe(x, 8);
  zero_acc(acc);
  conv_acc<S, P, G::C, 3, 1, false>(acc, x.m.ha, x.m.w1, x.kslice, wave, lane, x.m.red);
  if constexpr (PROJ) round_acc<S, P, true>(xr, acc, pr);
  else round_acc<S, P, true>(xr, acc, xr);
  probe(x, 9);
  if constexpr (P > 1) publish<S, P, 1>(xr, B.out + img_o, x.kslice, wave, lane);
  fwd_sums<S, P>(x, xr, bi_next, wave, lane);
  probe(x, 10);
  grid_arrive(a.bar + PRN_FWD, a.shards);
  publish<S, P, P == 1 ? 0 : 2, true>(xr, B.out + img_o, x.kslice, wave, lane);
  probe(x, 11);
  bf16x8 w1r[nreg_next_fwd<S>()], wpr[1];
  w_prefetch(next_w1, w1r);
  w_prefetch(next_wp, wpr);
  bn_prefetch_fwd(ld_const(a.bns + (bi_next)), G::C, x.bnr);   // the next BN normalizes this output
  if (!wait_fwd(x)) return false;
  probe(x, 12);
  w_store(next_w1, w1r, x.m.w1);   // visible after the next block's first __syncthreads
  w_store(next_wp, wpr, x.m.w2);
  return true;
}

template <int P>
__device__ __forceinline__ void prn_forward_body(const PrnArgs& a, char* smem) {
  using G0 = Stg<0, P>;
  Ctx x;
  x.a = &a;
  x.m = carve(smem);
  x.img = blockIdx.x / P;
  x.kslice = blockIdx.x % P;
  x.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  x.lane = threadIdx.x & 63;
  x.nbar = 0;
  x.slices = (unsigned)(a.N * P);
  x.pc = 0;
  x.mark = nullptr;
  const int tid = threadIdx.x;
  probe(x, 0);

  // ---- stem: 3x3 8 -> 16 on the 32x32 image (no BN before it): the slice's rows plus
  //      one halo row above and below straight from the input ----
  {
    const bf16* src = a.x_in + (long)x.img * 1024 * 8;
    for (int q = tid; q < G0::HR * 34; q += PT) {
      const int lr = q / 34, lc = q - lr * 34;
      const int gr = x.kslice * G0::RS + lr - 1, gc = lc - 1;
      bf16x8 v = {};
      if (gr >= 0 && gr < 32 && gc >= 0 && gc < 32)
        v = *reinterpret_cast<const bf16x8*>(src + (gr * 32 + gc) * 8);
      *reinterpret_cast<bf16x8*>(x.m.ha + q * 8) = v;
    }
    constexpr int SKP = kpad_of(72);
    for (int q = tid; q < 16 * (SKP / 8); q += PT) {
      const int row = q / (SKP / 8), j = q - row * (SKP / 8);
      bf16x8 v = {};
      if (j < 9) v = *reinterpret_cast<const bf16x8*>(a.stem_w + row * 72 + j * 8);
      *reinterpret_cast<bf16x8*>(x.m.w1 + row * SKP + j * 8) = v;
    }
    __syncthreads();
  }
  const PrnBlock& B0 = ld_const(a.blocks + (0));
  bf16x4 xr[8];
  {
    f32x4 acc[8];
    zero_acc(acc);
    conv_acc<0, P, 8, 3, 1, false>(acc, x.m.ha, x.m.w1, x.kslice, x.wave, x.lane, x.m.red);
    round_acc<0, P, false>(xr, acc, xr);
    if constexpr (P > 1) publish<0, P, 1>(xr, B0.x + (long)x.img * 1024 * 16, x.kslice, x.wave, x.lane);
    fwd_sums<0, P>(x, xr, B0.bn1, x.wave, x.lane);
    grid_arrive(a.bar + PRN_FWD, a.shards);
    publish<0, P, P == 1 ? 0 : 2, true>(xr, B0.x + (long)x.img * 1024 * 16, x.kslice, x.wave, x.lane);
    const WLoad L1 = wl_fwd(B0.w1f, 16, 16, 3);
    WLoad LP{};
    if (B0.wpf) LP = wl_fwd(B0.wpf, 16, 16, 1);
    bf16x8 w1r[nreg(conv_units(16, 16, 3))], wpr[1];
    w_prefetch(L1, w1r);
    w_prefetch(LP, wpr);
    bn_prefetch_fwd(ld_const(a.bns + (B0.bn1)), 16, x.bnr);
    if (!wait_fwd(x)) return;
    w_store(L1, w1r, x.m.w1);
    w_store(LP, wpr, x.m.w2);
  }

  // ---- blocks: per stage a transition block then identity blocks (straight-line
  //      stages, no per-block switch: one register allocation region per variant) ----
  const int nps = a.nblocks / 3;   // blocks per stage
  auto run = [&](auto tag, int bi) -> bool {
    constexpr int S = decltype(tag)::S, STR = decltype(tag)::STR;
    constexpr bool PROJ = decltype(tag)::PROJ;
    const PrnBlock& B = ld_const(a.blocks + (bi));
    const bool last = bi + 1 == a.nblocks;
    const int bnx = last ? 2 * a.nblocks : ld_const(a.blocks + (bi + 1)).bn1;
    WLoad n1{}, np{};
    if (!last) {
      const PrnBlock& Bn = ld_const(a.blocks + (bi + 1));
      const int so = Bn.stage, si = Bn.stride == 2 ? so - 1 : so;
      n1 = wl_fwd(Bn.w1f, 16 << so, 16 << si, 3);
      if (Bn.wpf) np = wl_fwd(Bn.wpf, 16 << so, 16 << si, 1);
    }
    return block_fwd<S, STR, PROJ, P>(x, xr, bnx, n1, np, B);
  };
  if (!run(BlkTag<0, 1, true>{}, 0)) return;
  for (int bi = 1; bi < nps; ++bi)
    if (!run(BlkTag<0, 1, false>{}, bi)) return;
  if (!run(BlkTag<1, 2, true>{}, nps)) return;
  for (int bi = nps + 1; bi < 2 * nps; ++bi)
    if (!run(BlkTag<1, 1, false>{}, bi)) return;
  if (!run(BlkTag<2, 2, true>{}, 2 * nps)) return;
  for (int bi = 2 * nps + 1; bi < 3 * nps; ++bi)
    if (!run(BlkTag<2, 1, false>{}, bi)) return;

  // ---- head (head.hip head_fused numerics): final BN + ReLU, the slice's average-pool
  //      sums (fp64 atomics per image), one barrier; then slice 0 of each image: dense,
  //      softmax cross-entropy row, dense dgrad, pool gradient ----
  probe(x, 200);
  using G2 = Stg<2, P>;
  const int fb = 2 * a.nblocks;
  const int dunits = 64 * a.kpad / 8;
  bf16x8 dwv = {};
  if (x.kslice == 0 && tid < dunits) dwv = *reinterpret_cast<const bf16x8*>(a.dense_w + tid * 8);
  bn_fwd_table(ld_const(a.bns + (fb)), x.bnr, 64, (double)a.N * 64, a.eps, a.momentum, a.update_moving, x.m.tbl);
  const float* tbl = x.m.tbl;
  {
    const int wave = opaque_s(x.wave), lane = opaque_v(x.lane);
    if (wave_active<2, P>(wave)) {
      float s[G2::CBW][4];
#pragma unroll
      for (int j = 0; j < G2::CBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[j][r] = 0.f;
#pragma unroll
      for (int t = 0; t < G2::TPW; ++t) {
        int pb, cb;
        tile_of<2, P>(wave, t, pb, cb);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb * 16 + 4 * (lane >> 4) + r;
          s[t % G2::CBW][r] += fmaxf((float)xr[t][r] * tbl[c] + tbl[64 + c], 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < G2::CBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[j][r] = row16_sum(s[j][r]);
      if ((lane & 15) == 0) {
        int pb, cb0;
        tile_of<2, P>(wave, 0, pb, cb0);
#pragma unroll
        for (int j = 0; j < G2::CBW; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) x.m.red[wave * 128 + (cb0 + j) * 16 + 4 * (lane >> 4) + r] = s[j][r];
      }
    }
    __syncthreads();
    if (tid < 64) {
      const int grp = (tid / 16) / G2::CBW;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w)
        if (w % G2::WPB == grp) v += x.m.red[w * 128 + tid];
      atomic_add_g(a.pool_acc + (long)x.img * 64 + tid, (double)v);
    }
  }
  grid_arrive(a.bar + PRN_FWD, a.shards);
  if (!wait_fwd(x)) return;
  if (x.kslice != 0) return;
  float* pool_s = x.m.tbl2;          // [0, 64) pooled, [64, 128) dp, [128, 192) g
  float* wd = reinterpret_cast<float*>(x.m.w1);   // dense weights as fp32 [64][kpad]
  if (tid < dunits)
#pragma unroll
    for (int j = 0; j < 8; ++j) wd[tid * 8 + j] = (float)dwv[j];
  if (tid < 64) {
    const bf16 pb = (bf16)((float)ld_sc1_d(a.pool_acc + (long)x.img * 64 + tid) / 64.f);
    a.pooled[(long)x.img * 64 + tid] = pb;
    pool_s[tid] = (float)pb;
  }
  __syncthreads();
  if (x.wave == 0) {
    const int lane = x.lane;
    const int y = a.labels[x.img];
    float z = -INFINITY;
    if (lane < a.classes) {
      float acc = 0.f;
#pragma unroll 8
      for (int c = 0; c < 64; ++c) acc += pool_s[c] * wd[c * a.kpad + lane];
      z = acc + a.dense_b[lane];
    }
    float mx = z;
    int amax = lane < a.classes ? lane : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {   // first max on ties, like tf.argmax
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(amax, o, 64);
      if (om > mx || (om == mx && oa < amax)) {
        mx = om;
        amax = oa;
      }
    }
    const float se = wave_sum(lane < a.classes ? __expf(z - mx) : 0.f);
    const float lse = mx + __logf(se);
    const float zy = __shfl(z, (y >= 0 && y < a.classes) ? y : 0, 64);
    float g = 0.f;
    if (lane < a.classes) g = (__expf(z - lse) - (lane == y ? 1.f : 0.f)) * a.grad_scale;
    if (lane < a.kpad) {
      const bf16 gb = (bf16)g;
      a.dlogits[(long)x.img * a.kpad + lane] = gb;
      a.ws[(long)x.img * a.kpad + lane] = g;
      pool_s[128 + lane] = (float)gb;
    }
    if (lane == 0) {
      float* rs = a.ws + (long)a.N * a.kpad + 2 * x.img;
      rs[0] = lse - ((y >= 0 && y < a.classes) ? zy : lse);
      rs[1] = (amax == y) ? 1.f : 0.f;
    }
  }
  __syncthreads();
  if (tid < 64) {
    float d = 0.f;
    for (int k = 0; k < a.kpad; ++k) d += pool_s[128 + k] * wd[tid * a.kpad + k];
    const float db = (float)(bf16)d;
    a.dpool[(long)x.img * 64 + tid] = (float)(bf16)(db * (1.f / 64.f));
  }
}

}  // namespace

template <int P>
__global__ void __launch_bounds__(PT, 1) prn_fwd_kernel(PrnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  prn_forward_body<P>(a, smem);
}

// =====================================================================================
// backward
// =====================================================================================
namespace {

// sums of g = da [xs*scale+shift > 0] and g * xhat with the forward table tb
template <int S, int P>
__device__ __forceinline__ void bwd_sums(Ctx& x, const bf16x4 (&da)[8], const bf16x4 (&xs)[8],
                                         const float* tb, int bi, int wave, int lane) {
  lane = opaque_v(lane);
  bn_sums<S, P>([&](int t, int r, float& s1, float& s2) {
    int pb, cb;
    tile_of<S, P>(wave, t, pb, cb);
    const int c = cb * 16 + 4 * (lane >> 4) + r;
    const float xf = (float)xs[t][r];
    const float gg = (xf * tb[c] + tb[64 + c] > 0.f) ? (float)da[t][r] : 0.f;
    s1 = gg;
    s2 = gg * fmaf(xf, tb[192 + c], tb[128 + c]);   // (tb[128] = -mean * rstd)
  }, x.m.red, ld_const(x.a->bns + (bi)).bacc, wave, lane);
}

// dh = a g - b - c xhat (+ add) with the backward coefficient table cf
template <int S, int P, bool ADD>
__device__ __forceinline__ void bwd_apply(bf16x4 (&out)[8], const bf16x4 (&da)[8],
                                          const bf16x4 (&xs)[8], const bf16x4 (&add)[8],
                                          const float* cf, int wave, int lane) {
  lane = opaque_v(lane);
  if (!wave_active<S, P>(wave)) return;
#pragma unroll
  for (int t = 0; t < Stg<S, P>::TPW; ++t) {
    int pb, cb;
    tile_of<S, P>(wave, t, pb, cb);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = cb * 16 + 4 * (lane >> 4) + r;
      float o = bwd1((float)da[t][r], (float)xs[t][r], cf, c);
      if (ADD) o += (float)add[t][r];
      out[t][r] = (bf16)o;
    }
  }
}

// The halo of a BN-backward output (stage S) for the next dgrad: own values from
// registers; the neighbour rows recomputed here from what the neighbours published
// before the barrier -- da (their dgrad output; nullptr: the per-channel constant dpc,
// the pooled head's gradient), the BN input xsrc (saved by the forward) and the residual
// gradient add (nullptr: none) -- with the coefficient table cf.  The loads are issued
// (bwd_nbr_issue) right after the barrier wait, before the BN-backward combine, so the
// two round trips overlap.
struct NbrBwd {
  bf16x8 dv, xv, av;
};
template <int S, int P>
__device__ __forceinline__ void bwd_nbr_issue(const Nbr<S, P>& nb, const bf16* da,
                                              const bf16* xsrc, const bf16* add, NbrBwd& q) {
  if ((int)threadIdx.x < Nbr<S, P>::UNITS && nb.ok) {
    q.dv = da ? ld_sc1_b128(da, nb.gofs) : bf16x8{};
    q.xv = ldg(reinterpret_cast<const bf16x8*>(xsrc + nb.gofs));
    q.av = add ? ld_sc1_b128(add, nb.gofs) : bf16x8{};
  }
}
template <int S, int P>
__device__ __forceinline__ void bwd_halo(Ctx& x, bf16* hal, const bf16x4 (&own)[8],
                                         const Nbr<S, P>& nb, NbrBwd& q, const float* dpc,
                                         bool has_add, const float* cf, int wave, int lane) {
  bf16x8 nv = {};
  if ((int)threadIdx.x < Nbr<S, P>::UNITS && nb.ok) {
    if (dpc) {
#pragma unroll
      for (int j = 0; j < 8; ++j) q.dv[j] = (bf16)dpc[nb.u * 8 + j];
    }
    nv = bwd8(q.dv, q.xv, q.av, has_add, cf, nb.u * 8);
  }
  to_halo<S, P, 0>(hal, own, nullptr, nullptr, nb, nv, x.kslice, wave, lane);
}

// One block's backward: dout (stage S) in registers and its halo in HB, the saved BN2
// input `hs` in registers, conv2's dgrad weights in W1, BN2's forward table in x.ftr;
// out: dx (input stage) in `dout`, its halo in HB, and for the previous block `Bn`
// (has_prev false: none) its conv2 dgrad weights (`next_w2`) in W1, its BN2 input in `hs`, its
// BN2 forward table in x.ftr.  Every global load on the critical path is issued a phase
// ahead (before a barrier wait, or before the halo work).
template <int S, int STR, bool PROJ, int P>
__device__ __forceinline__ bool block_bwd(Ctx& x, bf16x4 (&dout)[8], bf16x4 (&hs)[8],
                                          const WLoad& next_w2, bool has_prev,
                                          const PrnBlock& Bn, const PrnBlock& B) {
  constexpr int SI = STR == 2 ? S - 1 : S;
  using GI = Stg<SI, P>;
  using G = Stg<S, P>;
  const PrnArgs& a = *x.a;
  const int wave = opaque_s(x.wave), lane = opaque_v(x.lane);
  const long img_o = (long)x.img * G::R * G::R * G::C;
  const long img_i = (long)x.img * GI::R * GI::R * GI::C;
  probe(x, 100 + S);
  bf16x4 xs[8];
  load_regs<SI, P>(xs, B.x + img_i, x.kslice, wave, lane);     // BN1 input (used after a barrier)
  tab_store(x.ftr, G::C, x.m.tbl);
  __syncthreads();
  probe(x, 1);
  f32x4 acc[8];
  zero_acc(acc);
  conv_acc<S, P, G::C, 3, 1, true>(acc, x.m.hb, x.m.w1, x.kslice, wave, lane, x.m.red);
  bf16x4 da[8];
  round_acc<S, P, false>(da, acc, da);
  probe(x, 3);
  if constexpr (P > 1)   // only the neighbouring slices read it, only its border rows
    publish<S, P, 1>(da, B.da2 + img_o, x.kslice, wave, lane);
  bwd_sums<S, P>(x, da, hs, x.m.tbl, B.bn2, wave, lane);
  probe(x, 4);
  arrive_bwd(x);
  // dout for the conv2 / projection weight gradients and the neighbours' residual rows:
  // stored after this arrive and the next phase's prefetches (its drain overlaps the
  // wait), drained by the next arrive; from its halo in HB as whole 16-B units (the
  // fragments' 8-B write-through stores left partial lines: bs128 0.749 -> 0.733 ms,
  // bs16 0.557 -> 0.550)
  {
    const WLoad L1 = wl_dgrad(B.w1b, G::C, GI::C, 3);
    WLoad LP{};
    if (PROJ) LP = wl_dgrad(B.wpb, G::C, GI::C, 1);
    bf16x8 w1r[nreg(conv_units(G::C, GI::C, 3))], wpr[1];
    w_prefetch(L1, w1r);
    w_prefetch(LP, wpr);
    bn_prefetch_bwd(ld_const(a.bns + (B.bn2)), G::C, x.bnr);
    bn_prefetch_tab(ld_const(a.bns + (B.bn1)), GI::C, x.ftr);
    halo_to_global<S, P>(x.m.hb, B.dout + img_o, x.kslice);
    probe(x, 5);
    if (!wait_bwd(x)) return false;
    probe(x, 6);
    const Nbr<S, P> nb(x.kslice);
    NbrBwd q;
    bwd_nbr_issue<S, P>(nb, B.da2 + img_o, B.h1 + img_o, nullptr, q);
    bn_bwd_table(ld_const(a.bns + (B.bn2)), x.bnr, G::C, (float)a.N * G::R * G::R, x.m.tbl2);
    bf16x4 dh[8];
    bwd_apply<S, P, false>(dh, da, hs, dh, x.m.tbl2, wave, lane);
    bwd_halo<S, P>(x, x.m.ha, dh, nb, q, nullptr, false, x.m.tbl2, wave, lane);
    tab_store(x.ftr, GI::C, x.m.tbl);
    w_store(L1, w1r, x.m.w1);
    w_store(LP, wpr, x.m.w2);
  }
  __syncthreads();
  probe(x, 8);
  zero_acc(acc);
  if constexpr (STR == 2) {
    dgrad_s2_acc<SI, P, G::C, false>(acc, x.m.ha, x.m.w1, x.kslice, wave, lane);
    dgrad_s2_acc<SI, P, G::C, true>(acc, x.m.hb, x.m.w2, x.kslice, wave, lane);
  } else {
    conv_acc<S, P, G::C, 3, 1, true>(acc, x.m.ha, x.m.w1, x.kslice, wave, lane, x.m.red);
    if constexpr (PROJ) conv_acc<S, P, G::C, 1, 1, false>(acc, x.m.hb, x.m.w2, x.kslice, wave, lane, x.m.red);
  }
  round_acc<SI, P, false>(da, acc, da);
  probe(x, 9);
  if constexpr (P > 1)   // only the neighbouring slices read it, only its border rows
    publish<SI, P, 1>(da, B.da1 + img_i, x.kslice, wave, lane);
  bwd_sums<SI, P>(x, da, xs, x.m.tbl, B.bn1, wave, lane);
  probe(x, 10);
  arrive_bwd(x);
  // dh1 for the conv1 weight gradient, from its halo (HA, intact until the next block
  // stages its own): stored after this arrive, drained by the next one
  halo_to_global<S, P>(x.m.ha, B.dh1 + img_o, x.kslice);
  probe(x, 11);
  bf16x8 w2r[nreg(conv_units(G::C, G::C, 3))];
  w_prefetch(next_w2, w2r);
  bn_prefetch_bwd(ld_const(a.bns + (B.bn1)), GI::C, x.bnr);
  if (has_prev) bn_prefetch_tab(ld_const(a.bns + (Bn.bn2)), GI::C, x.ftr);
  if (!wait_bwd(x)) return false;
  probe(x, 12);
  const Nbr<SI, P> nb(x.kslice);
  NbrBwd q;
  bwd_nbr_issue<SI, P>(nb, B.da1 + img_i, B.x + img_i, PROJ ? nullptr : B.dout + img_o, q);
  bn_bwd_table(ld_const(a.bns + (B.bn1)), x.bnr, GI::C, (float)a.N * GI::R * GI::R, x.m.tbl2);
  probe(x, 13);
  // a stage's first block is the last one the backward reaches: its BN1 gradient completes
  // the stage's BatchNorm gradients (overlap mode: counted on the stage's bucket line)
  if (PROJ && a.overlap && blockIdx.x == 0 && a.bucket_of_stage[S] >= 0)
    x.mark = a.bar + PRN_BUCKET + a.bucket_of_stage[S] * PRN_LINE;
  if constexpr (PROJ) bwd_apply<SI, P, false>(dout, da, xs, dout, x.m.tbl2, wave, lane);
  else bwd_apply<SI, P, true>(dout, da, xs, dout, x.m.tbl2, wave, lane);
  probe(x, 14);
  if (has_prev) load_regs<SI, P>(hs, Bn.h1 + img_i, x.kslice, wave, lane);   // previous block's BN2 input
  // the halo of dx for the previous block's conv2 dgrad (its neighbour rows: this block's
  // published da1, the saved block input, and -- identity blocks -- the published dout)
  bwd_halo<SI, P>(x, x.m.hb, dout, nb, q, nullptr, !PROJ, x.m.tbl2, wave, lane);
  probe(x, 15);
  w_store(next_w2, w2r, x.m.w1);   // visible after the next block's first __syncthreads
  return true;
}

// ---- weight-gradient items ---------------------------------------------------------------
// dW[co][tap][ci] = sum_{images, p} dy[p][co] * A[p @ tap][ci], A = relu(bn(x)) (or x):
// per image, dy [Ro^2][CO] and the A halo [(Ri+2)^2][CI] go to LDS pixel-major; MFMA
// fragments by the transposed read ds_read_b64_tr_b16 (conv_wgrad_direct.hip's scheme);
// waves = WT tile groups x (8 / WT) pixel slices, summed in LDS in a fixed order.
template <int CO, int CI, int KSZ, int STR, int RO, int WT>
__device__ __forceinline__ void wgrad_item(const PrnItem& it, char* smem, int wave, int lane, bool wt) {
  constexpr int RI = RO * STR, W2 = RI + 2, OFF = KSZ == 1 ? 1 : 0;
  constexpr int KN = KSZ * KSZ * CI, NB = (KN + 15) / 16, MB = CO / 16;
  constexpr int TILES = MB * NB, TPW = TILES / WT, WKS = NW / WT;
  constexpr int KSI = RO * RO / 32, KPW = KSI / WKS;   // k-steps per image / per wave
  static_assert(TILES % WT == 0 && KSI % WKS == 0 && TPW <= 36, "wgrad tiles");
  static_assert(NB % TPW == 0, "a wave's tiles share one output-channel block");
  bf16* dys = reinterpret_cast<bf16*>(smem);                    // [RO*RO][CO]
  bf16* hal = dys + RO * RO * CO;                               // [W2*W2][CI]
  float* tb = reinterpret_cast<float*>(hal + W2 * W2 * CI);     // [2][64]
  const int tid = threadIdx.x;
  wave = opaque_s(wave);
  lane = opaque_v(lane);
  const int tg = wave % WT, kq = wave / WT;
  const int gq = lane >> 4, li = lane & 15, qr = li >> 2, pc = li & 3;
  if (it.scale != nullptr && tid < CI) {
    tb[tid] = ldg(it.scale + tid);
    tb[64 + tid] = ldg(it.shift + tid);
  }
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // operands of image n + 1 are loaded into registers while image n's MFMAs run
  constexpr int DU = RO * RO * CO / 8, CU = CI / 8, XU = W2 * W2 * CU;
  constexpr int ND = (DU + PT - 1) / PT, NX = (XU + PT - 1) / PT;
  bf16x8 rd[ND], rx[NX];
  auto fetch = [&](int n) {
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int q = tid + i * PT;
      if (q < DU) rd[i] = ld_sc1_b128(it.dy, (long)n * RO * RO * CO + q * 8);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int q = tid + i * PT, pix = q / CU, u = q - pix * CU;
      const int hr = pix / W2, hc = pix - hr * W2;
      rx[i] = bf16x8{};
      if (q < XU && hr >= 1 && hr <= RI && hc >= 1 && hc <= RI)
        rx[i] = ldg(reinterpret_cast<const bf16x8*>(it.x + (((long)n * RI + hr - 1) * RI + hc - 1) * CI + u * 8));
    }
  };
  const int nend = it.img0 + it.nimg;
  fetch(it.img0);
  for (int n = it.img0; n < nend; ++n) {
    __syncthreads();   // the previous image's operands are dead; tb written
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int q = tid + i * PT;
      if (q < DU) *reinterpret_cast<bf16x8*>(dys + q * 8) = rd[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int q = tid + i * PT, pix = q / CU, u = q - pix * CU;
      const int hr = pix / W2, hc = pix - hr * W2;
      if (q < XU) {
        bf16x8 v = rx[i];
        if (it.scale != nullptr && hr >= 1 && hr <= RI && hc >= 1 && hc <= RI)
          v = affine_relu8(v, tb + u * 8, tb + 64 + u * 8);
        *reinterpret_cast<bf16x8*>(hal + pix * CI + u * 8) = v;
      }
    }
    __syncthreads();
    if (n + 1 < nend) fetch(n + 1);
#pragma unroll 1
    for (int kk = 0; kk < KPW; ++kk) {
      const int ks = kq * KPW + kk;
      const int r1 = ks * 32 + 4 * gq + qr, r2 = r1 + 16;     // output pixels of this lane
      int hp[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int p = e ? r2 : r1, oh = p / RO, ow = p - oh * RO;
        hp[e] = (oh * STR + OFF) * W2 + ow * STR + OFF;
      }
      const int mbw = (tg * TPW) / NB;                            // this wave's channel block
      bf16x8 af;
      {
        const s16x4 lo = lds_read_tr16(dys + r1 * CO + mbw * 16 + 4 * pc);
        const s16x4 hi = lds_read_tr16(dys + r2 * CO + mbw * 16 + 4 * pc);
        af = __builtin_bit_cast(bf16x8, (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int nb = (tg * TPW + t) % NB;
        const int col = nb * 16 + 4 * pc;                         // (tap, ci) of this lane's address
        int tap = col / CI;
        const int ci = col - tap * CI;
        tap = tap < KSZ * KSZ ? tap : KSZ * KSZ - 1;
        const int toff = (tap / KSZ) * W2 + tap % KSZ;
        const s16x4 lo = lds_read_tr16(hal + (hp[0] + toff) * CI + ci);
        const s16x4 hi = lds_read_tr16(hal + (hp[1] + toff) * CI + ci);
        const bf16x8 bfr =
            __builtin_bit_cast(bf16x8, (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        acc[t] = mfma16(af, bfr, acc[t]);
      }
    }
  }
  // fixed-order tree sum of the WKS pixel slices (slice kq += slice kq + h, h = WKS/2 .. 1;
  // each level writes a fresh LDS region, so one barrier per level), then the slab
  float* red = reinterpret_cast<float*>(smem);
  static_assert((WKS - 1) * TILES * 64 * 16 <= OFF_MISC, "wgrad reduction LDS");
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int h = WKS / 2; h >= 1; h /= 2) {
    if (kq >= h && kq < 2 * h)
#pragma unroll
      for (int t = 0; t < TPW; ++t)
        *reinterpret_cast<f32x4*>(red + (((base + kq - h) * TILES + tg * TPW + t) * 64 + lane) * 4) = acc[t];
    __syncthreads();
    if (kq < h)
#pragma unroll
      for (int t = 0; t < TPW; ++t)
        acc[t] += *reinterpret_cast<const f32x4*>(red + (((base + kq) * TILES + tg * TPW + t) * 64 + lane) * 4);
    base += h;
  }
  if (kq == 0) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = tg * TPW + t, mb = tile / NB, nb = tile - mb * NB;
      const int n = nb * 16 + li;
      if (n < KN) {
        if (wt) {   // overlap mode: read by the comm stream while the launch runs
#pragma unroll
          for (int i = 0; i < 4; ++i) st_sc1_f32(it.part + (long)(mb * 16 + 4 * gq + i) * KN + n, acc[t][i]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) stg(it.part + (long)(mb * 16 + 4 * gq + i) * KN + n, acc[t][i]);
        }
      }
    }
  }
  __syncthreads();
}

constexpr int PRN_KINDS = 9;
// LDS of the weight-gradient role per kind: dy + halo + table
__host__ __device__ constexpr int wg_lds(int co, int ci, int str, int ro) {
  return ro * ro * co * 2 + (ro * str + 2) * (ro * str + 2) * ci * 2 + 512;
}

__device__ __forceinline__ void run_item(const PrnItem& it, char* smem, int wave, int lane, bool wt) {
  switch (it.kind) {
    case 0: wgrad_item<16, 16, 3, 1, 32, 1>(it, smem, wave, lane, wt); break;   // stage-0 3x3
    case 1: wgrad_item<32, 32, 3, 1, 16, 2>(it, smem, wave, lane, wt); break;   // stage-1 3x3
    case 2: wgrad_item<64, 64, 3, 1, 8, 8>(it, smem, wave, lane, wt); break;    // stage-2 3x3
    case 3: wgrad_item<32, 16, 3, 2, 16, 2>(it, smem, wave, lane, wt); break;   // 3x3/2 16->32
    case 4: wgrad_item<64, 32, 3, 2, 8, 8>(it, smem, wave, lane, wt); break;    // 3x3/2 32->64
    case 5: wgrad_item<16, 16, 1, 1, 32, 1>(it, smem, wave, lane, wt); break;   // 1x1 16->16
    case 6: wgrad_item<32, 16, 1, 2, 16, 2>(it, smem, wave, lane, wt); break;   // 1x1/2 16->32
    case 7: wgrad_item<64, 32, 1, 2, 8, 8>(it, smem, wave, lane, wt); break;    // 1x1/2 32->64
    case 8: wgrad_item<16, 8, 3, 1, 32, 1>(it, smem, wave, lane, wt); break;    // stem 8->16
    default: break;
  }
}


}  // namespace

// The slice role of the backward launch: the dgrad chain with its BatchNorm backwards
// (returns false when a barrier wait timed out).
template <int P>
__device__ __forceinline__ bool prn_bwd_slices(const PrnArgs& a, char* smem, int wave, int lane) {
  const int nsl = a.N * P;
  const int tid = threadIdx.x;
  Ctx x;
  x.a = &a;
  x.m = carve(smem);
  x.img = blockIdx.x / P;
  x.kslice = blockIdx.x % P;
  x.wave = wave;
  x.lane = lane;
  x.nbar = 0;
  x.slices = (unsigned)nsl;
  x.pc = 0;
  x.mark = nullptr;
  probe(x, 0);
  const int nb = a.nblocks;
  const PrnBlock& BL = ld_const(a.blocks + (nb - 1));
  {   // the last block's conv2 dgrad weights (stage 2: 64 x 576)
    const WLoad L = wl_dgrad(BL.w2b, 64, 64, 3);
    bf16x8 r[nreg(conv_units(64, 64, 3))];
    w_prefetch(L, r);
    w_store(L, r, x.m.w1);
  }
  // ---- final BN backward: sums of g = dpool * relu'(bn(XL)), one barrier, then
  //      dXL = a g - b - c xhat and its halo ----
  using G2 = Stg<2, P>;
  bf16x4 dout[8], hs[8];
  {
    const int fb = 2 * nb;
    const long img_o = (long)x.img * 64 * 64;
    bf16x4 xs[8];
    load_regs<2, P>(xs, BL.out + img_o, x.kslice, wave, lane);
    float* dps = x.m.tbl + 256;   // this image's dpool row
    bn_load_table(ld_const(a.bns + (fb)), 64, x.m.tbl);
    if (tid < 64) dps[tid] = a.dpool[(long)x.img * 64 + tid];
    __syncthreads();
    bf16x4 dp[8];
#pragma unroll
    for (int t = 0; t < G2::TPW; ++t) {
      int pb, cb;
      tile_of<2, P>(wave, t, pb, cb);
#pragma unroll
      for (int r = 0; r < 4; ++r) dp[t][r] = (bf16)dps[(cb * 16 + 4 * (lane >> 4) + r) & 63];
    }
    bwd_sums<2, P>(x, dp, xs, x.m.tbl, fb, wave, lane);
    arrive_bwd(x);
    bn_prefetch_bwd(ld_const(a.bns + (fb)), 64, x.bnr);
    bn_prefetch_tab(ld_const(a.bns + (BL.bn2)), 64, x.ftr);
    if (!wait_bwd(x)) return false;
    const Nbr<2, P> nb(x.kslice);
    NbrBwd q;
    bwd_nbr_issue<2, P>(nb, nullptr, BL.out + img_o, nullptr, q);
    bn_bwd_table(ld_const(a.bns + (fb)), x.bnr, 64, (float)a.N * 64, x.m.tbl2);
    bwd_apply<2, P, false>(dout, dp, xs, dout, x.m.tbl2, wave, lane);
    load_regs<2, P>(hs, BL.h1 + img_o, x.kslice, wave, lane);
    bwd_halo<2, P>(x, x.m.hb, dout, nb, q, dps, false, x.m.tbl2, wave, lane);
  }
  // ---- blocks, last to first (straight-line stages, as in the forward) ----
  const int nps = nb / 3;
  auto run = [&](auto tag, int bi) -> bool {
    constexpr int S = decltype(tag)::S, STR = decltype(tag)::STR;
    constexpr bool PROJ = decltype(tag)::PROJ;
    WLoad n2{};
    const bool hp = bi > 0;
    const PrnBlock Bp = ld_const(a.blocks + (hp ? bi - 1 : bi));
    if (hp) n2 = wl_dgrad(Bp.w2b, 16 << Bp.stage, 16 << Bp.stage, 3);
    return block_bwd<S, STR, PROJ, P>(x, dout, hs, n2, hp, Bp, ld_const(a.blocks + (bi)));
  };
  for (int bi = nb - 1; bi > 2 * nps; --bi)
    if (!run(BlkTag<2, 1, false>{}, bi)) return false;
  if (!run(BlkTag<2, 2, true>{}, 2 * nps)) return false;
  for (int bi = 2 * nps - 1; bi > nps; --bi)
    if (!run(BlkTag<1, 1, false>{}, bi)) return false;
  if (!run(BlkTag<1, 2, true>{}, nps)) return false;
  for (int bi = nps - 1; bi > 0; --bi)
    if (!run(BlkTag<0, 1, false>{}, bi)) return false;
  if (!run(BlkTag<0, 1, true>{}, 0)) return false;
  probe(x, 200);
  // ---- the stem output's gradient: published for the stem's weight gradient ----
  if constexpr (P == 1) {   // from its halo (block_bwd's dout store)
    __syncthreads();
    halo_to_global<0, P>(x.m.hb, a.dx0 + (long)x.img * 1024 * 16, x.kslice);
  } else {
    publish<0, P>(dout, a.dx0 + (long)x.img * 1024 * 16, x.kslice, wave, lane);
  }
  arrive_bwd(x);
  if (blockIdx.x == 0) wait_bwd(x);   // publishes the stem item's readiness
  return true;
}

// The head's batch folds in one workgroup, launched on the main stream right after the
// backward launch: the loss / precision / bias-gradient folds of
// softmax_xent_reduce_kernel (head.hip, same thread mapping and order) and the dense
// weight gradient pooled^T x dlogits (bf16 operands staged in LDS, fp32 sums over the
// images in order).  These were a side-stream softmax_xent_reduce + conv_wgrad pair
// whose fork and join events cost ~11 us per step between the launches.  (Run by the
// backward launch's first weight-gradient workgroup instead, this code perturbed the
// register allocation of the whole backward kernel: 76 -> 272 B of scratch per lane,
// +55 us per step.)
__device__ void prn_head_fold(const PrnArgs& a, char* smem, int tid) {
  const int N = a.N, ld = a.kpad, classes = a.classes;
  // every operand into LDS with one round of 16-byte loads: the fp32 gradient rows and
  // the per-image (loss, correct) pairs of the softmax workspace, pooled [N][64] and
  // dlogits [N][ld] (bf16); rows of 64 and ld (% 16) elements are whole 16-B chunks,
  // the pair block goes in 8-byte pieces
  float* red = reinterpret_cast<float*>(smem);           // [4][64]
  float* sw = red + 256;                                  // [N][ld] + [N][2]
  bf16* sp = reinterpret_cast<bf16*>(sw + ((N * ld + 2 * N + 3) & ~3));   // 16-B aligned
  bf16* sd = sp + N * 64;
  for (int i = tid; i < N * ld / 4; i += PT)
    reinterpret_cast<f32x4*>(sw)[i] = ldg(reinterpret_cast<const f32x4*>(a.ws) + i);
  for (int i = tid; i < N; i += PT)
    reinterpret_cast<float2*>(sw + N * ld)[i] = ldg(reinterpret_cast<const float2*>(a.ws + N * ld) + i);
  for (int i = tid; i < N * 8; i += PT)
    reinterpret_cast<uint4*>(sp)[i] = ldg(reinterpret_cast<const uint4*>(a.pooled) + i);
  for (int i = tid; i < N * ld / 8; i += PT)
    reinterpret_cast<uint4*>(sd)[i] = ldg(reinterpret_cast<const uint4*>(a.dlogits) + i);
  __syncthreads();
  const int lane = tid & 63, q = tid >> 6;
  if (q < 4) {   // bias gradient: thread (class, row slice q) sums rows q, q + 4, ...
    float t = 0.f;
    if (lane < classes) {
#pragma unroll 8
      for (int r = q; r < N; r += 4) t += sw[r * ld + lane];
    }
    red[q * 64 + lane] = t;
  } else if (q == 4) {   // loss and precision
    const float* rs = sw + N * ld;
    float l = 0.f, k = 0.f;
    for (int r = lane; r < N; r += 64) {
      l += rs[2 * r];
      k += rs[2 * r + 1];
    }
    l = wave_sum(l);
    k = wave_sum(k);
    if (lane == 0) {
      stg(a.loss_sum, l);
      stg(a.correct, k);
    }
  }
  // dense weight gradient: thread (f = tid % 64, image chunk tid / 64 of 8) holds 16
  // classes' sums in registers over its images (the dlogits row is a broadcast LDS read),
  // the 8 chunk partials are added in chunk order through LDS.  (One thread per output
  // over all images ran 10-14 us: ~2.5k LDS instructions queued on this one CU.)
  static_assert(PT == 512, "8 image chunks of 64 threads");
  float* part = reinterpret_cast<float*>(sd + ((N * ld + 7) & ~7));   // [8][64][16]
  {
    const int f = tid & 63, c = tid >> 6;
    const int n0 = (N * c) >> 3, n1 = (N * (c + 1)) >> 3;
    for (int k0 = 0; k0 < classes; k0 += 16) {   // ld % 16 == 0: k0 + 15 < ld
      float acc[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      for (int n = n0; n < n1; ++n) {
        const float x = (float)sp[n * 64 + f];
        const bf16* drow = sd + n * ld + k0;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] += x * (float)drow[j];
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) part[(c * 64 + f) * 16 + j] = acc[j];
      __syncthreads();
      for (int o = tid; o < 64 * 16; o += PT) {
        const int ff = o >> 4, j = o & 15;
        if (k0 + j < classes) {
          float t = part[ff * 16 + j];
#pragma unroll
          for (int cc = 1; cc < 8; ++cc) t += part[(cc * 64 + ff) * 16 + j];
          stg(a.dense_grad + ff * classes + k0 + j, t);   // HWIO [64][classes]
        }
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (q == 0 && lane < classes)
    stg(a.dbias + lane, red[lane] + red[64 + lane] + red[128 + lane] + red[192 + lane]);
}

template <int P>
__global__ void __launch_bounds__(PT, 1) prn_bwd_kernel(PrnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if ((int)blockIdx.x < a.N * P && !prn_bwd_slices<P>(a, smem, wave, lane)) return;
  // ---- weight-gradient items from one queue in readiness order: the workgroups beyond
  //      the slices from the start, every slice once its dgrad chain is done (the last
  //      items -- the first stage and the stem -- only become ready at the very end) ----
  int* flag = reinterpret_cast<int*>(smem + OFF_MISC);
  int* slot = flag + 1;
  for (;;) {
    __syncthreads();   // the previous item's LDS and the slot word are free
    if (tid == 0)
      *slot = (int)__hip_atomic_fetch_add(a.bar + PRN_QUEUE, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int i = __builtin_amdgcn_readfirstlane(*slot);
    if (i >= a.nitems) {
      if (a.probe != nullptr && tid == 0)   // diagnostics: when the last workgroup ran out of items
        __hip_atomic_fetch_max(a.probe + 8191, (long long)wall_clock64(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    const PrnItem& it = ld_const(a.items + i);
    if (!count_wait<8>(a.bar, PRN_READY, (unsigned)it.ready, a.err, flag)) return;
    run_item(it, smem, wave, lane, a.overlap != 0);
    if (a.overlap && it.bucket >= 0) {   // the slab's write-through stores drained, then counted
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(a.bar + PRN_BUCKET + it.bucket * PRN_LINE, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// comm-stream bucket wait (overlap mode): lane 0 polls the bucket line (bounded)
__global__ void __launch_bounds__(64) prn_bucket_wait_kernel(unsigned* bar, int bucket, unsigned target,
                                                            int* err) {
  if (threadIdx.x != 0) return;
  const unsigned* ctr = bar + PRN_BUCKET + bucket * PRN_LINE;
  const long long t0 = wall_clock64();
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(4);
    if (wall_clock64() - t0 > kSpinTicks) {
      __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}

__global__ void __launch_bounds__(PT, 1) prn_head_kernel(PrnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  prn_head_fold(a, smem, threadIdx.x);
}

// ---- host ------------------------------------------------------------------------------
static long long* g_prn_probe = nullptr;
void prn_set_probe(long long* p) { g_prn_probe = p; }

int device_cus() { return cu_count(); }
std::vector<uint32_t> device_cu_mask() { return cu_mask_words(); }

size_t prn_lds_bytes() { return LDS_TOTAL; }
int prn_bar_words() { return PRN_BAR_WORDS; }
int prn_acc_rep() { return PRN_ACC_REP; }

bool prn_supported(int N, int P, int nblocks, int classes, int kpad) {
  return N >= 1 && (P == 1 || P == 2 || P == 4) && N * P <= 256 && nblocks >= 3 && nblocks % 3 == 0 &&
         classes >= 1 && classes <= kpad && kpad <= 64 && kpad % 16 == 0;
}

int prn_item_kind(int cin, int cout, int ksize, int stride) {
  if (cin == 8 && cout == 16 && ksize == 3 && stride == 1) return 8;
  if (ksize == 3 && stride == 1 && cin == cout) return cin == 16 ? 0 : cin == 32 ? 1 : cin == 64 ? 2 : -1;
  if (ksize == 3 && stride == 2) return cin == 16 && cout == 32 ? 3 : cin == 32 && cout == 64 ? 4 : -1;
  if (ksize == 1 && stride == 1 && cin == 16 && cout == 16) return 5;
  if (ksize == 1 && stride == 2) return cin == 16 && cout == 32 ? 6 : cin == 32 && cout == 64 ? 7 : -1;
  return -1;
}

static_assert(wg_lds(16, 16, 1, 32) <= LDS_TOTAL && wg_lds(32, 16, 2, 16) <= LDS_TOTAL &&
                  wg_lds(16, 8, 1, 32) <= LDS_TOTAL,
              "weight-gradient LDS");

// Arrival shards of a launch whose barriers N x P slices arrive at.  Auto (tune -1): 64
// (about two arrivals per line) when 128 or more slices of at most half an image each
// arrive together, else 8 -- more lines cost every poll (one load per line) and pay only
// where the arrivals cluster.  Same-process A/B, step ms, 8 / 32 / 64 shards (scripts/
// tune_ab.py): bs16 0.5573 / 0.5592 / 0.5598, bs32 0.5764 / 0.5710 / 0.5676, bs64 0.6439
// / 0.6434 / 0.6409, bs128 (one slice per image) 0.7332 / 0.7323 / 0.7351.
static int prn_shards(int N, int P) {
  const long t = tune(T_PRN_SHARDS);
  if (t == 1 || t == 8 || t == 16 || t == 32 || t == 64) return (int)t;
  return N * P >= 128 && P >= 2 ? 64 : 8;
}

static size_t prn_head_lds(int N, int kpad) {
  return 1024 + 32 + (size_t)N * ((64 + kpad) * sizeof(bf16) + (kpad + 2) * sizeof(float)) +
         8 * 64 * 16 * sizeof(float);
}

// workgroups of `kern` (PT threads, `lds` bytes) the device keeps resident at once
template <typename K>
static long resident_blocks(K kern, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, PT, lds) != hipSuccess) return -1;
  return (long)per_cu * cu_count();
}

std::string prn_check(int N, int P, int P_fwd, int nblocks, int classes, int kpad) {
  if (!prn_supported(N, P, nblocks, classes, kpad) || !prn_supported(N, P_fwd, nblocks, classes, kpad))
    return "unsupported shape (slices 1/2/4, N x slices <= 256, 3n blocks, classes <= kpad <= 64)";
  const int cus = cu_count();
  if (N * P_fwd > cus) return "forward grid (N x slices) exceeds the CUs";
  if (N * P + 1 > cus) return "backward grid (N x slices + weight-gradient workgroups) exceeds the CUs";
  if (N > 240 || prn_head_lds(N, kpad) > LDS_TOTAL) return "head folds: batch too large for LDS";
  // co-residency: every workgroup of a grid must be resident at once (grid barriers)
  const long rf = P_fwd == 1 ? resident_blocks(prn_fwd_kernel<1>, LDS_TOTAL)
                  : P_fwd == 2 ? resident_blocks(prn_fwd_kernel<2>, LDS_TOTAL)
                               : resident_blocks(prn_fwd_kernel<4>, LDS_TOTAL);
  const long rb = P == 1 ? resident_blocks(prn_bwd_kernel<1>, LDS_TOTAL)
                  : P == 2 ? resident_blocks(prn_bwd_kernel<2>, LDS_TOTAL)
                           : resident_blocks(prn_bwd_kernel<4>, LDS_TOTAL);
  if (rf < 0 || rb < 0) return "occupancy query failed";
  if (rf < (long)N * P_fwd) return "forward grid not co-resident (occupancy API)";
  if (rb < (long)N * P + 1) return "backward grid not co-resident (occupancy API)";
  return "";
}

void prn_forward(const PrnArgs& a, hipStream_t s) {
  if (!prn_supported(a.N, a.P, a.nblocks, a.classes, a.kpad) || a.N * a.P > cu_count())
    throw std::invalid_argument("prn_forward: unsupported shape (N x P <= CUs, 3n blocks, <= 64 classes)");
  PrnArgs b = a;
  b.probe = g_prn_probe;
  b.shards = prn_shards(a.N, a.P);
  if (a.P == 1) hipLaunchKernelGGL(prn_fwd_kernel<1>, dim3(a.N), dim3(PT), LDS_TOTAL, s, b);
  else if (a.P == 2) hipLaunchKernelGGL(prn_fwd_kernel<2>, dim3(a.N * 2), dim3(PT), LDS_TOTAL, s, b);
  else hipLaunchKernelGGL(prn_fwd_kernel<4>, dim3(a.N * 4), dim3(PT), LDS_TOTAL, s, b);
  DTR_CHECK_LAUNCH();
}

void prn_head(const PrnArgs& a, hipStream_t s) {
  if (!prn_supported(a.N, a.P, a.nblocks, a.classes, a.kpad) || a.N > 240 || !a.dense_grad ||
      !a.loss_sum || !a.correct || !a.dbias)
    throw std::invalid_argument("prn_head: unsupported shape or missing outputs");
  const size_t lds = prn_head_lds(a.N, a.kpad);
  if (lds > LDS_TOTAL) throw std::invalid_argument("prn_head: batch too large for LDS");
  hipLaunchKernelGGL(prn_head_kernel, dim3(1), dim3(PT), lds, s, a);
  DTR_CHECK_LAUNCH();
}

void prn_bucket_wait(unsigned* bar, int bucket, unsigned target, int* err, hipStream_t s) {
  if (bucket < 0 || bucket >= PRN_NBUCKET || bar == nullptr || err == nullptr)
    throw std::invalid_argument("prn_bucket_wait: bucket 0..2, bar and err required");
  hipLaunchKernelGGL(prn_bucket_wait_kernel, dim3(1), dim3(64), 0, s, bar, bucket, target, err);
  DTR_CHECK_LAUNCH();
}

void prn_backward(const PrnArgs& a, int wgrad_wgs, hipStream_t s) {
  if (!prn_supported(a.N, a.P, a.nblocks, a.classes, a.kpad))
    throw std::invalid_argument("prn_backward: unsupported shape");
  const int grid = a.N * a.P + std::max(1, wgrad_wgs);
  if (grid > cu_count())
    throw std::invalid_argument("prn_backward: the grid must be co-resident (<= one per CU)");
  PrnArgs b = a;
  b.probe = g_prn_probe;
  b.shards = prn_shards(a.N, a.P);
  if (a.P == 1) hipLaunchKernelGGL(prn_bwd_kernel<1>, dim3(grid), dim3(PT), LDS_TOTAL, s, b);
  else if (a.P == 2) hipLaunchKernelGGL(prn_bwd_kernel<2>, dim3(grid), dim3(PT), LDS_TOTAL, s, b);
  else hipLaunchKernelGGL(prn_bwd_kernel<4>, dim3(grid), dim3(PT), LDS_TOTAL, s, b);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
