// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// Everything here is wave64 / MFMA-first: vector types match the register
// footprint of `v_mfma_f32_16x16x32_bf16` operands (8 x bf16 = 4 VGPRs) and
// accumulators (4 x f32).  No CUDA-compat shims: HIP on gfx950 only.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "tune.h"

namespace dtr {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }  // v_cvt_pk_bf16_f32 (RNE, NaN-safe)

__device__ __forceinline__ float bits2f(unsigned short u) {
  return __uint_as_float(((unsigned)u) << 16);
}

// D = A(16x32) * B(32x16) + C, bf16 inputs, fp32 accumulate.
// Lane l holds A[l&15][8*(l>>4)+j] and B[8*(l>>4)+j][l&15], j=0..7;
// C/D: col = l&15, row = 4*(l>>4)+i.
// XCD-aware block order.  MI355X deals workgroups round-robin over its 8 XCDs (linear
// block b to XCD b % 8, each XCD with its own L2): the logical block of physical block b
// such that every XCD gets one contiguous range of logical blocks, so neighbouring
// logical blocks that share operands share an L2.  Bijective for any grid size
// (cdna_hip_programming.md, "XCD swizzle must be bijective"); placement is a speed
// matter only, never correctness.
__device__ __forceinline__ unsigned xcd_logical_block(unsigned b, unsigned nwg) {
  const unsigned xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// gfx950 transposed LDS read: per 16-lane group, lane 4q+p supplies the address
// of row q, columns 4p..4p+3 of a 4x16 block of 16-bit values; lane i receives
// column i of the 4 rows (row q in element q).
__device__ __forceinline__ s16x4 lds_read_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
}

// Workgroup barrier that orders LDS only: s_waitcnt lgkmcnt(0) + s_barrier.
// __syncthreads() is a release on ALL address spaces, so with global stores in
// flight it also waits vmcnt(0) -- in a multi-phase epilogue that put every
// phase's store round trip on the critical path.  Use where the barrier only
// protects LDS data (staging tiles, reduction planes).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 8 bf16 <-> 8 float with a per-channel affine + ReLU (pre-activation BN fold).
__device__ __forceinline__ bf16x8 affine_relu8(bf16x8 v, const float* sc, const float* sh) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = (float)v[j] * sc[j] + sh[j];
    r[j] = (bf16)(x > 0.f ? x : 0.f);
  }
  return r;
}

// Same op with the 8 channels' scale/shift already in registers (one table read
// per k-step shared by all of a thread's chunks) and packed math: bf16 -> f32 is
// a shift / mask of each 32-bit pair, the affine is v_pk_fma_f32 on float2, the
// ReLU and the RNE bf16 pack (v_cvt_pk_bf16_f32) per pair.  The per-element form
// above cost ~+50 % on ImageNet convs with the fused BN prologue.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16x8 affine_relu8_reg(bf16x8 v, const f32x4& s0, const f32x4& s1,
                                                   const f32x4& b0, const f32x4& b1) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 u = __builtin_bit_cast(u32x4, v);
  const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
  const float sh[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  bf16x8 r;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    f32x2 x = {__uint_as_float(u[p] << 16), __uint_as_float(u[p] & 0xffff0000u)};
    const f32x2 a = {sc[2 * p], sc[2 * p + 1]}, b = {sh[2 * p], sh[2 * p + 1]};
    x = x * a + b;
    r[2 * p] = (bf16)fmaxf(x[0], 0.f);
    r[2 * p + 1] = (bf16)fmaxf(x[1], 0.f);
  }
  return r;
}

// The staging form used beside the MFMAs (FAST loops): scalar FMAs (a packed
// v_pk_fma_f32 costs more than two v_fma_f32 in an MFMA gap, MI355X_MICROARCH
// constants), the RNE pack first and the ReLU on the packed bf16 pair as a signed
// 16-bit max against 0 (bf16 is sign-magnitude: every negative pattern, -0 too, is
// a negative int16) -- one v_pk_max_i16 instead of two v_max_f32, bit-identical --
// then `sel` (all-ones for a real pixel, 0 for padding; padding chunks were loaded
// as zeros by the out-of-range buffer loads) as one AND per dword.
__device__ __forceinline__ bf16x8 affine_relu8_sel(bf16x8 v, const f32x4& s0, const f32x4& s1,
                                                   const f32x4& b0, const f32x4& b1,
                                                   unsigned sel) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const u32x4 u = __builtin_bit_cast(u32x4, v);
  const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
  const float sh[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  u32x4 r;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float lo = fmaf(__uint_as_float(u[p] << 16), sc[2 * p], sh[2 * p]);
    const float hi = fmaf(__uint_as_float(u[p] & 0xffff0000u), sc[2 * p + 1], sh[2 * p + 1]);
    const bf16x2 pk = {(bf16)lo, (bf16)hi};
    const s16x2 m = __builtin_elementwise_max(__builtin_bit_cast(s16x2, pk), (s16x2){0, 0});
    r[p] = __builtin_bit_cast(unsigned, m) & sel;
  }
  return __builtin_bit_cast(bf16x8, r);
}

// Host: conv epilogue / dh stores write-through (sc1).  tune wt_store = 1 forces it on
// for every conv, 0 off; -1 (default): the direct 3x3 convs decide by output size
// (wt_store_direct), the implicit-GEMM / ring convs write through (round 6, RN50 bs128
// step, four interleaved rounds: 10.316-10.325 -> 10.260-10.286 ms -- their outputs are
// read next by kernels on other CUs / XCDs while the side stream's weight gradients
// fill the L2s; CIFAR per-layer bs128 / bs256 and RN101 bs256 unchanged within noise).
inline int wt_store_mode() { return (int)tune(T_WT_STORE); }
inline bool wt_store_enabled() { return wt_store_mode() != 0; }

// Compute units this process may dispatch to on the current device, queried once per
// device (persistent-grid sizing on the launch path without a runtime query per launch):
// the device's CUs, or the set bits of the process-wide CU mask (ROC_GLOBAL_CU_MASK, set
// by parallel/dist.py apply_cu_partition when several ranks split one GPU's CUs) -- the
// null stream's mask is that global mask, every stream of the process inherits it.
inline int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    // (the runtime copies its whole global mask, which may hold more words than the
    // CUs need: a generous buffer)
    uint32_t mask[256] = {0};
    const uint32_t words = (uint32_t)((n + 31) / 32);
    if (words <= 32 && hipExtStreamGetCUMask(nullptr, words, mask) == hipSuccess) {
      int bits = 0;
      for (uint32_t w = 0; w < words; ++w) bits += __builtin_popcount(mask[w]);
      if (bits > 0 && bits < n) n = bits;
    }
    cache[dev] = n;
  }
  return cache[dev];
}
// The process's CU mask on the current device (32-bit words, bit i = CU i).
inline std::vector<uint32_t> cu_mask_words() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return {};
  const size_t words = (n + 31) / 32;
  std::vector<uint32_t> mask(256, 0xA5A5A5A5u);   // generous: see cu_count
  if (hipExtStreamGetCUMask(nullptr, (uint32_t)words, mask.data()) != hipSuccess) return {};
  size_t used = mask.size();   // words the runtime wrote (beyond `words`: diagnostics)
  while (used > words && mask[used - 1] == 0xA5A5A5A5u) --used;
  mask.resize(used);
  return mask;
}
// Direct convs: write-through once a launch writes >= 2 MB.  A kernel boundary pays
// ~bytes / 6 TB/s to write back the dirty lines its predecessor left in L2
// (MI355X_MICROARCH.md "boundary"); write-through stores leave none.  Measured, CIFAR
// RN50 bs128: boundaries 2.4-2.6 -> 1.6-2.1 us, step 1.304 -> 1.282 ms; bs16 / bs64
// (outputs < 2 MB per launch) unchanged.
inline bool wt_store_direct(long out_bytes) {
  const int m = wt_store_mode();
  return m == 1 || (m == -1 && out_bytes >= (2L << 20));
}

}  // namespace dtr

#define DTR_CHECK_LAUNCH()                                                      \
  do {                                                                          \
    hipError_t e__ = hipGetLastError();                                         \
    if (e__ != hipSuccess) {                                                    \
      fprintf(stderr, "HIP launch error %s at %s:%d\n", hipGetErrorString(e__), \
              __FILE__, __LINE__);                                              \
    }                                                                           \
  } while (0)
