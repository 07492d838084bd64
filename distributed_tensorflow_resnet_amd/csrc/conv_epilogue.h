// Shared conv epilogue (implicit-GEMM conv_gemm.hip and direct conv_direct.hip).
#pragma once
#include "bn_fused.h"
#include "common.h"
#include "kernels.h"

namespace dtr {

enum { F_PRE = 1, F_STATS = 2, F_BNB = 4, F_ABWD = 8 };

// The epilogue's thread index: 256 threads per tile (a 512-thread kernel may run two
// epilogues side by side, one per half of its tile, each on its own LDS, with SYNC_ALL).
__device__ __forceinline__ int ep_tid() { return (int)(threadIdx.x & 255); }

// Epilogue staging: PR rows of the fp32 tile at a time -- the whole tile when
// it fits in 64 KiB (one phase), else one wave-row per phase (128x128 tiles).
template <int BM, int BN, int WM>
struct EpiLayout {
  static constexpr int LDC = BN + 4;              // fp32 staging row stride (floats)
  static constexpr int CPR = BN / 8;              // 8-channel chunks per row
  static constexpr int RPP = 256 / CPR;           // rows per pass
  // reduction planes: colsum8's 4 wave totals per column, or the last-arriver /
  // prologue combines' (256 / BN) slices per column -- whichever is larger
  static constexpr int REDP = (4 * BN > 256) ? 4 * BN : 256;
  static constexpr int RED = 2 * REDP + BN;       // floats (two reduction planes + means)
  static constexpr int PHASES = ((BM * LDC + RED) * 4 <= 64 * 1024) ? 1 : WM;
  static constexpr int PR = BM / PHASES;          // rows staged per phase
  static constexpr int TILE = PR * LDC;           // floats
  static constexpr size_t BYTES = (size_t)(TILE + RED) * sizeof(float);
};

// Last-arriver combines (bn_fused.h protocol).  Thread (c = tid % BN, q = tid / BN)
// loads items q, q + G, ... (G = 256 / BN; the host keeps cnt <= G * FIN_UNROLL so
// every load is in flight at once), folds them, then thread q == 0 of each column
// folds the G partial results from LDS in fixed order -> deterministic.  Results
// are valid in threads tid < BN (column n0 + tid).
//   welford_combine: items are (mean, M2) pairs at src[i * 2NC + col] / [+ NC]; item
//                    i of the range holds min(rows_per, rows_left - i * rows_per) rows.
//   sum_combine:     items are (sum1, sum2) pairs, added.
template <int BN>
__device__ __forceinline__ void welford_combine(const float* src, int NC, int n0, int first,
                                                int cnt, int rows_per, int rows_left,
                                                float* red, float* red2, float* red3,
                                                float& out_n, float& out_mu, float& out_m2) {
  constexpr int G = 256 / BN;
  const int tid = ep_tid(), c = tid % BN, q = tid / BN, col = n0 + c;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (col < NC) {
    float mv[FIN_UNROLL], qv[FIN_UNROLL];
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const int t = q + u * G;
      const long o = (long)(first + t) * 2 * NC + col;
      mv[u] = t < cnt ? src[o] : 0.f;
      qv[u] = t < cnt ? src[o + NC] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const int t = q + u * G;
      if (t < cnt) {
        const float nb = (float)min(rows_per, rows_left - t * rows_per);
        const float nn = n + nb, d = mv[u] - mu;
        mu += d * nb / nn;
        m2 += qv[u] + d * d * n * nb / nn;
        n = nn;
      }
    }
  }
  red[q * BN + c] = n;
  red2[q * BN + c] = mu;
  red3[q * BN + c] = m2;
  __syncthreads();
  if (q == 0 && col < NC) {
    float fn_ = red[c], fmu = red2[c], fm2 = red3[c];
    for (int k = 1; k < G; ++k) {
      const float nb = red[k * BN + c], mb = red2[k * BN + c], qb = red3[k * BN + c];
      const float nn = fn_ + nb;
      if (nn > 0.f) {
        const float d = mb - fmu;
        fmu += d * nb / nn;
        fm2 += qb + d * d * fn_ * nb / nn;
        fn_ = nn;
      }
    }
    out_n = fn_;
    out_mu = fmu;
    out_m2 = fm2;
  }
}

template <int BN>
__device__ __forceinline__ void sum_combine(const float* src, int NC, int n0, int first, int cnt,
                                            float* red, float* red2, float& o1, float& o2) {
  constexpr int G = 256 / BN;
  const int tid = ep_tid(), c = tid % BN, q = tid / BN, col = n0 + c;
  float a1 = 0.f, a2 = 0.f;
  if (col < NC) {
    float v1[FIN_UNROLL], v2[FIN_UNROLL];
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const int t = q + u * G;
      const long o = (long)(first + t) * 2 * NC + col;
      v1[u] = t < cnt ? src[o] : 0.f;
      v2[u] = t < cnt ? src[o + NC] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      a1 += v1[u];
      a2 += v2[u];
    }
  }
  red[q * BN + c] = a1;
  red2[q * BN + c] = a2;
  __syncthreads();
  if (q == 0 && col < NC) {
    float s1 = 0.f, s2 = 0.f;
    for (int k = 0; k < G; ++k) {
      s1 += red[k * BN + c];
      s2 += red2[k * BN + c];
    }
    o1 = s1;
    o2 = s2;
  }
}

// Column sums of the epilogue's 8-column row vectors: thread (r0 = tid / CPR,
// cc = tid % CPR) holds v[j] for column cc*8+j.  The lanes with equal cc are
// summed by DPP row_ror steps of CPR, 2*CPR, .. within each 16-lane row (VALU, fused
// into v_add_f32_dpp), then two xor shuffles across the four rows, leaving every lane
// with its column's wave total (was: a __shfl_xor tree of log2(64 / CPR) ds_bpermute
// steps per value -> 80-116 per conv, ~1 us of the epilogue,
// profiles/cifar_direct_conv_phases.md).  Lanes < CPR then write the 4 wave totals
// to wred[4][BN] (fixed order, deterministic).  Ends with a barrier; the caller
// adds wred[0..3][col].
template <int OFF>
__device__ __forceinline__ float row_ror_add(float v) {   // v + v of lane (l - OFF) mod 16
  if constexpr (OFF < 16)
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                             0, __builtin_bit_cast(int, v), 0x120 + OFF, 0xf, 0xf,
                                             false));
  return v;
}

// Output row (pixel) of epilogue row `row`: the identity, or for a stride-2 dgrad parity
// class (GemmArgs::par) the class's row-major pixel (n, h0 + 2 hh, w0 + 2 ww).
__device__ __forceinline__ long epi_row(const GemmArgs& a, int row) {
  if (!a.par) return row;
  const int per = a.par_hc * a.par_wc;
  const int n = row / per, rem = row - n * per;
  const int hh = rem / a.par_wc, ww = rem - hh * a.par_wc;
  return ((long)n * a.g.H + a.par_h0 + 2 * hh) * a.g.W + a.par_w0 + 2 * ww;
}

template <int CPR>
__device__ __forceinline__ float lanes_colsum(float v) {
  v = row_ror_add<CPR>(v);
  if constexpr (2 * CPR < 16) v = row_ror_add<2 * CPR>(v);
  if constexpr (4 * CPR < 16) v = row_ror_add<4 * CPR>(v);
  if constexpr (8 * CPR < 16) v = row_ror_add<8 * CPR>(v);
  // the four 16-lane rows: two shuffles.  (v_permlane16/32_swap on two copies of the
  // value does it on the VALU, but a VALU write feeding the swap is a hazard: without
  // wait states a row is silently dropped -- caught by test_conv_fused_prologue_epilogue
  // and test_direct_conv3x3_matches_reference_and_generic.  Inline asm with s_nop 1
  // before each swap passes every test but measured no faster than the shuffles:
  // colsum phase 0.68-0.72 us vs 0.64-0.76, CIFAR bs16 0.946 vs 0.938-0.950 ms.)
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

template <int CPR, int BN>
__device__ __forceinline__ void colsum8(float (&v)[8], float* wred) {
  static_assert(CPR >= 1 && CPR <= 16 && (CPR & (CPR - 1)) == 0, "CPR");
  const int lane = ep_tid() & 63, wave = ep_tid() >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = lanes_colsum<CPR>(v[j]);
  if (lane < CPR) {
#pragma unroll
    for (int j = 0; j < 8; ++j) wred[wave * BN + lane * 8 + j] = v[j];
  }
  lds_barrier();   // LDS-only: the caller's global stores stay in flight
}

// Two column sums (8 columns per thread each) behind ONE barrier.
template <int CPR, int BN>
__device__ __forceinline__ void colsum8x2(float (&v)[8], float (&w)[8], float* wred,
                                          float* wred2) {
  static_assert(CPR >= 1 && CPR <= 16 && (CPR & (CPR - 1)) == 0, "CPR");
  const int lane = ep_tid() & 63, wave = ep_tid() >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = lanes_colsum<CPR>(v[j]);
    w[j] = lanes_colsum<CPR>(w[j]);
  }
  if (lane < CPR) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wred[wave * BN + lane * 8 + j] = v[j];
      wred2[wave * BN + lane * 8 + j] = w[j];
    }
  }
  lds_barrier();
}

// Epilogue operand prefetch (single-phase tiles): the residual / accumulate-into /
// BN-input row vectors each epilogue thread will combine are independent of the
// GEMM, so kernels issue their loads at kernel start (epi_prefetch) and the
// epilogue finds them in registers instead of paying a global round trip.
// XO ("x only"): prefetch just the BN-backward operands (BN input rows + the
// per-column scale/shift/mean/rstd) -- the implicit-GEMM dgrad, whose occupancy
// cannot afford the residual / accumulate registers too.
// Multi-phase tiles (128x128) prefetch only in XO mode: the BN-input rows of every
// phase (RIT * PHASES vectors).  Their occupancy is LDS-bound (2 workgroups per
// CU), so the extra registers are free, while loading them per phase put a global
// round trip into each phase of every tile (~0.1 ms per 56x56 dgrad).
template <int BM, int BN, int WM, bool XO = false>
struct EpiPre {
  using EL = EpiLayout<BM, BN, WM>;
  static constexpr bool ON = EL::PHASES == 1 || XO;
  static constexpr bool X_ONLY = XO;
  static constexpr int RIT = ON ? (EL::PR + EL::RPP - 1) / EL::RPP : 1;   // per phase
  static constexpr int NX = ON ? RIT * EL::PHASES : 1;
  static constexpr int RR = (XO || EL::PHASES > 1) ? 1 : RIT;
  // per-column BN coefficients held from kernel start.  In the multi-phase (128x128)
  // dgrad this pushes the kernel to 256 VGPRs + 24 spilled, yet reading them at the
  // epilogue instead (0 spills) measured 1 % SLOWER on ImageNet RN50 (13.29 -> 13.43
  // ms/step): the spill traffic hides in the K loop, the epilogue round trip does not.
  // The single-phase direct-conv dgrad prefetches them too (reading them at its epilogue
  // cost ~1 us of LDS-staging time per launch, profiles/cifar_direct_conv_phases.md).
  static constexpr bool COEF = XO || EL::PHASES == 1;
  bf16x8 res[RR], acc[RR], x[NX];
  f32x4 bsc[COEF ? 2 : 1], bsh[COEF ? 2 : 1], bmu[COEF ? 2 : 1], brs[COEF ? 2 : 1];
};

template <int BM, int BN, int WM, int FLAGS, bool XO = false>
__device__ __forceinline__ void epi_prefetch(const GemmArgs& args, const int m0, const int n0,
                                             EpiPre<BM, BN, WM, XO>& P) {
  using EL = EpiLayout<BM, BN, WM>;
  using PP = EpiPre<BM, BN, WM, XO>;
  if constexpr (PP::ON) {
    const int tid = ep_tid();
    const int cc = tid % EL::CPR, r0 = tid / EL::CPR;
    const int col0 = n0 + cc * 8;
    const bf16x8 zero8 = {};
#pragma unroll
    for (int ph = 0; ph < EL::PHASES; ++ph)
#pragma unroll
      for (int it = 0; it < PP::RIT; ++it) {
        const int row = m0 + ph * EL::PR + r0 + it * EL::RPP;
        const bool ok = col0 < args.Ncol && r0 + it * EL::RPP < EL::PR && row < args.M;
        const long o = epi_row(args, row) * args.Ncol + col0;
        if constexpr (!XO && EL::PHASES == 1) {
          P.res[it] = (ok && args.residual) ? *reinterpret_cast<const bf16x8*>(args.residual + o)
                                            : zero8;
          P.acc[it] = (ok && args.accumulate && !args.out_f32)
                          ? *reinterpret_cast<const bf16x8*>(args.out + o) : zero8;
        }
        if constexpr ((FLAGS & F_BNB) != 0)
          P.x[ph * PP::RIT + it] = ok ? *reinterpret_cast<const bf16x8*>(args.bnb_x + o) : zero8;
      }
    if constexpr (PP::COEF && (FLAGS & F_BNB) != 0) {
      const bool colok = col0 < args.Ncol;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        P.bsc[h] = colok ? *reinterpret_cast<const f32x4*>(args.bnb_scale + col0 + 4 * h) : z;
        P.bsh[h] = colok ? *reinterpret_cast<const f32x4*>(args.bnb_shift + col0 + 4 * h) : z;
        P.bmu[h] = colok ? *reinterpret_cast<const f32x4*>(args.bnb_mean + col0 + 4 * h) : z;
        P.brs[h] = colok ? *reinterpret_cast<const f32x4*>(args.bnb_rstd + col0 + 4 * h) : z;
      }
    }
  }
}

// Split-K combine of the implicit-GEMM loops (conv_gemm.hip FAST, conv_ring.hip):
// slice blockIdx.z of args.ksplit publishes its fp32 tile (write-through, thread-native
// order) and takes a ticket; the last slice of the tile sums all slices in slice order
// (bitwise independent of arrival order) and alone returns true (runs the epilogue).
// 256 threads, wave tile MR x NR fragments of 16x16; the caller's LDS must be dead.
template <int MR, int NR>
__device__ __forceinline__ bool splitk_combine(const GemmArgs& args, f32x4 (&acc)[MR][NR],
                                               char* smem, int tm, int tn, int z) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int tile = tm * gridDim.y + tn;
  const int S = args.ksplit;   // z: this workgroup's (logical) slice
  const long slab = (long)MR * NR * 1024;                 // floats per slice tile
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + (long)tile * S * slab, 0,
                                                    0x7fffffff, 0x00020000);
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b)
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4_t, acc[a][b]), rs,
          (int)((((long)z * slab) + ((long)(a * NR + b) * 256 + tid) * 4) * 4), 0, 16);
  int* flag = reinterpret_cast<int*>(smem);
  if (!last_arriver(args.sk_cnt + tile, (unsigned)S, flag)) return false;
  // sum every slice -- this one's too, read back from the slab it just wrote -- into acc,
  // 0 + s0 + s1 + ... in slice order: the same fp32 sum as a separate total, without
  // holding a second MR x NR register tile beside acc (that spilled the ring dgrad)
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int zz = 0; zz < S; ++zz) {
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b)
        acc[a][b] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
            rs, (int)((((long)zz * slab) + ((long)(a * NR + b) * 256 + tid) * 4) * 4), 0, 16));
  }
  reset_counter(args.sk_cnt + tile);
  __syncthreads();   // the flag word's LDS is the epilogue's
  return true;
}

// Shared epilogue of every conv kernel (implicit-GEMM and direct): the wave
// fragments acc[MR][NR] of the BM x BN tile at (m0, n0) -> LDS-staged 16-byte
// row stores with bias / residual / accumulate, BN statistics (STATS), BN
// backward sums (BNB) and the optional last-arriver finalize.  Entered after a
// workgroup barrier (the caller's LDS is dead).
// SYNC_ALL (two side-by-side epilogues of a 512-thread kernel): every phase runs, rows
// past M included (as no-ops), so both halves pass the same barriers; the caller then
// uses accumulator-mode BN statistics / sums only (no per-tile partial rows, no
// last-arriver finalize).
template <int BM, int BN, int WM, int WN, int FLAGS, bool XO = false, bool SYNC_ALL = false>
__device__ __forceinline__ void conv_epilogue(const GemmArgs& args,
                                              f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                              char* smem, const int m0, const int n0,
                                              const EpiPre<BM, BN, WM, XO>* pre = nullptr,
                                              int tile_m = -1, int tile_n = -1) {
  // (tile_m, tile_n): this workgroup's logical tile when the kernel remaps blockIdx
  // (XCD swizzle, conv_gemm.hip); -1 = blockIdx.x / blockIdx.y.
  if (tile_m < 0) tile_m = blockIdx.x;
  if (tile_n < 0) tile_n = blockIdx.y;
  constexpr bool STATS = (FLAGS & F_STATS) != 0;
  constexpr bool BNB = (FLAGS & F_BNB) != 0;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MR = WTM / 16, NR = WTN / 16;
  const int M = args.M, NC = args.Ncol;
  const int tid = ep_tid();
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;
  // ---------------- epilogue ----------------
  // Processed in EL::PHASES phases of EL::PR rows (1 phase unless the tile is 128x128):
  //  (a) the waves owning those rows write their fragments (+bias) to an fp32 LDS tile
  //      (the K loop ended with a barrier: staging buffers/PRE table are dead);
  //  (b) all 256 threads sweep it as 16-byte row vectors (8 channels per lane):
  //      residual / accumulate, ONE bf16 rounding, 16-B store, BN partials;
  //  (c) STATS: per-phase two-pass (mean, M2) folded across phases with Chan's
  //      formula in fixed order; BNB: sums carried in registers.
  using EL = EpiLayout<BM, BN, WM>;
  float* cs = reinterpret_cast<float*>(smem);
  float* red = cs + EL::TILE;
  float* red2 = red + EL::REDP;
  float* mean_s = red + 2 * EL::REDP;
  const int cc = tid % EL::CPR, r0 = tid / EL::CPR;
  const int col0 = n0 + cc * 8;
  const bool colok = col0 < NC;  // NC % 16 == 0 -> a chunk is all-in or all-out
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  float bnb_t1 = 0.f, bnb_t2 = 0.f;   // BNB column totals (thread tid < BN)
  float bsc[8], bsh[8], bmu[8], brs[8];
  if constexpr (BNB) {
    constexpr bool COEF = EpiPre<BM, BN, WM, XO>::COEF;
    if (COEF && EpiPre<BM, BN, WM, XO>::ON && pre) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bsc[j] = pre->bsc[COEF ? j / 4 : 0][j % 4];
        bsh[j] = pre->bsh[COEF ? j / 4 : 0][j % 4];
        bmu[j] = pre->bmu[COEF ? j / 4 : 0][j % 4];
        brs[j] = pre->brs[COEF ? j / 4 : 0][j % 4];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bsc[j] = colok ? args.bnb_scale[col0 + j] : 0.f;
        bsh[j] = colok ? args.bnb_shift[col0 + j] : 0.f;
        bmu[j] = colok ? args.bnb_mean[col0 + j] : 0.f;
        brs[j] = colok ? args.bnb_rstd[col0 + j] : 0.f;
      }
    }
  }
  float wn_run = 0.f, wmean_run = 0.f, wm2_run = 0.f;  // STATS, thread tid < BN owns column tid

#pragma unroll 1
  for (int ph = 0; ph < EL::PHASES; ++ph) {
    const int prow0 = m0 + ph * EL::PR;
    const int nph = min(EL::PR, M - prow0);   // block-uniform
    if (nph <= 0 && !SYNC_ALL) break;
    // Operand loads of this phase's rows, all issued before the staging writes and
    // the barrier so they overlap them (one round trip, not one per row iteration);
    // kernels that prefetched them at kernel start (EpiPre) skip this.
    // (the BN-input loads of dgrad+BNB; the residual rows too in the multi-phase
    // 128x128 tiles, whose occupancy is LDS-bound anyway -- batching them in the
    // single-phase tiles cost more occupancy than it gained on the ImageNet shapes.)
    constexpr int RIT = (EL::PR + EL::RPP - 1) / EL::RPP;
    constexpr bool PREL = EpiPre<BM, BN, WM, XO>::ON;
    constexpr bool PRER = PREL && !XO;   // single-phase: residual / accumulate rows too
    constexpr bool BATCH = BNB;
    constexpr bool BATCHR = EL::PHASES > 1 && !BNB;   // (BNB: no residual; the registers spill)
    bf16x8 lx[BATCH ? RIT : 1], lr[BATCHR ? RIT : 1];
    if (BATCH && PREL && pre) {   // this phase's prefetched BN-input rows (selects, no indexing)
#pragma unroll
      for (int it = 0; it < RIT; ++it) {
        lx[it] = pre->x[it];
#pragma unroll
        for (int q = 1; q < EL::PHASES; ++q)
          if (ph == q) lx[it] = pre->x[q * RIT + it];
      }
    }
    if (BATCH && !(PREL && pre)) {
#pragma unroll
      for (int it = 0; it < RIT; ++it) {
        const int r = r0 + it * EL::RPP;
        if (!colok || r >= nph) continue;
        const long o = epi_row(args, prow0 + r) * NC + col0;
        if constexpr (BNB) lx[BATCH ? it : 0] = *reinterpret_cast<const bf16x8*>(args.bnb_x + o);
      }
    }
    if (BATCHR && args.residual) {
#pragma unroll
      for (int it = 0; it < RIT; ++it) {
        const int r = r0 + it * EL::RPP;
        const bool ok = colok && r < nph;
        const long o = epi_row(args, prow0 + (ok ? r : 0)) * NC + (ok ? col0 : 0);
        lr[BATCHR ? it : 0] = *reinterpret_cast<const bf16x8*>(args.residual + o);
      }
    }
    if ((wm * WTM) / EL::PR == ph) {
      const int rbase = wm * WTM - ph * EL::PR;
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int cl = wn * WTN + b * 16 + fr;
        const int col = n0 + cl;
        const float bias = (args.bias != nullptr && col < args.nbias) ? args.bias[col] : 0.f;
#pragma unroll
        for (int a = 0; a < MR; ++a)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            cs[(rbase + a * 16 + fq * 4 + i) * EL::LDC + cl] = acc[a][b][i] + bias;
      }
    }
    lds_barrier();
    if (args.probe && tid == 0) args.probe[8 * (tile_m + gridDim.x * tile_n) + 4] = wall_clock64();
    // Pass 1: values of this thread's rows (residual / accumulate, ONE bf16
    // rounding) kept in registers; BN sums accumulated.  Global stores are issued
    // only AFTER the statistics' barriers: a __syncthreads() waits for every
    // outstanding store of the wave (vmcnt(0)), so storing first put a full
    // store round trip in the middle of the epilogue (~2 us per STATS/BNB conv).
    bf16x8 ob[RIT];
    // STATS, one pass of shifted sums: d = y - K with K = the phase's row-0 value of
    // the column (any per-column constant; close to the data, so sum d^2 - (sum d)^2/n
    // does not cancel).  One reduction barrier per phase instead of the two-pass
    // mean-then-M2 (two barriers and a second sweep).
    float p1[8], p2[8], ksh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p1[j] = p2[j] = 0.f;
      ksh[j] = 0.f;
    }
    if constexpr (STATS) {
      if (colok) {
        const f32x4 k0 = *reinterpret_cast<const f32x4*>(cs + cc * 8);
        const f32x4 k1 = *reinterpret_cast<const f32x4*>(cs + cc * 8 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ksh[j] = k0[j];
          ksh[4 + j] = k1[j];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int r = r0 + it * EL::RPP;
      if (!colok || r >= nph) continue;
      const int row = prow0 + r;
      float* cp = cs + r * EL::LDC + cc * 8;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(cp);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(cp + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const long o = epi_row(args, row) * NC + col0;
      if (args.residual) {
        const bf16x8 rv = (PRER && pre) ? pre->res[PRER ? it : 0]
                          : BATCHR      ? lr[BATCHR ? it : 0]
                                        : *reinterpret_cast<const bf16x8*>(args.residual + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += (float)rv[j];
      }
      if (args.out_f32) {   // fp32 output (dense logits): no BN fusion on this path
        float* op = args.out_f32 + o;
        if (args.accumulate) {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(op);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(op + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] += a0[j];
            v[4 + j] += a1[j];
          }
        }
        *reinterpret_cast<f32x4*>(op) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(op + 4) = f32x4{v[4], v[5], v[6], v[7]};
        continue;
      }
      if (args.accumulate) {
        const bf16x8 av = (PRER && pre) ? pre->acc[PRER ? it : 0]
                                        : *reinterpret_cast<const bf16x8*>(args.out + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += (float)av[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ob[it][j] = (bf16)v[j];
        v[j] = (float)ob[it][j];
      }
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[j] - ksh[j];
          p1[j] += d;
          p2[j] += d * d;
        }
      }
      if constexpr (BNB) {
        const bf16x8 xv = BATCH ? lx[BATCH ? it : 0]
                                : *reinterpret_cast<const bf16x8*>(args.bnb_x + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = (float)xv[j];
          const float gg = (xf * bsc[j] + bsh[j] > 0.f) ? v[j] : 0.f;
          s1[j] += gg;
          s2[j] += gg * (xf - bmu[j]) * brs[j];
        }
      }
    }
    // Pass 2: the stores, issued BEFORE the statistics' reductions: those end in
    // lds_barrier()s, which wait for LDS only, so the stores drain while the column
    // sums run (args.wt: write-through sc1 buffer stores, so the tile does not
    // sit dirty in this XCD's L2 for the end-of-kernel release to write back)
    if (!args.out_f32) {
      if (args.wt) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.out, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int it = 0; it < RIT; ++it) {
          const int r = r0 + it * EL::RPP;
          if (!colok || r >= nph) continue;
          typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, ob[it]), rs,
                                                 (int)((epi_row(args, prow0 + r) * NC + col0) * 2), 0,
                                                 16);
        }
      } else {
#pragma unroll
        for (int it = 0; it < RIT; ++it) {
          const int r = r0 + it * EL::RPP;
          if (!colok || r >= nph) continue;
          *reinterpret_cast<bf16x8*>(args.out + epi_row(args, prow0 + r) * NC + col0) = ob[it];
        }
      }
    }
    if (args.probe && tid == 0) args.probe[8 * (tile_m + gridDim.x * tile_n) + 5] = wall_clock64();
    if constexpr (STATS) {
      colsum8x2<EL::CPR, BN>(p1, p2, red, red2);
      if (tid < BN && nph > 0) {
        const float sd = red[tid] + red[BN + tid] + red[2 * BN + tid] + red[3 * BN + tid];
        const float sdd = red2[tid] + red2[BN + tid] + red2[2 * BN + tid] + red2[3 * BN + tid];
        const float nb = (float)nph, dm = sd / nb;
        const float mb = cs[tid] + dm;                 // K of column tid + mean of d
        const float m2 = fmaxf(sdd - sd * dm, 0.f);
        const float n = wn_run + nb;
        const float d = mb - wmean_run;
        wmean_run += d * nb / n;
        wm2_run += m2 + d * d * wn_run * nb / n;
        wn_run = n;
      }
    }
    if constexpr (BNB) {
      if (ph == EL::PHASES - 1 || (!SYNC_ALL && prow0 + EL::PR >= M)) {   // last phase: reduce
        colsum8x2<EL::CPR, BN>(s1, s2, red, red2);   // both sums behind one barrier
        if (tid < BN) {
          bnb_t1 = red[tid] + red[BN + tid] + red[2 * BN + tid] + red[3 * BN + tid];
          bnb_t2 = red2[tid] + red2[BN + tid] + red2[2 * BN + tid] + red2[3 * BN + tid];
        }
      }
    }
    if (args.probe && tid == 0) args.probe[8 * (tile_m + gridDim.x * tile_n) + 6] = wall_clock64();
    // the next phase overwrites the tile (LDS-only: this phase's stores stay in flight)
    if constexpr (EL::PHASES > 1) lds_barrier();
  }

  if constexpr (STATS) {
    if (tid < BN && n0 + tid < NC) {
      float* tile_out = args.stat_part + (long)tile_m * 2 * NC;
      if (args.stat_acc != nullptr) {       // accumulator mode: sum y, sum y^2 of the tile
        const double n = wn_run, mu = wmean_run;
        bn_acc_add(args.stat_acc, NC, n0 + tid, n * mu, (double)wm2_run + n * mu * mu);
      } else if (args.fin.counters != nullptr) {   // handed to the last arriver: write-through (sc1)
        publish_f32(tile_out + n0 + tid, wmean_run);
        publish_f32(tile_out + NC + n0 + tid, wm2_run);
      } else {
        tile_out[n0 + tid] = wmean_run;     // tile mean
        tile_out[NC + n0 + tid] = wm2_run;  // tile M2
      }
    }
    const BnFwdFin& F = args.fin;
    if (F.counters != nullptr) {
      int* flag = reinterpret_cast<int*>(mean_s);
      const int T = gridDim.x;
      bool last;
      float fn_ = 0.f, fmu = 0.f, fm2 = 0.f;
      if (F.group == 0) {          // single level: combine every tile
        last = last_arriver(F.counters + tile_n, T, flag);
        if (last) welford_combine<BN>(args.stat_part, NC, n0, 0, T, BM, M, red, red2, cs,
                                      fn_, fmu, fm2);
      } else {                     // two levels: groups of F.group tiles, then the groups
        const int GS = F.group, ng = (T + GS - 1) / GS, gi = tile_m / GS;
        const int gsize = min(GS, T - gi * GS);
        last = last_arriver(F.counters + gridDim.y + tile_n * ng + gi, gsize, flag);
        if (last) {
          welford_combine<BN>(args.stat_part, NC, n0, gi * GS, gsize, BM, M - gi * GS * BM,
                              red, red2, cs, fn_, fmu, fm2);
          if (tid < BN && n0 + tid < NC) {
            publish_f32(F.gpart + (long)gi * 2 * NC + n0 + tid, fmu);
            publish_f32(F.gpart + (long)gi * 2 * NC + NC + n0 + tid, fm2);
          }
          reset_counter(F.counters + gridDim.y + tile_n * ng + gi);
          if (F.groups_only) {
            last = false;   // a consumer's BnPreFin combines the group partials
          } else {
            last = last_arriver(F.counters + tile_n, ng, flag);
            if (last) welford_combine<BN>(F.gpart, NC, n0, 0, ng, GS * BM, M, red, red2, cs,
                                          fn_, fmu, fm2);
          }
        }
      }
      if (last) {
        const int col = n0 + tid;
        if (tid < BN && col < NC) {
          const float var = fm2 / fn_;
          const float rs = rsqrtf(var + F.eps);
          const float sc = F.gamma[col] * rs;
          F.mean[col] = fmu;
          F.rstd[col] = rs;
          F.scale[col] = sc;
          F.shift[col] = F.beta[col] - fmu * sc;
          if (F.update_moving) {
            const float uvar = fn_ > 1.f ? fm2 / (fn_ - 1.f) : fm2;
            F.mmean[col] -= (1.f - F.momentum) * (F.mmean[col] - fmu);
            F.mvar[col] -= (1.f - F.momentum) * (F.mvar[col] - uvar);
          }
        }
        reset_counter(F.counters + tile_n);
      }
    }
  }
  if constexpr (BNB) {
    if (tid < BN && n0 + tid < NC) {
      const float t1 = bnb_t1, t2 = bnb_t2;
      float* tile_out = args.bnb_part + (long)tile_m * 2 * NC;
      if (args.bnb_acc != nullptr) {        // accumulator mode
        bn_acc_add(args.bnb_acc, NC, n0 + tid, (double)t1, (double)t2);
      } else if (args.bfin.counters != nullptr) {
        publish_f32(tile_out + n0 + tid, t1);
        publish_f32(tile_out + NC + n0 + tid, t2);
      } else {
        tile_out[n0 + tid] = t1;        // sum g
        tile_out[NC + n0 + tid] = t2;   // sum g * xhat
      }
    }
    const BnBwdFin& F = args.bfin;
    if (F.counters != nullptr) {
      int* flag = reinterpret_cast<int*>(mean_s);
      const int T = gridDim.x;
      bool last;
      float sg = 0.f, sgx = 0.f;
      if (F.group == 0) {
        last = last_arriver(F.counters + tile_n, T, flag);
        if (last) sum_combine<BN>(args.bnb_part, NC, n0, 0, T, red, red2, sg, sgx);
      } else {
        const int GS = F.group, ng = (T + GS - 1) / GS, gi = tile_m / GS;
        const int gsize = min(GS, T - gi * GS);
        last = last_arriver(F.counters + gridDim.y + tile_n * ng + gi, gsize, flag);
        if (last) {
          sum_combine<BN>(args.bnb_part, NC, n0, gi * GS, gsize, red, red2, sg, sgx);
          if (tid < BN && n0 + tid < NC) {
            publish_f32(F.gpart + (long)gi * 2 * NC + n0 + tid, sg);
            publish_f32(F.gpart + (long)gi * 2 * NC + NC + n0 + tid, sgx);
          }
          reset_counter(F.counters + gridDim.y + tile_n * ng + gi);
          if (F.groups_only) {
            last = false;   // the consumer dgrad's BnBwdPre combines the group sums
          } else {
            last = last_arriver(F.counters + tile_n, ng, flag);
            if (last) sum_combine<BN>(F.gpart, NC, n0, 0, ng, red, red2, sg, sgx);
          }
        }
      }
      if (last) {
        const int col = n0 + tid;
        if (tid < BN && col < NC) {
          F.dbeta[col] = sg;
          F.dgamma[col] = sgx;
          const float a = F.gamma[col] * F.rstd[col];
          F.coef[col] = a;
          F.coef[NC + col] = a * sg / (float)M;
          F.coef[2 * NC + col] = a * sgx / (float)M;
        }
        reset_counter(F.counters + tile_n);
      }
    }
  }
}

}  // namespace dtr
