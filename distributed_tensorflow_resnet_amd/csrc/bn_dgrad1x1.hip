// Streaming 1x1 data gradient with a narrow reduction (K = 64..256 input rows) fused with
// the BatchNorm+ReLU backward of its wide output, for the first conv of the ImageNet
// identity bottleneck blocks (engine _conv_bwd ``bap``; reference: Conv2DBackpropInput
// followed by FusedBatchNormGrad + ReluGrad, resnet_model_official.py:133-175).
//
//   g[m][c]  = bf16( sum_k dz[m][k] * W[c][k] ) * [x[m][c]*scale[c] + shift[c] > 0]
//   SUMS  : bacc += (sum_m g, sum_m g * (x - mean) * rstd)          (fp64 replicas)
//   APPLY : dx[m][c] = bf16( a[c] g - b[c] - c[c] (x - mean) rstd + add[m][c] )
//   STORE+SUMS (mode 2): the unfused BNB dgrad -- out = the bf16 dgrad, plus SUMS
// Shapes: K = 64..512 narrow-or-wide reductions whose weights fit in VGPRs, over 256-column
// slices of a wide output (the bottlenecks' first conv) or the whole 64 / 128-column output
// (the expanding conv's dgrad at stages 1-2).
//
// Why a separate kernel: as an implicit-GEMM tile with a fat epilogue (conv_gemm.hip /
// conv_ring.hip, F_BNB; an apply-epilogue variant was measured and removed) these passes moved their bytes at 2.1-2.9 TB/s -- each
// 128x128 workgroup loads its operands once, then spends its life in the LDS-staged
// epilogue with nothing in flight -- while the standalone BN-backward apply streams at
// 4.7 TB/s (scripts/bap_probe.py).  Here the GEMM is a side show (K = 64..128: 2-4 MFMA
// k-steps per tile) and the kernel is shaped like the streaming apply:
//   * persistent workgroups, one column slice of CW = 256 (K = 256: 128) channels each,
//     walking row tiles of RT rows; the slice's weights live in VGPRs as MFMA B fragments
//     for the workgroup's whole life (K x CW/4 columns per wave: 32-64 VGPRs);
//   * the A fragments (dz rows, 16-B loads straight to VGPRs) and the x / add row vectors
//     of tile t+1 are issued before tile t's epilogue, so a tile's loads have the whole
//     previous epilogue to land (two register sets);
//   * the fp32 tile is rounded to bf16 (the value the unfused path stores) through a
//     padded LDS tile, then every thread owns one 8-channel group and RT*CW/2048 rows:
//     16-B x / add loads and dx stores, per-channel parameters from LDS.
// The MFMA order per output element (k-steps 0..K/32-1, v_mfma_f32_16x16x32_bf16) equals
// the implicit-GEMM dgrad's, so g is bitwise the unfused path's stored gradient and the
// APPLY output is bitwise the separate apply's for the same coefficients.
#include <stdexcept>

#include "bn_fused.h"
#include "common.h"
#include "kernels.h"

namespace dtr {

namespace {
constexpr int BND_WG_PER_CU = 2;

// Columns per workgroup: 256-column slices of wide outputs, or the whole 64 / 128-column
// output of the narrowing dgrads.  The resident B fragments ((K / 32) x (CW / 64) per wave)
// and the A operand stay within 2 waves per SIMD -- A as double-buffered MFMA fragments in
// VGPRs up to K = 128 (each wave loads its own copy, L1-served), as one shared LDS tile
// from K = 256.  Rows per tile: the epilogue's 8-channel groups cover whole rows.
constexpr bool bnd_fits(int K, int CW) { return CW > 0 && (K / 32) * (CW / 64) <= 32; }
constexpr int bnd_cw(int C, int K) {
  return (C % 256 == 0 && bnd_fits(K, 256)) ? 256
         : (C % 128 == 0 && bnd_fits(K, 128)) ? 128
         : (C % 64 == 0 && bnd_fits(K, 64)) ? 64 : 0;
}
constexpr int bnd_rt(int K, int CW) {
  return CW == 256 ? (K <= 64 ? 32 : 16) : (2048 / CW > 16 ? 2048 / CW : 16);
}
}  // namespace

template <int MODE, int K, int CW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
bnd1x1_kernel(BndArgs a) {
  constexpr int RT = bnd_rt(K, CW);
  constexpr int MR = RT / 16, WC = CW / 4, NR = WC / 16, KS = K / 32;
  constexpr bool ALDS = K >= 256;            // A through a shared LDS tile
  constexpr int LDA = K + 8;                 // its padded row (conflict-free b128 reads)
  constexpr int ACH = ALDS ? RT * K / 8 / 256 : 1;   // 16-B A chunks per thread and tile
  static_assert(!ALDS || RT * K >= 2048, "every thread stages an A chunk");
  constexpr int CG = CW / 8;           // 8-channel groups per tile row
  constexpr int RPI = 256 / CG;        // tile rows one pass of the 256 threads covers
  constexpr int VPT = RT / RPI;        // row vectors per thread per tile
  constexpr int LDO = CW + 8;          // bf16 row stride of the staging tile
  static_assert(VPT >= 1 && RT % RPI == 0, "tile rows");
  // staging tile; at the end (SUMS) the two [RPI][CW] fp64 reduction planes
  constexpr int SO = RT * LDO > 8 * RPI * CW ? RT * LDO : 8 * RPI * CW;
  __shared__ __attribute__((aligned(16))) bf16 so[SO];
  __shared__ __attribute__((aligned(16))) float prm[7][CW];
  __shared__ __attribute__((aligned(16))) bf16 sa[ALDS ? RT * LDA : 8];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.C;
  const int CT = C / CW;
  const int c0 = (int)(blockIdx.x % CT) * CW;
  const int nrt = a.M / RT, rstep = (int)gridDim.x / CT;   // host: gridDim.x % CT == 0
  int rt = (int)blockIdx.x / CT;
  if (rt >= nrt) return;

  for (int i = tid; i < CW; i += 256) {
    prm[0][i] = a.scale[c0 + i];
    prm[1][i] = a.shift[c0 + i];
    prm[2][i] = a.mean[c0 + i];
    prm[3][i] = a.rstd[c0 + i];
    if constexpr (MODE == 1) {
      prm[4][i] = a.coef[c0 + i];
      prm[5][i] = a.coef[C + c0 + i];
      prm[6][i] = a.coef[2 * C + c0 + i];
    }
  }
  // resident B fragments: lane holds W[col = wave cols + b*16 + lane%16][k = kk*32 + 8*(lane/16) ..+8]
  bf16x8 bfr[KS][NR];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
#pragma unroll
    for (int b = 0; b < NR; ++b)
      bfr[kk][b] = *reinterpret_cast<const bf16x8*>(
          a.w + (long)(c0 + wave * WC + b * 16 + (lane & 15)) * K + kk * 32 + 8 * (lane >> 4));

  const int cg = tid % CG, r0 = tid / CG;
  const bf16x8 zero8 = {};
  bf16x8 af[ALDS ? 1 : MR][ALDS ? 1 : KS], an[ACH], xv[VPT], av[VPT];
  auto load_tile = [&](int t, bf16x8 (&A)[ALDS ? 1 : MR][ALDS ? 1 : KS], bf16x8 (&AN)[ACH],
                       bf16x8 (&X)[VPT], bf16x8 (&D)[VPT]) {
    if constexpr (ALDS) {
#pragma unroll
      for (int q = 0; q < ACH; ++q) {
        const int ch = tid + 256 * q;   // chunk: row ch / (K/8), 8 k's at (ch % (K/8)) * 8
        AN[q] = *reinterpret_cast<const bf16x8*>(a.dz + (long)(t * RT + ch / (K / 8)) * K +
                                                 (ch % (K / 8)) * 8);
      }
    } else {
#pragma unroll
      for (int r = 0; r < MR; ++r)
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
          A[r][kk] = *reinterpret_cast<const bf16x8*>(
              a.dz + (long)(t * RT + r * 16 + (lane & 15)) * K + kk * 32 + 8 * (lane >> 4));
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const long o = (long)(t * RT + r0 + v * RPI) * C + c0 + cg * 8;
      X[v] = *reinterpret_cast<const bf16x8*>(a.x + o);
      if constexpr (MODE == 1) D[v] = a.add ? *reinterpret_cast<const bf16x8*>(a.add + o) : zero8;
    }
  };
  load_tile(rt, af, an, xv, av);
  __syncthreads();   // parameter table

  // per-thread sums: each tile's VPT rows in fp32, the running sum over tiles in fp64
  // (like bn_fwd1x1; RN101 bs256 folds ~200 rows per thread) -- ADVICE r3
  double s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.0;

  for (; rt < nrt; rt += rstep) {
    f32x4 acc[MR][NR];
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[r][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (ALDS) {
#pragma unroll
      for (int q = 0; q < ACH; ++q) {
        const int ch = tid + 256 * q;
        *reinterpret_cast<bf16x8*>(sa + (ch / (K / 8)) * LDA + (ch % (K / 8)) * 8) = an[q];
      }
      lds_barrier();
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int r = 0; r < MR; ++r) {
          const bf16x8 fa = *reinterpret_cast<const bf16x8*>(
              sa + (r * 16 + (lane & 15)) * LDA + kk * 32 + 8 * (lane >> 4));
#pragma unroll
          for (int b = 0; b < NR; ++b) acc[r][b] = mfma16(fa, bfr[kk][b], acc[r][b]);
        }
    } else {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int r = 0; r < MR; ++r)
#pragma unroll
          for (int b = 0; b < NR; ++b) acc[r][b] = mfma16(af[r][kk], bfr[kk][b], acc[r][b]);
    }
    // C fragment (r, b): rows r*16 + 4*(lane/16) + i, column wave*WC + b*16 + lane%16
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
      for (int b = 0; b < NR; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          so[(r * 16 + 4 * (lane >> 4) + i) * LDO + wave * WC + b * 16 + (lane & 15)] =
              (bf16)acc[r][b][i];
    lds_barrier();
    // next tile's loads go out now; this tile's x / add were loaded one tile ago
    bf16x8 xc[VPT], ac[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      xc[v] = xv[v];
      ac[v] = av[v];
    }
    if (rt + rstep < nrt) load_tile(rt + rstep, af, an, xv, av);

    float sc[8], sh[8], mu[8], rs[8], t1[8], t2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t1[j] = t2[j] = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 p0 = *reinterpret_cast<const f32x4*>(&prm[0][cg * 8 + 4 * h]);
      const f32x4 p1 = *reinterpret_cast<const f32x4*>(&prm[1][cg * 8 + 4 * h]);
      const f32x4 p2 = *reinterpret_cast<const f32x4*>(&prm[2][cg * 8 + 4 * h]);
      const f32x4 p3 = *reinterpret_cast<const f32x4*>(&prm[3][cg * 8 + 4 * h]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sc[4 * h + j] = p0[j];
        sh[4 * h + j] = p1[j];
        mu[4 * h + j] = p2[j];
        rs[4 * h + j] = p3[j];
      }
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const int rl = r0 + v * RPI;
      const bf16x8 gv = *reinterpret_cast<const bf16x8*>(so + rl * LDO + cg * 8);
      if constexpr (MODE != 1) {
        if constexpr (MODE == 2)   // the dgrad itself, as the implicit-GEMM BNB dgrad stores it
          *reinterpret_cast<bf16x8*>(a.out + (long)(rt * RT + rl) * C + c0 + cg * 8) = gv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = (float)xc[v][j];
          const float gg = (xf * sc[j] + sh[j] > 0.f) ? (float)gv[j] : 0.f;
          t1[j] += gg;
          t2[j] += gg * (xf - mu[j]) * rs[j];
        }
      } else {
        float ca[8], cb[8], cc[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 p4 = *reinterpret_cast<const f32x4*>(&prm[4][cg * 8 + 4 * h]);
          const f32x4 p5 = *reinterpret_cast<const f32x4*>(&prm[5][cg * 8 + 4 * h]);
          const f32x4 p6 = *reinterpret_cast<const f32x4*>(&prm[6][cg * 8 + 4 * h]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ca[4 * h + j] = p4[j];
            cb[4 * h + j] = p5[j];
            cc[4 * h + j] = p6[j];
          }
        }
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = (float)xc[v][j];
          const float gg = (xf * sc[j] + sh[j] > 0.f) ? (float)gv[j] : 0.f;
          const float xh = (xf - mu[j]) * rs[j];
          o[j] = (bf16)(ca[j] * gg - cb[j] - cc[j] * xh + (float)ac[v][j]);
        }
        *reinterpret_cast<bf16x8*>(a.out + (long)(rt * RT + rl) * C + c0 + cg * 8) = o;
      }
    }
    if constexpr (MODE != 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += (double)t1[j];
        s2[j] += (double)t2[j];
      }
    }
    lds_barrier();   // the staging tile is rewritten by the next tile
  }

  if constexpr (MODE != 1) {
    // fold the RPI threads of each channel group (fixed order), then one fp64 atomic pair
    // per channel and workgroup into the accumulator replica
    double* red = reinterpret_cast<double*>(so);   // [2][RPI][CW]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[r0 * CW + cg * 8 + j] = s1[j];
      red[RPI * CW + r0 * CW + cg * 8 + j] = s2[j];
    }
    __syncthreads();
    for (int c = tid; c < CW; c += 256) {
      double t1 = 0.0, t2 = 0.0;
      for (int q = 0; q < RPI; ++q) {
        t1 += red[q * CW + c];
        t2 += red[RPI * CW + q * CW + c];
      }
      bn_acc_add(a.bacc, C, c0 + c, t1, t2);
    }
  }
}

bool bnd1x1_covers(int M, int C, int K) {
  const int CW = bnd_cw(C, K);
  return (K == 64 || K == 128 || K == 256 || K == 512) && CW > 0 && C % CW == 0 &&
         M > 0 && M % bnd_rt(K, CW) == 0 && (K < 256 || bnd_rt(K, CW) * K >= 2048);
}

template <int K, int CW>
static void bnd_launch(const BndArgs& a, int mode, dim3 g, hipStream_t s) {
  if constexpr (bnd_fits(K, CW)) {
    if (mode == 0) hipLaunchKernelGGL((bnd1x1_kernel<0, K, CW>), g, dim3(256), 0, s, a);
    else if (mode == 1) hipLaunchKernelGGL((bnd1x1_kernel<1, K, CW>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((bnd1x1_kernel<2, K, CW>), g, dim3(256), 0, s, a);
  }
}

template <int CW>
static void bnd_launch_k(const BndArgs& a, int mode, dim3 g, hipStream_t s) {
  if (a.K == 64) bnd_launch<64, CW>(a, mode, g, s);
  else if (a.K == 128) bnd_launch<128, CW>(a, mode, g, s);
  else if (a.K == 256) bnd_launch<256, CW>(a, mode, g, s);
  else bnd_launch<512, CW>(a, mode, g, s);
}

void bnd1x1(const BndArgs& a, int mode, hipStream_t s) {
  if (!bnd1x1_covers(a.M, a.C, a.K))
    throw std::runtime_error("bnd1x1: shape not covered (K in 64..512, C = 64 / 128 or a "
                             "multiple of 256, resident weights <= 128 VGPRs, M % row tile)");
  const int CW = bnd_cw(a.C, a.K);
  const int CT = a.C / CW;
  const long tiles = (long)(a.M / bnd_rt(a.K, CW)) * CT;
  const int cus = cu_count();
  long grid = (long)cus * BND_WG_PER_CU;
  grid -= grid % CT;
  if (grid > tiles) grid = tiles;
  if (grid < CT) grid = CT;
  const dim3 g((unsigned)grid);
  if (CW == 256) bnd_launch_k<256>(a, mode, g, s);
  else if (CW == 128) bnd_launch_k<128>(a, mode, g, s);
  else bnd_launch_k<64>(a, mode, g, s);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
