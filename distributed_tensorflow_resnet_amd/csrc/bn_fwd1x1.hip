// Streaming 1x1 forward conv fused with the BN+ReLU prologue of its input, the residual
// add and the BatchNorm statistics of its output, for the ImageNet bottleneck blocks'
// 1x1 convs whose weights fit in VGPRs: the expanding third conv (K = 64..256 input
// channels, 256-column slices of a wide output) and the narrowing first conv of stages
// 1-2 (256 -> 64, 512 -> 128: the whole output per workgroup) (reference: batch_norm ->
// relu -> conv2d_fixed_padding -> + shortcut, resnet_model_official.py:133-175; the
// sums feed the next BN).
//
//   a[m][k]  = bf16(relu(x[m][k] * scale[k] + shift[k]))        (or x itself: no PRE)
//   y[m][c]  = bf16( sum_k a[m][k] * W[c][k] + res[m][c] )
//   stats   += (sum_m y, sum_m y^2) per channel                  (fp64 replicas)
//
// The backward counterpart (bn_dgrad1x1.hip) explains the shape: as a 128x128 implicit-
// GEMM tile with this epilogue the stage-1 conv moved its 461 MB at ~2.8 TB/s (162 us).
// Here: persistent workgroups, one 256-column slice each, the slice's weights resident
// as MFMA B fragments; per row tile of RT rows the A tile (RT x K) goes through LDS with
// the BN+ReLU applied on the way in (each thread owns fixed channels there: its 8 scale /
// shift pairs stay in registers), the residual rows of tile t+1 are in flight during tile
// t's epilogue, the fp32 tile is staged through LDS and swept as 16-B row vectors: one
// bf16 rounding of acc + res, 16-B stores, per-channel fp64 sums per thread, one fp64
// atomic pair per channel and workgroup at the end.
// The MFMA order per output (k-steps 0..K/32-1) and the prologue arithmetic are the
// implicit-GEMM forward's, so y equals conv_gemm's output bitwise.
#include <stdexcept>

#include "bn_fused.h"
#include "common.h"
#include "kernels.h"

namespace dtr {

namespace {
constexpr int BNF_WG_PER_CU = 2;
// resident B fragments per wave ((K / 32) x (CW / 64)) within 32 (128 VGPRs)
constexpr bool bnf_fits(int K, int CW) { return CW > 0 && (K / 32) * (CW / 64) <= 32; }
// output columns per workgroup: the widest of 256 / 128 / 64 that divides C and whose
// weights fit (narrower slices re-read the A rows once per slice, from L2 / MALL)
constexpr int bnf_cw(int C, int K) {
  return (C % 256 == 0 && bnf_fits(K, 256)) ? 256
         : (C % 128 == 0 && bnf_fits(K, 128)) ? 128
         : (C % 64 == 0 && bnf_fits(K, 64)) ? 64 : 0;
}
// rows per tile: the epilogue's 8-channel groups cover whole rows (RT >= 2048 / CW), every
// thread stages at least one 16-B A chunk (RT >= 2048 / K), one MFMA row block at least
constexpr int bnf_max(int a, int b) { return a > b ? a : b; }
constexpr int bnf_rt(int K, int CW) { return bnf_max(bnf_max(2048 / CW, 2048 / K), 16); }
}  // namespace

template <int K, bool PRE, int CW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
bnf1x1_kernel(BnfArgs a) {
  constexpr int RT = bnf_rt(K, CW);
  constexpr int MR = RT / 16, WC = CW / 4, NR = WC / 16, KS = K / 32;
  constexpr int CG = CW / 8, RPI = 256 / CG, VPT = RT / RPI;
  constexpr int LDC = CW + 4;                  // fp32 staging row stride
  constexpr int LDA = K + 8;                   // bf16 A tile row stride (conflict-free reads)
  constexpr int ACH = RT * K / 8 / 256;        // 16-B A chunks per thread and tile
  constexpr bool PREG = ACH <= 2;              // PRE scale / shift in VGPRs (else LDS reads)
  static_assert(ACH >= 1 && VPT >= 1 && NR >= 1, "tile shape");
  // fp32 staging tile; at the end the two [RPI][CW] fp64 reduction planes
  constexpr int STF = RT * LDC > 4 * RPI * CW ? RT * LDC : 4 * RPI * CW;
  __shared__ __attribute__((aligned(16))) float st[STF];
  __shared__ __attribute__((aligned(16))) bf16 sa[RT * LDA];
  __shared__ __attribute__((aligned(16))) float pre_s[PRE ? 2 * K : 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.C;
  const int CT = C / CW;
  const int c0 = (int)(blockIdx.x % CT) * CW;
  const int nrt = a.M / RT, rstep = (int)gridDim.x / CT;   // host: gridDim.x % CT == 0
  int rt = (int)blockIdx.x / CT;
  if (rt >= nrt) return;

  // BN+ReLU table of the input (finalized here from the fp64 accumulators if pending)
  if constexpr (PRE) {
    if (a.pfin.acc != nullptr) {
      bn_prefin_table(a.pfin, K, pre_s, pre_s + K, nullptr);   // ends with a barrier
    } else {
      for (int i = tid; i < K; i += 256) {
        pre_s[i] = a.pre_scale[i];
        pre_s[K + i] = a.pre_shift[i];
      }
      __syncthreads();
    }
  }
  // this thread's A chunks: chunk ch = tid + 256 q -> row ch / (K/8), channels (ch % (K/8)) * 8
  constexpr int PQ = PREG ? ACH : 1;
  f32x4 ps0[PQ], ps1[PQ], pb0[PQ], pb1[PQ];
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const int kc = ((tid + 256 * q) % (K / 8)) * 8;
    if constexpr (PRE && PREG) {
      ps0[q] = *reinterpret_cast<const f32x4*>(pre_s + kc);
      ps1[q] = *reinterpret_cast<const f32x4*>(pre_s + kc + 4);
      pb0[q] = *reinterpret_cast<const f32x4*>(pre_s + K + kc);
      pb1[q] = *reinterpret_cast<const f32x4*>(pre_s + K + kc + 4);
    }
  }
  // resident B fragments: W[c0 + wave*WC + b*16 + lane%16][kk*32 + 8*(lane/16) ..+8]
  bf16x8 bfr[KS][NR];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
#pragma unroll
    for (int b = 0; b < NR; ++b)
      bfr[kk][b] = *reinterpret_cast<const bf16x8*>(
          a.w + (long)(c0 + wave * WC + b * 16 + (lane & 15)) * K + kk * 32 + 8 * (lane >> 4));

  const int cg = tid % CG, r0 = tid / CG;
  const bf16x8 zero8 = {};
  bf16x8 an[ACH], rv[VPT];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int q = 0; q < ACH; ++q) {
      const int ch = tid + 256 * q;
      an[q] = *reinterpret_cast<const bf16x8*>(a.x + (long)(t * RT + ch / (K / 8)) * K +
                                               (ch % (K / 8)) * 8);
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v)
      rv[v] = a.res ? *reinterpret_cast<const bf16x8*>(
                          a.res + (long)(t * RT + r0 + v * RPI) * C + c0 + cg * 8)
                    : zero8;
  };
  load_tile(rt);

  double s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.0;

  for (; rt < nrt; rt += rstep) {
    // A tile -> LDS, BN+ReLU applied on the way in
#pragma unroll
    for (int q = 0; q < ACH; ++q) {
      const int ch = tid + 256 * q;
      bf16x8 v = an[q];
      if constexpr (PRE && PREG) {
        v = affine_relu8_sel(v, ps0[q], ps1[q], pb0[q], pb1[q], ~0u);
      } else if constexpr (PRE) {
        const int kc = (ch % (K / 8)) * 8;
        v = affine_relu8_sel(v, *reinterpret_cast<const f32x4*>(pre_s + kc),
                             *reinterpret_cast<const f32x4*>(pre_s + kc + 4),
                             *reinterpret_cast<const f32x4*>(pre_s + K + kc),
                             *reinterpret_cast<const f32x4*>(pre_s + K + kc + 4), ~0u);
      }
      *reinterpret_cast<bf16x8*>(sa + (ch / (K / 8)) * LDA + (ch % (K / 8)) * 8) = v;
    }
    lds_barrier();
    f32x4 acc[MR][NR];
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[r][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(
            sa + (r * 16 + (lane & 15)) * LDA + kk * 32 + 8 * (lane >> 4));
#pragma unroll
        for (int b = 0; b < NR; ++b) acc[r][b] = mfma16(fa, bfr[kk][b], acc[r][b]);
      }
    // C fragment (r, b): rows r*16 + 4*(lane/16) + i, column wave*WC + b*16 + lane%16
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
      for (int b = 0; b < NR; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          st[(r * 16 + 4 * (lane >> 4) + i) * LDC + wave * WC + b * 16 + (lane & 15)] =
              acc[r][b][i];
    lds_barrier();
    bf16x8 rc[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) rc[v] = rv[v];
    if (rt + rstep < nrt) load_tile(rt + rstep);   // next tile's A chunks + residual rows
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const int rl = r0 + v * RPI;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(st + rl * LDC + cg * 8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(st + rl * LDC + cg * 8 + 4);
      const float y[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (bf16)(y[j] + (float)rc[v][j]);
        const double d = (double)(float)o[j];
        s1[j] += d;
        s2[j] += d * d;
      }
      *reinterpret_cast<bf16x8*>(a.out + (long)(rt * RT + rl) * C + c0 + cg * 8) = o;
    }
    lds_barrier();   // staging and A tiles are rewritten by the next tile
  }

  if (a.stat_acc != nullptr) {
    double* red = reinterpret_cast<double*>(st);   // [2][RPI][CW]
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
      bn_acc_add(a.stat_acc, C, c0 + c, t1, t2);
    }
  }
}

bool bnf1x1_covers(int M, int C, int K) {
  const int CW = bnf_cw(C, K);
  return (K == 64 || K == 128 || K == 256 || K == 512) && CW > 0 && C % CW == 0 &&
         M > 0 && M % bnf_rt(K, CW) == 0;
}

template <int K, int CW>
static void bnf_launch(const BnfArgs& a, dim3 g, hipStream_t s) {
  if constexpr (bnf_fits(K, CW)) {
    const bool pre = a.pre_scale != nullptr || a.pfin.acc != nullptr;
    if (pre) hipLaunchKernelGGL((bnf1x1_kernel<K, true, CW>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((bnf1x1_kernel<K, false, CW>), g, dim3(256), 0, s, a);
  }
}

template <int CW>
static void bnf_launch_k(const BnfArgs& a, dim3 g, hipStream_t s) {
  if (a.K == 64) bnf_launch<64, CW>(a, g, s);
  else if (a.K == 128) bnf_launch<128, CW>(a, g, s);
  else if (a.K == 256) bnf_launch<256, CW>(a, g, s);
  else bnf_launch<512, CW>(a, g, s);
}

void bnf1x1(const BnfArgs& a, hipStream_t s) {
  if (!bnf1x1_covers(a.M, a.C, a.K))
    throw std::runtime_error("bnf1x1: shape not covered (K in 64..512, C = 64 / 128 or a "
                             "multiple of 256, resident weights <= 128 VGPRs, M % row tile)");
  const int CW = bnf_cw(a.C, a.K);
  const int CT = a.C / CW;
  const long tiles = (long)(a.M / bnf_rt(a.K, CW)) * CT;
  const int cus = cu_count();
  long grid = (long)cus * BNF_WG_PER_CU;
  grid -= grid % CT;
  if (grid > tiles) grid = tiles;
  if (grid < CT) grid = CT;
  const dim3 g((unsigned)grid);
  if (CW == 256) bnf_launch_k<256>(a, g, s);
  else if (CW == 128) bnf_launch_k<128>(a, g, s);
  else bnf_launch_k<64>(a, g, s);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
