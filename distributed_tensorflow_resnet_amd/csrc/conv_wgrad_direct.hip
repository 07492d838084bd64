// Direct (halo-tiled) weight gradient of the 3x3 / stride-1 / pad-1 small-C
// convolutions (the CIFAR stages, C = K in {16, 32, 64}; the
// generic split-K kernel is conv_wgrad.hip).
//
//   dW[co][t=(r,c)][ci] = sum_p DY[p][co] * A[p + off(t)][ci],  A = relu(bn(x)) (PRE)
//
// The generic kernel gathers an im2col tile per K step (9 reads of every input
// element, one dependent global round trip per 64 pixels).  Here a workgroup owns
// BMP whole-row pixels (R rows of one image, or whole images) and one group of
// TJ taps:
//   1. ONE round of global loads into VGPRs: the dy tile [BMP][K] and the x halo
//      [(R+2)][(W+2)][C] (zero padding; the BatchNorm+ReLU of x applied once per
//      element while staging);
//   2. both to LDS, pixel-major as they come from HBM;
//   3. MFMA 16x16x32 with the fragments gathered by the transposed LDS read
//      ds_read_b64_tr_b16 (both operands are K(=pixel)-major): lane (q, pc) of a
//      16-lane group points at pixel row q of a 4-row block -- for B at that
//      pixel's halo position shifted by the tap -- and columns 4pc..4pc+3, and
//      receives one column of the transposed 4 x 16 block.  Waves split M
//      (16 output channels each) and, when K < 64, the pixels (WK slices);
//   4. the WK slice results are summed in LDS in fixed order and the workgroup's
//      [K][TJ*C] block is written into its split's fp32 partial slab -- the same
//      [split][K][9C] layout the grouped deterministic reduce already consumes.
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace dtr {

template <int C, int KO, int WI, int HI, int BMP, int TJ, bool PRE>
__global__ void __launch_bounds__(256)
conv_wgrad_direct_kernel(WgradArgs args) {
  constexpr int HW = HI * WI;
  constexpr int NIMG = BMP >= HW ? BMP / HW : 1;
  constexpr int RH = BMP >= HW ? HI : BMP / WI;       // rows per image in the tile
  constexpr int W2 = WI + 2;
  constexpr int U = C / 8;                            // 16-B units per pixel
  constexpr int HU = NIMG * (RH + 2) * W2 * U;        // halo units
  constexpr int HPT = (HU + 255) / 256;
  constexpr int DU = BMP * KO / 8;                    // dy units
  constexpr int DPT = (DU + 255) / 256;
  constexpr int WM = KO / 16, WK = 4 / WM;            // waves: M blocks x pixel slices
  constexpr int NJ = TJ * C;                          // output columns per workgroup
  constexpr int NT = NJ / 16;                         // n-tiles per wave
  constexpr int PX = BMP / WK;                        // pixels per wave
  constexpr int KS = PX / 32;                         // k-steps per wave
  static_assert(WM * WK == 4 && PX % 32 == 0 && NJ % 16 == 0, "tile");
  static_assert(BMP >= HW ? BMP % HW == 0 : (HW % BMP == 0 && BMP % WI == 0), "rows");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* dys = reinterpret_cast<bf16*>(smem);                  // [BMP][KO]
  bf16* halo = dys + BMP * KO;                                // [NIMG][RH+2][W2][C]
  float* pre_s = reinterpret_cast<float*>(halo + HU * 8);     // [2][C]

  const int split = blockIdx.x, tj = blockIdx.y;
  const int p0 = split * BMP;                                 // first pixel of the tile
  const int img0 = p0 / HW, h0 = (p0 - img0 * HW) / WI;       // h0 = 0 for whole images
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wk = wave / WM;
  const bf16x8 zero8 = {};

  // ---- 1. one round of loads: dy tile + x halo ----
  bf16x8 dv[DPT], hv[HPT];
  unsigned hmask = 0;
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    const int q = tid + i * 256;
    dv[i] = q < DU ? *reinterpret_cast<const bf16x8*>(args.dy + (long)p0 * KO + q * 8) : zero8;
  }
#pragma unroll
  for (int i = 0; i < HPT; ++i) {
    const int q = tid + i * 256;
    bf16x8 v = zero8;
    if (q < HU) {
      const int u = q % U, pix = q / U;
      const int hc = pix % W2, rr = pix / W2;
      const int im = rr / (RH + 2), hr = rr - im * (RH + 2);
      const int h = h0 - 1 + hr, w = hc - 1;
      if (h >= 0 && h < HI && w >= 0 && w < WI) {
        v = *reinterpret_cast<const bf16x8*>(
            args.x + (((long)(img0 + im) * HI + h) * WI + w) * C + u * 8);
        if constexpr (PRE) hmask |= 1u << i;
      }
    }
    hv[i] = v;
  }
  if constexpr (PRE) {
    if (tid < C) {
      pre_s[tid] = args.pre_scale[tid];
      pre_s[C + tid] = args.pre_shift[tid];
    }
    __syncthreads();
  }
  // ---- 2. to LDS ----
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    const int q = tid + i * 256;
    if (q < DU) *reinterpret_cast<bf16x8*>(dys + q * 8) = dv[i];
  }
#pragma unroll
  for (int i = 0; i < HPT; ++i) {
    const int q = tid + i * 256;
    if (q < HU) {
      bf16x8 v = hv[i];
      if constexpr (PRE) {
        const int u = q % U;
        if ((hmask >> i) & 1u) v = affine_relu8(v, pre_s + u * 8, pre_s + C + u * 8);
      }
      *reinterpret_cast<bf16x8*>(halo + q * 8) = v;
    }
  }
  __syncthreads();

  // ---- 3. MFMA: acc[n-tile] for output channels [16 wm, 16 wm + 16) ----
  f32x4 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int gq = lane >> 4, li = lane & 15;
  const int qr = li >> 2, pc = li & 3;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    // the two 4-row blocks of this lane group: pixels r1 (elements 0..3), r2 (4..7)
    const int r1 = wk * PX + ks * 32 + 4 * gq + qr;
    const int r2 = r1 + 16;
    const s16x4 alo = lds_read_tr16(dys + r1 * KO + wm * 16 + 4 * pc);
    const s16x4 ahi = lds_read_tr16(dys + r2 * KO + wm * 16 + 4 * pc);
    const s16x8 av = {alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
    const bf16x8 af = __builtin_bit_cast(bf16x8, av);
    // halo pixel (top-left of the 3x3 window) of the two rows
    int hb[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int p = e == 0 ? r1 : r2;
      const int im = p / (RH * WI), rem = p - im * (RH * WI);
      const int hl = rem / WI, w = rem - hl * WI;
      hb[e] = (im * (RH + 2) + hl) * W2 + w;
    }
#pragma unroll
    for (int t = 0; t < TJ; ++t) {
      const int tap = tj * TJ + t;
      const int toff = (tap / 3) * W2 + (tap % 3);
#pragma unroll
      for (int cb = 0; cb < C / 16; ++cb) {
        const int col = cb * 16 + 4 * pc;
        const s16x4 blo = lds_read_tr16(halo + (hb[0] + toff) * C + col);
        const s16x4 bhi = lds_read_tr16(halo + (hb[1] + toff) * C + col);
        const s16x8 bv = {blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]};
        acc[t * (C / 16) + cb] = mfma16(af, __builtin_bit_cast(bf16x8, bv), acc[t * (C / 16) + cb]);
      }
    }
  }
  __syncthreads();   // operands dead: LDS becomes the [WK][KO][NJ] reduction tile

  // ---- 4. fixed-order sum over the WK pixel slices, write the partial block ----
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      red[(wk * KO + wm * 16 + gq * 4 + i) * NJ + n * 16 + li] = acc[n][i];
  __syncthreads();
  float* out = args.part + (long)split * KO * (9 * C) + tj * NJ;
  for (int e = tid; e < KO * NJ; e += 256) {
    const int co = e / NJ, n = e - co * NJ;
    float s = red[e];
#pragma unroll
    for (int k = 1; k < WK; ++k) s += red[k * KO * NJ + e];
    if (args.wt) __hip_atomic_store(out + (long)co * (9 * C) + n, s, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);   // sc1 write-through
    else out[(long)co * (9 * C) + n] = s;
  }
}

// (C, W, H, BMP, TJ) variants; BMP pixels per split, TJ taps per workgroup.
template <int C, int WI, int HI, int BMP, int TJ>
static void wgd_launch(const WgradArgs& a0, hipStream_t s) {
  // Partial slabs stored write-through (sc1, tune wgd_wt): the grouped reduce reads
  // them from another launch, and no dirty slab lines are left for the kernel boundary
  // to write back.
  WgradArgs a = a0;
  a.wt = tune(T_WGD_WT) ? 1 : 0;
  constexpr int NIMG = BMP >= HI * WI ? BMP / (HI * WI) : 1;
  constexpr int RH = BMP >= HI * WI ? HI : BMP / WI;
  constexpr size_t MAIN = (size_t)BMP * C * 2 + (size_t)NIMG * (RH + 2) * (WI + 2) * C * 2 +
                          2 * C * sizeof(float);
  constexpr int WK = 4 / (C / 16);
  constexpr size_t RED = (size_t)WK * C * TJ * C * sizeof(float);
  const size_t lds = ((MAIN > RED ? MAIN : RED) + 15) & ~(size_t)15;
  dim3 grid(a.splits, 9 / TJ);
  if (a.pre_scale)
    hipLaunchKernelGGL((conv_wgrad_direct_kernel<C, C, WI, HI, BMP, TJ, true>), grid, dim3(256),
                       lds, s, a);
  else
    hipLaunchKernelGGL((conv_wgrad_direct_kernel<C, C, WI, HI, BMP, TJ, false>), grid,
                       dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

void set_wgrad_direct(int enabled) { tune_set(T_DIRECT_WGRAD, enabled ? 1 : 0); }

// Workgroups the direct kernel should at least launch: below it the tile shrinks (fewer
// pixels per split, then fewer taps per workgroup).  At 16-32 images per rank (the
// 8-GPU strong-scaling share of the global batch 128) the bs128-tuned tiles left 12-32
// workgroups per stage-3/2 wgrad, ~10 us each, and the side stream became the
// backward's critical path.
static int wgd_target() { return 96; }

// Pixels per split by (channels, pixels) -- the selection that replaced the wgd_bmp16 /
// 32 / 64 keys, measured on the CIFAR RN50 step (MI355X, round 3): 512 for 16 and 32
// channels (256 -> 512: bs128 1.396 -> 1.320 ms); 64 channels 256, or 0 = the split-K
// implicit-GEMM wgrad at <= 1024 pixels (16 images: bs16 step 0.928 -> 0.919 ms).
static int wgd_bmp_for(int C, long P) {
  if (C == 16 || C == 32) return 512;
  return P <= 1024 ? 0 : 256;
}

// smallest pixel tile instantiated per channel count
static int wgd_min_bmp(int C) { return C == 16 ? 128 : 64; }

// Taps per workgroup for this tile: the bs128 default (9 for C 16, 3 otherwise),
// or 1 when even the smallest tile leaves fewer workgroups than the target.
static int wgd_taps(const ConvGeom& g, int bmp) {
  const long P = (long)g.N * g.H * g.W;
  const int tj = g.C == 16 ? 9 : 3;
  if (g.C != 16 && bmp == wgd_min_bmp(g.C) && (P / bmp) * (9 / tj) < wgd_target()) return 1;
  return tj;
}

// Pixels per split of the direct kernel for this conv, 0 if not covered.
int wgrad_direct_bmp(const ConvGeom& g) {
  if (!tune(T_DIRECT_WGRAD)) return 0;
  if (g.kh != 3 || g.kw != 3 || g.stride != 1 || g.pad != 1 || g.C != g.K || g.H != g.W ||
      g.Ho != g.H || g.Wo != g.W)
    return 0;
  // pixels per split (= per workgroup): larger -> fewer split-K slabs for the grouped
  // reduce to read, fewer workgroups
  const long P = (long)g.N * g.H * g.W;
  int bmp = 0;
  if ((g.C == 16 && g.W == 32) || (g.C == 32 && g.W == 16) || (g.C == 64 && g.W == 8))
    bmp = wgd_bmp_for(g.C, P);
  const int lo = wgd_min_bmp(g.C);               // smallest instantiated tile
  const int hi = g.C == 16 ? 1024 : g.C == 32 ? 512 : 256;
  if (bmp < lo || bmp > hi || (bmp & (bmp - 1))) return 0;
  while (bmp > lo && P % bmp != 0) bmp >>= 1;     // the largest tile that divides P
  if (P % bmp != 0) return 0;
  const int tj0 = g.C == 16 ? 9 : 3;
  while (bmp > lo && (P / bmp) * (9 / tj0) < wgd_target() && P % (bmp >> 1) == 0) bmp >>= 1;
  return bmp;
}

bool conv_wgrad_direct(const WgradArgs& a, hipStream_t s) {
  const int bmp = wgrad_direct_bmp(a.g);
  if (bmp == 0 || a.px_per_split != bmp) return false;
  const ConvGeom& g = a.g;
  const int tj = wgd_taps(g, bmp);
  if (g.C == 16) {
    if (bmp == 1024) wgd_launch<16, 32, 32, 1024, 9>(a, s);
    else if (bmp == 512) wgd_launch<16, 32, 32, 512, 9>(a, s);
    else if (bmp == 256) wgd_launch<16, 32, 32, 256, 9>(a, s);
    else wgd_launch<16, 32, 32, 128, 9>(a, s);
  } else if (g.C == 32) {
    if (bmp == 512) wgd_launch<32, 16, 16, 512, 3>(a, s);
    else if (bmp == 256) wgd_launch<32, 16, 16, 256, 3>(a, s);
    else if (bmp == 128) wgd_launch<32, 16, 16, 128, 3>(a, s);
    else if (tj == 3) wgd_launch<32, 16, 16, 64, 3>(a, s);
    else wgd_launch<32, 16, 16, 64, 1>(a, s);
  } else {
    if (bmp == 256) wgd_launch<64, 8, 8, 256, 3>(a, s);
    else if (bmp == 128) wgd_launch<64, 8, 8, 128, 3>(a, s);
    else if (tj == 3) wgd_launch<64, 8, 8, 64, 3>(a, s);
    else wgd_launch<64, 8, 8, 64, 1>(a, s);
  }
  return true;
}

}  // namespace dtr
