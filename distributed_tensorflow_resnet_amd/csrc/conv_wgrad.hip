// Convolution weight gradient (replaces cuDNN Conv2DBackpropFilter).
//
//   dW[co][r][c][ci] = sum_{p=(n,ho,wo)} DY[p][co] * X[n, ho*s-pad+r, wo*s-pad+c, ci]
//
// GEMM view: M = Cout, N = kh*kw*Cin (tap-major, channel-minor), K = pixels.  In
// NHWC both operands are pixel-major (channels contiguous), i.e. K-major, which
// is the wrong way round for MFMA fragments.  Instead of transposing through
// scattered LDS writes, tiles are staged as they come from HBM ([64 px][ch],
// 16-byte loads) and the fragments are gathered with gfx950's transposed LDS
// read `ds_read_b64_tr_b16` (two per 8-element fragment).  Any permutation of
// the K index is legal as long as A and B use the same one, so each 16-lane
// group reads four consecutive pixel rows per instruction, which with the 32-B
// unit XOR swizzle below makes each 32-lane half of the read conflict-free.
//
// K (= N*Ho*Wo, up to 1.6M for the ImageNet stem) is split over a grid
// dimension; every split writes its own fp32 partial slab and wgrad_reduce
// sums the slabs in fixed order (deterministic; no float atomics), writing the
// TF HWIO layout of the master gradient.  Optional fused BN+ReLU is applied to
// X while staging (the pre-activation tensor is never stored).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace dtr {

template <int U>
__device__ __forceinline__ int unit_swz(int row) {
  if constexpr (U <= 1) return 0;
  else return (row / (8 / U)) & (U - 1);
}

// FAST (both tensors < 2^30 elements): 2-deep branch-free register pipeline, as in
// conv_gemm.hip -- the loads of K tile t+2 are in flight while tile t is multiplied
// and tile t+1 is written to LDS; a thread's B column (tap, ci) is fixed for the
// whole loop, so its BN+ReLU scale/shift live in registers (no LDS table, no
// per-chunk channel division at store time).
template <int BM, int BN, int WM, int WN, bool PRE, bool FAST = false>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(2, 8)))
conv_wgrad_kernel(WgradArgs args) {
  constexpr int BK = 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MR = WTM / 16, NR = WTN / 16;
  constexpr int UA = BM / 16, UB = BN / 16;  // 32-byte units per staged row
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;  // 16-byte chunks per row
  constexpr int A_CH = BK * A_CPR, B_CH = BK * B_CPR;
  constexpr int A_PER_T = (A_CH + 255) / 256, B_PER_T = (B_CH + 255) / 256;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(UA <= 8 && UB <= 8, "row <= 256 B");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);        // [2][BK][BM]
  bf16* Bs = As + 2 * BK * BM;                     // [2][BK][BN]
  float* pre_s = reinterpret_cast<float*>(Bs + 2 * BK * BN);

  const ConvGeom& g = args.g;
  const int Cout = g.K, Cin = g.C;
  const int NT = g.kh * g.kw * Cin;
  const int P = g.N * g.Ho * g.Wo;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // (logical tile: args.xcd keeps a split's column tiles -- which read the same dy rows
  // and x pixels -- on one XCD)
  const unsigned pblk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned lblk = args.xcd ? xcd_logical_block(pblk, gridDim.x * gridDim.y * gridDim.z) : pblk;
  const int n0 = (int)(lblk % gridDim.x) * BN;
  const int m0 = (int)((lblk / gridDim.x) % gridDim.y) * BM;
  const int split = (int)(lblk / (gridDim.x * gridDim.y));
  const int p_begin = split * args.px_per_split;
  const int p_end = min(P, p_begin + args.px_per_split);

  if constexpr (PRE && !FAST) {
    for (int i = tid; i < Cin; i += 256) {
      pre_s[i] = args.pre_scale[i];
      pre_s[Cin + i] = args.pre_shift[i];
    }
    __syncthreads();
  }

  bf16x8 ra[A_PER_T], rb[B_PER_T];
  const bf16x8 zero8 = {};
  const int HoWo = g.Ho * g.Wo;

  unsigned bmask = 0;   // PRE: which B chunks of the in-flight tile are real pixels

  // Incremental im2col state: a thread's B chunks keep their column n (so tap and
  // ci are fixed for the whole K loop) and their pixel rows advance by BK each
  // k-step, so (img, ho, wo) are stepped by the launch constants (BK / Wo, BK % Wo)
  // instead of re-derived with 4 runtime divisions per chunk per k-step.  Loads are
  // range-checked buffer loads (invalid chunk -> out-of-range offset -> 0), so there
  // are no exec-mask branches around them.
  const long x_elems = (long)g.N * g.H * g.W * Cin;
  const long dy_elems = (long)P * Cout;
  const bool fast = x_elems < (1L << 30) && dy_elems < (1L << 30);
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.x), 0,
                                                      (int)(fast ? x_elems * 2 : 0), 0x00020000);
  const auto rs_dy = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.dy), 0,
                                                       (int)(fast ? dy_elems * 2 : 0), 0x00020000);
  constexpr int kOOB = 0x7ffffff0;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  auto bload = [&](const __amdgpu_buffer_rsrc_t& rs, int byte_off) -> bf16x8 {
    return __builtin_bit_cast(bf16x8, (u32x4)__builtin_amdgcn_raw_buffer_load_b128(rs, byte_off,
                                                                                   0, 0));
  };
  // per-thread B-chunk state (all of a thread's chunks share the column: B_CPR | 256)
  const int bcc = tid % B_CPR;
  const int bn_ = n0 + bcc * 8;
  const bool bcol_ok = bn_ < NT;
  const int btap = bcol_ok ? bn_ / Cin : 0, bci = bn_ - btap * Cin;
  const int bdr = btap / g.kw, bdc = btap - bdr * g.kw;
  const int d_ho = BK / g.Wo, d_wo = BK - d_ho * g.Wo;
  int b_img[B_PER_T], b_ho[B_PER_T], b_wo[B_PER_T];
#pragma unroll
  for (int i = 0; i < B_PER_T; ++i) {
    const int p = p_begin + (tid + i * 256) / B_CPR;
    b_img[i] = p / HoWo;
    const int rem = p - b_img[i] * HoWo;
    b_ho[i] = rem / g.Wo;
    b_wo[i] = rem - b_ho[i] * g.Wo;
  }
  auto load_tile_fast = [&](int t) {
    if constexpr (PRE) bmask = 0;
    const int pbase = p_begin + t * BK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * 256;
      const int row = q / A_CPR, cc = q % A_CPR;
      const int p = pbase + row;
      const int off = (q < A_CH && p < p_end && m0 + cc * 8 < Cout)
                          ? (p * Cout + m0 + cc * 8) * 2 : kOOB;
      ra[i] = bload(rs_dy, off);
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      const int p = pbase + q / B_CPR;
      const int hi = b_ho[i] * g.stride - g.pad + bdr, wi = b_wo[i] * g.stride - g.pad + bdc;
      int off = kOOB;
      if (q < B_CH && p < p_end && bcol_ok && (unsigned)hi < (unsigned)g.H &&
          (unsigned)wi < (unsigned)g.W) {
        off = (((b_img[i] * g.H + hi) * g.W + wi) * Cin + bci) * 2;
        if constexpr (PRE) bmask |= 1u << i;
      }
      rb[i] = bload(rs_x, off);
      // advance this chunk's pixel by BK for the next k-step
      b_wo[i] += d_wo;
      b_ho[i] += d_ho;
      if (b_wo[i] >= g.Wo) {
        b_wo[i] -= g.Wo;
        b_ho[i] += 1;
      }
      if (b_ho[i] >= g.Ho) {
        b_img[i] += b_ho[i] / g.Ho;
        b_ho[i] -= (b_ho[i] / g.Ho) * g.Ho;
      }
    }
  };
  auto load_tile = [&](int t) {
    if (fast) {
      load_tile_fast(t);
      return;
    }
    if constexpr (PRE) bmask = 0;
    const int pbase = p_begin + t * BK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * 256;
      const int row = q / A_CPR, cc = q % A_CPR;
      const int p = pbase + row;
      bf16x8 v = zero8;
      if (q < A_CH && p < p_end && m0 + cc * 8 < Cout)
        v = *reinterpret_cast<const bf16x8*>(args.dy + (long)p * Cout + m0 + cc * 8);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      const int row = q / B_CPR, cc = q % B_CPR;
      const int p = pbase + row;
      const int n = n0 + cc * 8;
      bf16x8 v = zero8;
      if (q < B_CH && p < p_end && n < NT) {
        const int tap = n / Cin, ci = n - tap * Cin;
        const int r = tap / g.kw, c = tap - r * g.kw;
        const int img = p / HoWo, rem = p - img * HoWo;
        const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
        const int hi = ho * g.stride - g.pad + r, wi = wo * g.stride - g.pad + c;
        if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
          v = *reinterpret_cast<const bf16x8*>(
              args.x + ((long)(img * g.H + hi) * g.W + wi) * Cin + ci);
          if constexpr (PRE) bmask |= 1u << i;   // BN+ReLU applied at LDS-store time
        }
      }
      rb[i] = v;
    }
  };

  auto store_tile = [&](int buf) {
    bf16* A = As + buf * BK * BM;
    bf16* B = Bs + buf * BK * BN;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * 256;
      if (q < A_CH) {
        const int row = q / A_CPR, cc = q % A_CPR;
        const int col = (((cc >> 1) ^ unit_swz<UA>(row)) << 4) + ((cc & 1) << 3);
        *reinterpret_cast<bf16x8*>(A + row * BM + col) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      if (q < B_CH) {
        const int row = q / B_CPR, cc = q % B_CPR;
        const int col = (((cc >> 1) ^ unit_swz<UB>(row)) << 4) + ((cc & 1) << 3);
        bf16x8 v = rb[i];
        if constexpr (PRE) {
          if ((bmask >> i) & 1u) {
            const int n = n0 + cc * 8;
            const int ci = n - (n / Cin) * Cin;
            v = affine_relu8_reg(v, *reinterpret_cast<const f32x4*>(pre_s + ci),
                                 *reinterpret_cast<const f32x4*>(pre_s + ci + 4),
                                 *reinterpret_cast<const f32x4*>(pre_s + Cin + ci),
                                 *reinterpret_cast<const f32x4*>(pre_s + Cin + ci + 4));
          }
        }
        *reinterpret_cast<bf16x8*>(B + row * BN + col) = v;
      }
    }
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = (p_end - p_begin + BK - 1) / BK;

  const int gq = lane >> 4;           // 16-lane group
  const int li = lane & 15;
  const int qr = li >> 2, pc = li & 3;  // row-in-block, 4-column piece
  auto mma_tile = [&](int buf) {
    const bf16* A = As + buf * BK * BM;
    const bf16* B = Bs + buf * BK * BN;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r1 = ks * 32 + 4 * gq + qr;  // pixel row for elements 0..3
      const int r2 = r1 + 16;                // pixel row for elements 4..7
      bf16x8 af[MR], bfr[NR];
#pragma unroll
      for (int a = 0; a < MR; ++a) {
        const int unit = (wm * WTM + a * 16) >> 4;
        const s16x4 lo = lds_read_tr16(A + r1 * BM + ((unit ^ unit_swz<UA>(r1)) << 4) + 4 * pc);
        const s16x4 hi = lds_read_tr16(A + r2 * BM + ((unit ^ unit_swz<UA>(r2)) << 4) + 4 * pc);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[a] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int unit = (wn * WTN + b * 16) >> 4;
        const s16x4 lo = lds_read_tr16(B + r1 * BN + ((unit ^ unit_swz<UB>(r1)) << 4) + 4 * pc);
        const s16x4 hi = lds_read_tr16(B + r2 * BN + ((unit ^ unit_swz<UB>(r2)) << 4) + 4 * pc);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[b] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int b = 0; b < NR; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
  };

  if constexpr (FAST) {
    // ---- 2-deep pipeline: register set P holds K tile t with t % 2 == P ----
    bf16x8 pa[2][A_PER_T], pb[2][B_PER_T];
    unsigned pmask[2] = {0u, 0u};
    f32x4 s0, s1, b0, b1;   // this thread's fixed 8 B channels (bci .. bci+7)
    if constexpr (PRE) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      s0 = bcol_ok ? *reinterpret_cast<const f32x4*>(args.pre_scale + bci) : z;
      s1 = bcol_ok ? *reinterpret_cast<const f32x4*>(args.pre_scale + bci + 4) : z;
      b0 = bcol_ok ? *reinterpret_cast<const f32x4*>(args.pre_shift + bci) : z;
      b1 = bcol_ok ? *reinterpret_cast<const f32x4*>(args.pre_shift + bci + 4) : z;
    }
    auto issue = [&](int t, auto P) {   // t >= KT: every chunk out of range -> zeros
      constexpr int p = decltype(P)::value;
      const int pbase = p_begin + t * BK;
#pragma unroll
      for (int i = 0; i < A_PER_T; ++i) {
        const int q = tid + i * 256;
        const int row = q / A_CPR, cc = q % A_CPR;
        const int px = pbase + row;
        const bool ok = (A_CH % 256 == 0 || q < A_CH) && px < p_end && m0 + cc * 8 < Cout;
        pa[p][i] = bload(rs_dy, ok ? (px * Cout + m0 + cc * 8) * 2 : kOOB);
      }
      unsigned msk = 0u;
#pragma unroll
      for (int i = 0; i < B_PER_T; ++i) {
        const int q = tid + i * 256;
        const int px = pbase + q / B_CPR;
        const int hi = b_ho[i] * g.stride - g.pad + bdr, wi = b_wo[i] * g.stride - g.pad + bdc;
        const bool ok = (B_CH % 256 == 0 || q < B_CH) && px < p_end && bcol_ok &&
                        (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
        pb[p][i] = bload(rs_x, ok ? (((b_img[i] * g.H + hi) * g.W + wi) * Cin + bci) * 2 : kOOB);
        msk |= ok ? (1u << i) : 0u;
        // advance this chunk's pixel by BK for the next k-step
        b_wo[i] += d_wo;
        b_ho[i] += d_ho;
        const bool wrap = b_wo[i] >= g.Wo;
        b_wo[i] -= wrap ? g.Wo : 0;
        b_ho[i] += wrap ? 1 : 0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {   // host: BK / Wo + 1 <= 3 * Ho, so 3 rounds suffice
          const bool nxt = b_ho[i] >= g.Ho;
          b_ho[i] -= nxt ? g.Ho : 0;
          b_img[i] += nxt ? 1 : 0;
        }
      }
      if constexpr (PRE) pmask[p] = msk;
    };
    auto stage = [&](int buf, auto P) {
      constexpr int p = decltype(P)::value;
      bf16* A = As + buf * BK * BM;
      bf16* B = Bs + buf * BK * BN;
#pragma unroll
      for (int i = 0; i < A_PER_T; ++i) {
        const int q = tid + i * 256;
        if (A_CH % 256 == 0 || q < A_CH) {
          const int row = q / A_CPR, cc = q % A_CPR;
          const int col = (((cc >> 1) ^ unit_swz<UA>(row)) << 4) + ((cc & 1) << 3);
          *reinterpret_cast<bf16x8*>(A + row * BM + col) = pa[p][i];
        }
      }
#pragma unroll
      for (int i = 0; i < B_PER_T; ++i) {
        const int q = tid + i * 256;
        if (B_CH % 256 == 0 || q < B_CH) {
          const int row = q / B_CPR, cc = q % B_CPR;
          const int col = (((cc >> 1) ^ unit_swz<UB>(row)) << 4) + ((cc & 1) << 3);
          bf16x8 v = pb[p][i];
          if constexpr (PRE) {
            const unsigned sel = 0u - ((pmask[p] >> i) & 1u);   // padding chunks loaded as 0
            v = affine_relu8_sel(v, s0, s1, b0, b1, sel);
          }
          *reinterpret_cast<bf16x8*>(B + row * BN + col) = v;
        }
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    issue(0, I0{});
    issue(1, I1{});
    stage(0, I0{});
    __syncthreads();
    auto body = [&](int t, auto P) {
      constexpr int p = decltype(P)::value;
      issue(t + 2, P);
      mma_tile(p);
      stage(p ^ 1, std::integral_constant<int, p ^ 1>{});
      __syncthreads();
    };
    int t = 0;
    for (; t + 1 < KT; t += 2) {
      body(t, I0{});
      body(t + 1, I1{});
    }
    if (t < KT) body(t, I0{});
  } else {
    if (KT > 0) {
      load_tile(0);
      store_tile(0);
    }
    __syncthreads();
    for (int t = 0; t < KT; ++t) {
      if (t + 1 < KT) load_tile(t + 1);
      mma_tile(t & 1);
      if (t + 1 < KT) store_tile((t + 1) & 1);
      __syncthreads();
    }
  }

  float* out = args.part + (long)split * Cout * NT;
#pragma unroll
  for (int b = 0; b < NR; ++b) {
    const int n = n0 + wn * WTN + b * 16 + li;
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * WTM + a * 16 + gq * 4 + i;
        if (m < Cout && n < NT) {
          out[(long)m * NT + n] = acc[a][b][i];
        }
      }
  }
}

// FAST eligibility: 32-bit buffer offsets, C % 8 == 0 (16-B channel chunks), and the
// branch-free pixel stepping's 3 image-wrap rounds cover BK = 64 pixels.
static bool wgrad_fast(const WgradArgs& a) {
  const ConvGeom& g = a.g;
  const long x_elems = (long)g.N * g.H * g.W * g.C;
  const long dy_elems = (long)g.N * g.Ho * g.Wo * g.K;
  // (A/B on the ImageNet shapes: 1.05-1.2x at 14x14 / 7x7 outputs, 0.91-1.04x at
  // 56x56 / 28x28, where the occupancy of the one-set loop hides the latency)
  return tune(T_CONV_PIPE) && x_elems < (1L << 30) && dy_elems < (1L << 30) &&
         64 / g.Wo + 1 <= 3 * g.Ho && g.Ho <= 14;
}

template <int BM, int BN, int WM, int WN>
static void wg_launch(const WgradArgs& a, hipStream_t s) {
  const int NT = a.g.kh * a.g.kw * a.g.C;
  size_t lds = (size_t)2 * 64 * (BM + BN) * sizeof(bf16);
  dim3 grid((NT + BN - 1) / BN, (a.g.K + BM - 1) / BM, a.splits);
  if constexpr (BM >= 64) {   // the pipelined loop: ImageNet-size tiles
    if (wgrad_fast(a)) {
      if (a.pre_scale)
        hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, true, true>), grid, dim3(256), lds,
                           s, a);
      else
        hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, false, true>), grid, dim3(256),
                           lds, s, a);
      DTR_CHECK_LAUNCH();
      return;
    }
  }
  if (a.pre_scale) lds += (size_t)2 * a.g.C * sizeof(float);
  if (a.pre_scale)
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, true>), grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, false>), grid, dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

static void wg_tile(const ConvGeom& g, int* bm, int* bn) {
  const int NT = g.kh * g.kw * g.C;
  *bm = g.K <= 16 ? 16 : g.K <= 32 ? 32 : g.K <= 64 ? 64 : 128;
  *bn = NT <= 64 ? 64 : 128;
  if (*bm == 16) *bn = 64;
}

int wgrad_pick_splits(const ConvGeom& g, int* px_per_split) {
  if (const int bmp = wgrad_direct_bmp(g)) {   // direct kernel: one split per pixel tile
    *px_per_split = bmp;
    return (int)((long)g.N * g.H * g.W / bmp);
  }
  int bm, bn;
  wg_tile(g, &bm, &bn);
  const long NT = (long)g.kh * g.kw * g.C;
  const long tiles = ((g.K + bm - 1) / bm) * ((NT + bn - 1) / bn);
  const long P = (long)g.N * g.Ho * g.Wo;
  // ~768 workgroups (3 per CU) hide the per-tile load latency; cap the fp32
  // partial slabs at ~32 MB so the split-K reduce stays cheap, and keep >= 256
  // pixels (4 K-tiles) per split.  (Measured sweep: scripts/sweep_wgrad.py; tune
  // wgrad_target_wg / wgrad_slab_mb.)
  const long target = tune(T_WGRAD_TARGET_WG), cap_mb = tune(T_WGRAD_SLAB_MB);
  long splits = (target + tiles / 2) / tiles;
  const long slab = (long)g.K * NT * 4;
  const long cap_bytes = (cap_mb << 20) / (slab > 0 ? slab : 1);
  if (splits > cap_bytes) splits = cap_bytes;
  long maxs = P / 256;
  if (maxs < 1) maxs = 1;
  if (splits > maxs) splits = maxs;
  if (splits < 1) splits = 1;
  long pps = (P + splits - 1) / splits;
  pps = (pps + 63) / 64 * 64;
  *px_per_split = (int)pps;
  return (int)((P + pps - 1) / pps);
}

void conv_wgrad(const WgradArgs& a0, hipStream_t s) {
  if (conv_wgrad_direct(a0, s)) return;
  WgradArgs a = a0;
  a.xcd = tune(T_WGRAD_XCD) ? 1 : 0;
  int bm, bn;
  wg_tile(a.g, &bm, &bn);
  if (bm == 16) wg_launch<16, 64, 1, 4>(a, s);
  else if (bm == 32 && bn == 64) wg_launch<32, 64, 2, 2>(a, s);
  else if (bm == 32) wg_launch<32, 128, 1, 4>(a, s);
  else if (bm == 64 && bn == 64) wg_launch<64, 64, 2, 2>(a, s);
  else if (bm == 64) wg_launch<64, 128, 2, 2>(a, s);
  else if (bn == 64) wg_launch<128, 64, 2, 2>(a, s);
  else if (conv_wgrad_ring_covers(a)) conv_wgrad_ring(a, s);
  else wg_launch<128, 128, 2, 2>(a, s);
}

// Deterministic split-K reduction + layout change [co][tap][ci] -> HWIO [tap][ci][co],
// dropping padded output channels (co >= Kv) and padded input channels (ci >= Cv).
// Block = 64 consecutive partial columns x 16 split-rows: coalesced slab reads,
// 16 independent accumulation chains per column, fixed-order LDS combine.
__global__ void __launch_bounds__(1024)
wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ grad, int splits, int K,
                    int Kv, int taps, int C, int Cv, float scale, int accumulate) {
  __shared__ float red[16][65];
  const long NT = (long)taps * C;
  const long total = (long)K * NT;
  const int cx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long idx = (long)blockIdx.x * 64 + cx;  // index into one slab [co][tap*C+ci]
  float s = 0.f;
  if (idx < total) {
#pragma unroll 4
    for (int sp = ty; sp < splits; sp += 16) s += part[(long)sp * total + idx];
  }
  red[ty][cx] = s;
  __syncthreads();
  if (ty == 0 && idx < total) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) a += red[k][cx];
    const long co = idx / NT, n = idx - co * NT;
    const long tap = n / C, ci = n - tap * C;
    if (co < Kv && ci < Cv) {
      const long o = (tap * Cv + ci) * Kv + co;
      grad[o] = accumulate ? grad[o] + a * scale : a * scale;
    }
  }
}

void wgrad_reduce(const float* part, float* grad_hwio, int splits, int K, int K_valid, int taps,
                  int C, int C_valid, float scale, int accumulate, hipStream_t s) {
  const long total = (long)K * taps * C;
  const unsigned blocks = (unsigned)((total + 63) / 64);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(1024), 0, s, part, grad_hwio,
                     splits, K, K_valid, taps, C, C_valid, scale, accumulate);
  DTR_CHECK_LAUNCH();
}

// Grouped split-K reduction: ONE launch reduces the partial slabs of many
// convolutions (all convs of a gradient bucket); a block finds its conv by binary
// search over the descriptors' first-chunk offsets.  Two work-unit shapes, chosen
// per conv by its split count (wgrad_reduce_chunks must match):
//   deep (> WGR_WIDE_MAX splits: the many-pixel, small-weight layers): 256
//     consecutive slab columns; 64 column groups of 4 (16-byte loads) x 4 split
//     rows, the 4 row sums combined in LDS in fixed order;
//   wide (few splits, large weights: the 14x14 / 7x7 stages): a 16 (co) x 64 (tap,
//     ci) tile, every thread summing all splits of its 4 columns with the loads in
//     flight together, then transposed through LDS so the HWIO gradient is written
//     as 64-byte co runs instead of one float per co row (measured: the deep form ran
//     the 3-split 28 MB slab of the 7x7 3x3 layer at 1.6 TB/s, half of a plain
//     torch.sum over the same bytes).
// Both sum the splits in a fixed order: deterministic.
constexpr int WGR_COLS = 256;
constexpr int WGR_WIDE_MAX = 8;
__host__ __device__ inline long long wgrad_reduce_chunks_of(int splits, int K, int taps, int C) {
  const long long NT = (long long)taps * C;
  if (splits <= WGR_WIDE_MAX) return ((K + 15) / 16) * ((NT + 63) / 64);
  return ((long long)K * NT + WGR_COLS - 1) / WGR_COLS;
}

long long wgrad_reduce_chunks(int splits, int K, int taps, int C) {
  return wgrad_reduce_chunks_of(splits, K, taps, C);
}

// (register budget: the deep form is latency-bound and wants occupancy -- one kernel
// holding both forms at 100 VGPRs ran the ImageNet step's reduces at 1.16 ms vs 0.78)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
wgrad_reduce_grouped_kernel(const WgReduceDesc* __restrict__ d, int nd, float scale) {
  __shared__ __attribute__((aligned(16))) float lds[64 * 17];
  const long chunk = blockIdx.x;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].chunk0 <= chunk) lo = mid;
    else hi = mid - 1;
  }
  const WgReduceDesc& q = d[lo];
  const long NT = (long)q.taps * q.C;
  const long total = (long)q.K * NT;           // multiple of 8 (C % 8 == 0)
  const int tid = threadIdx.x;
  if (q.splits <= WGR_WIDE_MAX) {
    const long ntn = (NT + 63) / 64;
    const long local = chunk - q.chunk0;
    const int co0 = (int)(local / ntn) * 16;
    const long n0 = (local % ntn) * 64;
    const int r = tid >> 4, c4 = (tid & 15) * 4;
    const int co = co0 + r;
    const long n = n0 + c4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (co < q.K && n < NT) {   // NT % 8 == 0: the 4 columns are all in range
      const float* src = q.part + (long)co * NT + n;
      for (int s0 = 0; s0 < q.splits; s0 += 4) {   // 4 loads in flight, fixed order
        f32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (s0 + j < q.splits) v[j] = *reinterpret_cast<const f32x4*>(src + (long)(s0 + j) * total);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (s0 + j < q.splits) acc += v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) lds[(c4 + j) * 17 + r] = acc[j];
    __syncthreads();
    const int nl = tid >> 2, cq = (tid & 3) * 4;
    const long nn = n0 + nl;
    if (nn < NT) {
      const long tap = nn / q.C, ci = nn - tap * q.C;
      if (ci < q.Cv) {
        float* dst = q.grad + (tap * q.Cv + ci) * q.Kv + co0 + cq;
        const float* t = lds + nl * 17 + cq;
        if ((q.Kv & 3) == 0 && co0 + cq + 3 < q.Kv) {
          *reinterpret_cast<f32x4*>(dst) = f32x4{t[0] * scale, t[1] * scale, t[2] * scale,
                                                 t[3] * scale};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (co0 + cq + j < q.Kv) dst[j] = t[j] * scale;
        }
      }
    }
    return;
  }
  f32x4* red = reinterpret_cast<f32x4*>(lds);  // [4][64]
  const int cg = tid & 63, sr = tid >> 6;
  const long idx = (chunk - q.chunk0) * WGR_COLS + cg * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (idx < total) {
    const float* src = q.part + idx;
#pragma unroll 4
    for (int sp = sr; sp < q.splits; sp += 4)
      acc += *reinterpret_cast<const f32x4*>(src + (long)sp * total);
  }
  red[sr * 64 + cg] = acc;
  __syncthreads();
  if (sr == 0 && idx < total) {
    const f32x4 a = red[cg] + red[64 + cg] + red[128 + cg] + red[192 + cg];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long e = idx + j;
      const long co = e / NT, n = e - co * NT;
      const long tap = n / q.C, ci = n - tap * q.C;
      if (co < q.Kv && ci < q.Cv) q.grad[(tap * q.Cv + ci) * q.Kv + co] = a[j] * scale;
    }
  }
}

void wgrad_reduce_grouped(const WgReduceDesc* descs_dev, int nd, long long total_chunks,
                          float scale, hipStream_t s) {
  hipLaunchKernelGGL(wgrad_reduce_grouped_kernel, dim3((unsigned)total_chunks), dim3(256), 0, s,
                     descs_dev, nd, scale);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
