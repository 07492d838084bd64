// Direct (halo-tiled) 3x3 / stride-1 / pad-1 convolution, forward and data
// gradient, for the small channel counts of the CIFAR stages (C = K in
// {16, 32, 64}; resnet_model_official.py:80-91 emits them through
// conv2d_fixed_padding, SURVEY Appendix A rows "32|16|16|3|1", "16|32|32|3|1",
// "8|64|64|3|1" -- 46 of the 52 CIFAR ResNet-50 convs).
//
// Why a second kernel: the implicit-GEMM path (conv_gemm.hip) gathers an
// im2col row per output pixel, i.e. every input element is fetched 9 times and
// the K loop runs ceil(9C/64) dependent global round trips per workgroup.  At
// C <= 64 the MFMA work is tiny and those round trips ARE the kernel time.
// Here a workgroup owns R = BM / W whole output rows of one image:
//   1. it issues, all at once, the loads of the (R+2) x (W+2) x C input halo
//      (zero rows/columns = TF's fixed padding; the previous layer's BN+ReLU
//      applied once per element in the PRE variant, never per tap) and the
//      per-lane B (weight) fragments of its output channels, straight into
//      VGPRs -- one memory latency for the whole tile;
//   2. stores the halo to LDS with a 16-B-unit XOR swizzle (unit ^ (col &
//      (U-1))) so the 16 consecutive-pixel lanes of a ds_read_b128 spread over
//      the banks;
//   3. runs ceil(9C/32) v_mfma_f32_16x16x32_bf16 k-steps per 16x16 fragment,
//      the k index being (tap, channel): lane group q of step s reads channels
//      [c, c+8) of tap t with s*32 + 8q = t*C + c (taps past 9 carry zero
//      weights);
//   4. hands the fp32 fragments to the shared conv epilogue (bias / residual /
//      BN statistics / BN-backward sums / last-arriver finalize).
// dgrad is the same convolution over dy with the taps flipped (offset 8 - t)
// and the HWIO weights read with K contiguous.
#include <algorithm>
#include <cstdlib>

#include "conv_epilogue.h"

namespace dtr {

template <int CA, int WI, int BM, int BN, int WM, int WN, int MODE, int FLAGS, bool LW>
__global__ void __launch_bounds__(256)
conv3x3_direct_kernel(GemmArgs args) {
  constexpr bool PRE = (FLAGS & F_PRE) != 0;
  constexpr bool ABWD = (FLAGS & F_ABWD) != 0;
  constexpr int U = CA / 8;                 // 16-B units per pixel
  constexpr int R = BM / WI;                // output rows per tile
  constexpr int HW2 = WI + 2;               // halo row length (pixels)
  constexpr int HU = (R + 2) * HW2 * U;     // halo units
  constexpr int HPT = (HU + 255) / 256;     // halo units per thread
  constexpr int KSTEPS = (9 * CA + 31) / 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MR = WTM / 16, NR = WTN / 16;
  static_assert(BM % WI == 0 && WM * WN == 4 && MR >= 1 && NR >= 1, "tile");
  static_assert((U & (U - 1)) == 0, "C/8 must be a power of two");
  // LW: the workgroup's weight slice is staged once through LDS ([BN][KP] rows,
  // padded 16 B so the 16 lanes of a fragment read hit distinct banks) instead of
  // every wave gathering its B fragments into VGPRs
  constexpr int KP = KSTEPS * 32 + 8;
  constexpr int WU = BN * KSTEPS * 4;                         // weight 16-B units
  constexpr int WPT = LW ? (WU + 255) / 256 : 1;
  constexpr int WBYTES = LW ? BN * KP * 2 : 0;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* halo = reinterpret_cast<bf16*>(smem);
  bf16* wl = reinterpret_cast<bf16*>(smem + HU * 16);
  float* pre_s = reinterpret_cast<float*>(smem + HU * 16 + WBYTES);   // PRE: [2][CA] scale, shift
  float* fin_scratch = pre_s + 7 * CA;                        // 768 floats (prologue sums)

  const ConvGeom& g = args.g;
  const int NC = args.Ncol;
  const int H = g.H;                        // stride 1: A and output share H x W
  const int HWp = H * WI;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int img = m0 / HWp;
  const int h0 = (m0 - img * HWp) / WI;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const bf16x8 zero8 = {};
  // diagnostics (scripts/probe_direct.py): wall-clock stamps (100 MHz) of this
  // workgroup's phases -- start, operands staged, MFMAs done, epilogue issued
  long long* const probe = args.probe ? args.probe + 8 * (blockIdx.x + gridDim.x * blockIdx.y) : nullptr;
  if (probe && tid == 0) probe[0] = wall_clock64();

  // ---- 1. all global loads in flight at once: weights (VGPR) + halo (VGPR) ----
  bf16x8 breg[LW ? 1 : KSTEPS][NR];
  bf16x8 wv[WPT];
  if constexpr (LW) {
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int q = tid + i * 256;
      const int nl = q / (KSTEPS * 4), kk = (q - nl * (KSTEPS * 4)) * 8;
      const int tap = kk / CA, c = kk - tap * CA, n = n0 + nl;
      bf16x8 v = zero8;
      if (q < WU && tap < 9 && n < NC) {
        const long off = (MODE == MODE_FWD) ? (long)n * (9 * CA) + kk
                                            : ((long)tap * NC + n) * CA + c;
        v = *reinterpret_cast<const bf16x8*>(args.b + off);
      }
      wv[i] = v;
    }
  }
#pragma unroll
  for (int s = 0; s < (LW ? 0 : KSTEPS); ++s) {
    const int kk = s * 32 + fq * 8;
    const int tap = kk / CA, c = kk - tap * CA;
#pragma unroll
    for (int nb = 0; nb < NR; ++nb) {
      const int n = n0 + wn * WTN + nb * 16 + fr;
      bf16x8 v = zero8;
      if (tap < 9 && n < NC) {
        const long off = (MODE == MODE_FWD) ? (long)n * (9 * CA) + kk        // W[co][r][c][ci]
                                            : ((long)tap * NC + n) * CA + c;  // W[r][c][ci][co]
        v = *reinterpret_cast<const bf16x8*>(args.b + off);
      }
      breg[s][nb] = v;
    }
  }
  bf16x8 hv[HPT];
  bf16x8 hx[ABWD ? HPT : 1], hadd[ABWD ? HPT : 1];   // ABWD: BN input and residual grad
  unsigned hmask = 0;
  const long ibase = (long)img * HWp * CA;
  const bf16* abase = args.a + ibase;
#pragma unroll
  for (int i = 0; i < HPT; ++i) {
    const int q = tid + i * 256;
    bf16x8 v = zero8;
    if constexpr (ABWD) {
      hx[i] = zero8;
      hadd[i] = zero8;
    }
    if (q < HU) {
      const int u = q % U, pix = q / U;
      const int hr = pix / HW2, hc = pix - hr * HW2;
      const int h = h0 - 1 + hr, w = hc - 1;
      if (h >= 0 && h < H && w >= 0 && w < WI) {
        const long o = ((long)h * WI + w) * CA + u * 8;
        v = *reinterpret_cast<const bf16x8*>(abase + o);
        if constexpr (PRE || ABWD) hmask |= 1u << i;   // padding stays zero
        if constexpr (ABWD) {
          hx[i] = *reinterpret_cast<const bf16x8*>(args.abwd.x + ibase + o);
          if (args.abwd.add) hadd[i] = *reinterpret_cast<const bf16x8*>(args.abwd.add + ibase + o);
        }
      }
    }
    hv[i] = v;
  }
  EpiPre<BM, BN, WM> epre;                    // epilogue operands, loaded now
  epi_prefetch<BM, BN, WM, FLAGS>(args, m0, n0, epre);
  // ---- BN scale/shift table for the fused BN+ReLU (finalized here when this is
  //      the BN's first consumer); its loads overlap the halo loads in flight ----
  if constexpr (PRE) {
    if (args.pfin.cnt > 0) {
      bn_prefin_table(args.pfin, CA, pre_s, pre_s + CA, fin_scratch);
    } else {
      if (tid < CA) {
        pre_s[tid] = args.pre_scale[tid];
        pre_s[CA + tid] = args.pre_shift[tid];
      }
      __syncthreads();
    }
  }
  // ---- ABWD: BN-backward coefficients from the producer's partial sums ----
  float* bw_s = pre_s;   // [7][CA]: a, b, c, mean, rstd, scale, shift (ABWD never has PRE)
  if constexpr (ABWD) {
    const BnBwdPre& Q = args.abwd;
    if (Q.cnt == 0) {   // coefficients precomputed by bn_bwd_finalize
      if (tid < CA) {
        bw_s[tid] = Q.coef[tid];
        bw_s[CA + tid] = Q.coef[CA + tid];
        bw_s[2 * CA + tid] = Q.coef[2 * CA + tid];
        bw_s[3 * CA + tid] = Q.mean[tid];
        bw_s[4 * CA + tid] = Q.rstd[tid];
        bw_s[5 * CA + tid] = Q.scale[tid];
        bw_s[6 * CA + tid] = Q.shift[tid];
      }
      __syncthreads();
    }
  }
  if constexpr (ABWD) if (args.abwd.cnt > 0) {
    const BnBwdPre& Q = args.abwd;
    const int c = tid;
    float ga = 0.f, rs = 0.f, mn = 0.f, scl = 0.f, shf = 0.f;   // ahead of the partials
    if (c < CA) {
      ga = Q.gamma[c];
      rs = Q.rstd[c];
      mn = Q.mean[c];
      scl = Q.scale[c];
      shf = Q.shift[c];
    }
    float sg = 0.f, sgx = 0.f;
    if (Q.acc != nullptr) {   // accumulator mode: the channel's two sums, no tile partials
      if (c < CA) {
        double s1, s2;
        bn_acc_sums(Q.acc, CA, c, s1, s2);
        sg = (float)s1;
        sgx = (float)s2;
      }
    } else {
      bn_prefin_sums(Q.part, Q.cnt, CA, fin_scratch, sg, sgx);
    }
    if (c < CA) {
      const float a = ga * rs;
      const float M = (float)args.M;
      bw_s[c] = a;
      bw_s[CA + c] = a * sg / M;
      bw_s[2 * CA + c] = a * sgx / M;
      bw_s[3 * CA + c] = mn;
      bw_s[4 * CA + c] = rs;
      bw_s[5 * CA + c] = scl;
      bw_s[6 * CA + c] = shf;
      if (blockIdx.x == 0 && blockIdx.y == 0) {
        Q.dbeta[c] = sg;
        Q.dgamma[c] = sgx;
        Q.coef[c] = a;
        Q.coef[CA + c] = a * sg / M;
        Q.coef[2 * CA + c] = a * sgx / M;
      }
    }
    __syncthreads();
  }
  // ---- 2. halo -> LDS (swizzled 16-B units) ----
#pragma unroll
  for (int i = 0; i < HPT; ++i) {
    const int q = tid + i * 256;
    if (q < HU) {
      const int u = q % U, pix = q / U;
      const int hc = pix % HW2;
      bf16x8 v = hv[i];
      if constexpr (PRE) {
        if ((hmask >> i) & 1u) v = affine_relu8(v, pre_s + u * 8, pre_s + CA + u * 8);
      }
      if constexpr (ABWD) {
        if ((hmask >> i) & 1u) {
          // dh = a*g - b - c*xhat (+ add), exactly bn_bwd_apply's formula and rounding
          const float* cb = bw_s + u * 8;
          bf16x8 r;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xv = (float)hx[i][j];
            const float gg = (xv * cb[5 * CA + j] + cb[6 * CA + j] > 0.f) ? (float)v[j] : 0.f;
            const float xh = (xv - cb[3 * CA + j]) * cb[4 * CA + j];
            float o2 = cb[j] * gg - cb[CA + j] - cb[2 * CA + j] * xh;
            if (args.abwd.add) o2 += (float)hadd[i][j];
            r[j] = (bf16)o2;
          }
          v = r;
          const int hr = pix / HW2;
          if (hr >= 1 && hr <= R && hc >= 1 && hc <= WI && blockIdx.y == 0) {   // interior: this tile's dh rows
            const long e = ibase + ((long)(h0 + hr - 1) * WI + hc - 1) * CA + u * 8;
            if (args.wt) {   // write-through (sc1), like the epilogue's stores under wt
              typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
              const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.abwd.a_out, 0, 0x7fffffff,
                                                                0x00020000);   // uniform base
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs,
                                                     (int)(e * 2), 0, 16);
            } else {
              *reinterpret_cast<bf16x8*>(args.abwd.a_out + e) = v;
            }
          }
        }
      }
      *reinterpret_cast<bf16x8*>(halo + (pix * U + (u ^ (hc & (U - 1)))) * 8) = v;
    }
  }
  if constexpr (LW) {
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int q = tid + i * 256;
      const int nl = q / (KSTEPS * 4), kk = (q - nl * (KSTEPS * 4)) * 8;
      if (q < WU) *reinterpret_cast<bf16x8*>(wl + nl * KP + kk) = wv[i];
    }
  }
  __syncthreads();
  if (probe && tid == 0) probe[1] = wall_clock64();

  // ---- 3. MFMA over (tap, channel) k-steps ----
  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pbase[MR], pw[MR];
#pragma unroll
  for (int a = 0; a < MR; ++a) {
    const int p = wm * WTM + a * 16 + fr;     // tile-local output pixel
    const int hl = p / WI, w = p - hl * WI;
    pbase[a] = hl * HW2 + w;                  // halo pixel of the window's top-left
    pw[a] = w;
  }
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) {
    const int kk = s * 32 + fq * 8;
    int tap = kk / CA;
    const int unit = (kk - tap * CA) >> 3;
    tap = tap < 9 ? tap : 8;                  // padded k: zero weights, any finite A
    const int ta = (MODE == MODE_FWD) ? tap : 8 - tap;
    const int dy = ta / 3, dx = ta - dy * 3;
#pragma unroll
    for (int a = 0; a < MR; ++a) {
      const int hc = pw[a] + dx;
      const int pix = pbase[a] + dy * HW2 + dx;
      const bf16x8 af =
          *reinterpret_cast<const bf16x8*>(halo + (pix * U + (unit ^ (hc & (U - 1)))) * 8);
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        if constexpr (LW) {
          const bf16x8 bf = *reinterpret_cast<const bf16x8*>(wl + (wn * WTN + b * 16 + fr) * KP + kk);
          acc[a][b] = mfma16(af, bf, acc[a][b]);
        } else {
          acc[a][b] = mfma16(af, breg[s][b], acc[a][b]);
        }
      }
    }
  }
  __syncthreads();   // halo dead: the epilogue reuses the LDS
  if (probe && tid == 0) probe[2] = wall_clock64();

  // ---- 4. shared epilogue ----
  conv_epilogue<BM, BN, WM, WN, FLAGS>(args, acc, smem, m0, n0, &epre);
  if (probe && tid == 0) probe[3] = wall_clock64();
}

static long long* g_probe = nullptr;   // set_direct_probe (diagnostics only): each launch
void set_direct_probe(long long* p) { g_probe = p; }   // advances it past its own stamps

// tune direct_ldsw: bitmask (1: C16, 2: C32, 4: C64) of the layers whose weights are
// staged through LDS.  Default 4, measured (CIFAR RN50, probe + bench): C64 stage
// phase 4.8 -> 4.0 us (dgrad) and 3.5 -> 3.1 (fwd); step bs16 0.978 -> 0.955 ms,
// bs128 unchanged (1.293 / 1.300); C16/C32 add LDS reads without a gain.

template <int CA, int WI, int BM, int BN, int WM, int WN, int MODE, int FLAGS, bool LW>
static void launch_direct_lw(const GemmArgs& a, hipStream_t s) {
  constexpr int HU = (BM / WI + 2) * (WI + 2) * (CA / 8);
  constexpr int KSTEPS = (9 * CA + 31) / 32;
  constexpr size_t WB = LW ? (size_t)BN * (KSTEPS * 32 + 8) * 2 : 0;
  constexpr size_t MAIN = (size_t)HU * 16 + WB + (size_t)(7 * CA + 768) * sizeof(float);
  const size_t lds = (std::max(MAIN, EpiLayout<BM, BN, WM>::BYTES) + 15) & ~(size_t)15;
  dim3 grid(a.M / BM, (a.Ncol + BN - 1) / BN);
  hipLaunchKernelGGL((conv3x3_direct_kernel<CA, WI, BM, BN, WM, WN, MODE, FLAGS, LW>), grid,
                     dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

template <int CA, int WI, int BM, int BN, int WM, int WN, int MODE, int FLAGS>
static void launch_direct_cfg(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  a.probe = g_probe;
  const long out_bytes = (long)a.M * a.Ncol * 2;
  a.wt = wt_store_direct(out_bytes) && out_bytes < (1L << 31) ? 1 : 0;
  if (tune(T_DIRECT_LDSW) & (CA / 16)) launch_direct_lw<CA, WI, BM, BN, WM, WN, MODE, FLAGS, true>(a, s);
  else launch_direct_lw<CA, WI, BM, BN, WM, WN, MODE, FLAGS, false>(a, s);
  if (g_probe) g_probe += 8L * (a.M / BM) * ((a.Ncol + BN - 1) / BN);
}

template <int CA, int WI, int BM, int BN, int WM, int WN, int MODE>
static void launch_direct_flags(const GemmArgs& a, hipStream_t s) {
  const bool pre = a.pre_scale != nullptr, st = a.stat_part != nullptr;
  if constexpr (MODE == MODE_FWD) {
    if (pre && st) launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, F_PRE | F_STATS>(a, s);
    else if (pre) launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, F_PRE>(a, s);
    else if (st) launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, F_STATS>(a, s);
    else launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, 0>(a, s);
  } else {
    const bool ab = a.abwd.x != nullptr;
    if (a.bnb_part != nullptr) {
      if (ab) launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, F_BNB | F_ABWD>(a, s);
      else launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, F_BNB>(a, s);
    } else {
      if (ab) launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, F_ABWD>(a, s);
      else launch_direct_cfg<CA, WI, BM, BN, WM, WN, MODE, 0>(a, s);
    }
  }
}

// Column-split mask for this launch (tune direct_splitn: bit 0 C32, bit 1 C64 in two, bit 2
// C64 in four).  Default (-1): always for the
// 8x8x64 layers, for 16x16x32 only while its grid has fewer workgroups than CUs
// (measured, CIFAR RN50 step: bs128 1.444 -> 1.400 ms, bs32 1.135 -> 1.077, bs16
// 1.074 -> 1.022; splitting 16x16x32 at bs128, 512 -> 1024 workgroups, cost 8 %).
static int direct_split_mask(const GemmArgs& a, int bm) {
  const long forced = tune(T_DIRECT_SPLITN);
  if (forced >= 0) return (int)forced;
  // four column tiles of the 8x8x64 layers at <= 32 images (<= 32 row tiles; measured
  // step: bs16 0.952 -> 0.951 / bs32 0.994 -> 0.977 ms; at 128 images 1.273 -> 1.291)
  const bool c64_4way = a.g.C == 64 || a.g.K == 64 ? (a.M / bm) <= 32 : false;
  return 2 | ((a.M / bm) < 256 ? 1 : 0) | (c64_4way ? 4 : 0);
}

void set_conv_direct(int enabled) { tune_set(T_DIRECT_CONV, enabled ? 1 : 0); }

// Whether the direct kernel covers this conv: 3x3, stride 1, pad 1, A channels ==
// output channels == {16 @ W 32, 32 @ W 16, 64 @ W 8}, and the tile height BM
// (= conv_gemm_bm, so the BN-stat partial layout is unchanged) divides the image.
bool conv_direct_covers(const GemmArgs& a, int mode) {
  if (!tune(T_DIRECT_CONV)) return false;
  const ConvGeom& g = a.g;
  if (g.kh != 3 || g.kw != 3 || g.stride != 1 || g.pad != 1 || g.H != g.Ho || g.W != g.Wo)
    return false;
  if (a.out_f32 != nullptr || a.bias != nullptr) return false;
  const int ca = (mode == MODE_FWD) ? g.C : g.K;
  if (ca != a.Ncol) return false;
  const int bm = conv_gemm_bm(a.M, a.Ncol);
  const int hw = g.H * g.W;
  if (bm % g.W != 0 || hw % bm != 0 || a.M % bm != 0) return false;
  return (ca == 16 && g.W == 32 && (bm == 256 || bm == 128 || bm == 64)) ||
         (ca == 32 && g.W == 16 && (bm == 128 || bm == 64)) ||
         (ca == 64 && g.W == 8 && bm == 64);
}

// Launches the direct kernel when it covers the conv (see above); false otherwise.
bool conv_direct(const GemmArgs& a, int mode, hipStream_t s) {
  if (!conv_direct_covers(a, mode)) return false;
  const ConvGeom& g = a.g;
  const int ca = (mode == MODE_FWD) ? g.C : g.K;
  const int bm = conv_gemm_bm(a.M, a.Ncol);
  const bool fwd = mode == MODE_FWD;
  const int split = direct_split_mask(a, bm);
#define DTR_DIRECT_BN(CA_, W_, BM_, BN_, WM_, WN_)                                      \
  if (ca == CA_ && g.W == W_ && bm == BM_) {                                          \
    if (fwd) launch_direct_flags<CA_, W_, BM_, BN_, WM_, WN_, MODE_FWD>(a, s);        \
    else launch_direct_flags<CA_, W_, BM_, BN_, WM_, WN_, MODE_DGRAD>(a, s);          \
    return true;                                                                      \
  }
#define DTR_DIRECT(CA_, W_, BM_, WM_, WN_) DTR_DIRECT_BN(CA_, W_, BM_, CA_, WM_, WN_)
  // two column tiles (half the weights and MFMAs per workgroup, twice the workgroups)
  // for the layers whose grids are small: 8x8x64 (16 workgroups per image batch of 16)
  // and, at small batch, 16x16x32
  if (split & 4) {   // four column tiles of the 8x8x64 layers
    DTR_DIRECT_BN(64, 8, 64, 16, 4, 1)
  }
  if (split & 2) {
    DTR_DIRECT_BN(64, 8, 64, 32, 2, 2)
  }
  if (split & 1) {
    DTR_DIRECT_BN(32, 16, 64, 16, 4, 1)
  }
  DTR_DIRECT(16, 32, 256, 4, 1)
  DTR_DIRECT(16, 32, 128, 4, 1)
  DTR_DIRECT(16, 32, 64, 4, 1)
  DTR_DIRECT(32, 16, 128, 2, 2)
  DTR_DIRECT(32, 16, 64, 2, 2)
  DTR_DIRECT(64, 8, 64, 1, 4)
#undef DTR_DIRECT
#undef DTR_DIRECT_BN
  return false;
}

}  // namespace dtr
