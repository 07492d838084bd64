// Implicit-GEMM convolution (forward and data-gradient) for NHWC bf16 tensors on
// gfx950 matrix cores.
//
// Replaces the reference's cuDNN Conv2D / Conv2DBackpropInput (the
// convs are emitted by `conv2d_fixed_padding`, resnet_model_official.py:80-91).
//
//   forward : C[m=(n,ho,wo)][co] = sum_{k=(r,c,ci)} X[n,ho*s-p+r,wo*s-p+c,ci] * W[co][r][c][ci]
//   dgrad   : C[m=(n,h,w)][ci]   = sum_{k=(r,c,co)} DY[n,(h+p-r)/s,(w+p-c)/s,co] * W[r][c][ci][co]
//
// Padding follows TF's conv2d_fixed_padding: pad_beg=(k-1)/2 on top/left, output
// Ho = (H-1)/s + 1 (identical for the stride-1 SAME and stride-2 fixed-pad cases),
// folded into index math -- no Pad kernel.
//
// Design (CDNA4): 256-thread workgroups = 4 wave64s arranged WM x WN; BK = 64
// (two k-steps of v_mfma_f32_16x16x32_bf16); A and B tiles are staged
// global->VGPR->LDS with a one-tile register prefetch and double-buffered LDS
// (one barrier per K tile), LDS rows XOR-swizzled (16-B chunk ^= row&7) so the
// 16-lane groups of ds_read_b128 hit 16 distinct bank slots.  Fused extras:
//   * PRE : apply the previous layer's BatchNorm+ReLU (per-input-channel affine)
//           while staging A, so BN-ReLU outputs are never materialised in HBM;
//   * epilogue: the fp32 accumulator tile is staged through LDS and written
//           back as 16-byte row vectors (8 channels per lane) with bias /
//           residual add / accumulate-into-output fused and ONE bf16 rounding;
//   * STATS: per-workgroup per-channel (mean, M2) Welford partials of the bf16
//           output, finalised by bn_finalize (Chan's parallel combine);
//   * BNB (dgrad): the BatchNorm+ReLU backward reduction of the produced
//           gradient g = d_a * [x*scale+shift > 0]:  per-tile sum(g) and
//           sum(g * xhat), so no separate pass re-reads d_a and x.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "conv_epilogue.h"

namespace dtr {

// NBUF = LDS tile buffers: 2 = one barrier per K tile (register prefetch written
// into the other buffer); 1 = two barriers per K tile but half the LDS, so more
// workgroups per CU (the 128x128 ImageNet tiles).
//
// FAST (every A channel count a multiple of BK, tensors < 2^30 elements: all
// ImageNet layers but the stem) runs a 2-deep register pipeline: the loads of
// K tile t+2 are issued while tile t is multiplied and tile t+1 (loaded one
// iteration earlier) is written to LDS, so each global round trip is hidden
// behind two MFMA blocks and a barrier instead of one.  The whole FAST loop is
// branch-free (out-of-range chunks are buffer loads at an out-of-range offset,
// the BN+ReLU padding mask is a select), so hipcc emits counted vmcnt(N) waits
// instead of vmcnt(0) per chunk.  The 1-deep loop measured latency-bound on the
// 7x7 / 14x14 layers: ~1 us per K tile whatever the tile's MFMA work.
// Register budget: at least 2 waves per SIMD (<= 256 VGPRs+AGPRs), the LDS-bound
// occupancy of the 128x128 tiles.  Without the hint hipcc spent 288-336 registers
// on every 128x128 instantiation (1 wave per SIMD; the pipelined loop 2x slower
// on the 56x56 layers); a budget for the higher LDS-bound occupancy of the smaller
// tiles (3-4 waves) spills the two register sets of the FAST loop.
template <int BM, int BN, int WM, int WN, int MODE, int FLAGS, bool FAST, int NBUF = 2>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(2, 8)))
conv_gemm_kernel(GemmArgs args) {
  constexpr bool PRE = (FLAGS & F_PRE) != 0;
  constexpr bool STATS = (FLAGS & F_STATS) != 0;
  constexpr bool BNB = (FLAGS & F_BNB) != 0;
  static_assert((FLAGS & F_ABWD) == 0, "the fused BN backward prologue is direct-conv only");
  constexpr int BK = 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MR = WTM / 16, NR = WTN / 16;
  constexpr int A_CHUNKS = BM * 8;                    // 16-byte chunks per A tile
  constexpr int B_CHUNKS = BN * 8;
  constexpr int A_PER_T = (A_CHUNKS + 255) / 256;
  constexpr int B_PER_T = (B_CHUNKS + 255) / 256;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(MR >= 1 && NR >= 1, "wave tile >= 16x16");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);                 // [NBUF][BM][BK]
  bf16* Bs = As + NBUF * BM * BK;                           // [NBUF][BN][BK]
  float* pre_s = reinterpret_cast<float*>(Bs + NBUF * BN * BK); // [2][Cin] (PRE)

  const ConvGeom& g = args.g;
  // stride-2 dgrad parity class (blockIdx.z): its rows, reduction depth and taps
  int par_ph = 0, par_pw = 0, par_ns = 1;
  if (MODE == MODE_DGRAD && args.par) {
    par_ph = blockIdx.z >> 1;
    par_pw = blockIdx.z & 1;
    args.par_h0 = (par_ph + g.pad) & 1;
    args.par_w0 = (par_pw + g.pad) & 1;
    args.par_hc = (g.H - args.par_h0 + 1) >> 1;
    args.par_wc = (g.W - args.par_w0 + 1) >> 1;
    par_ns = (g.kw - par_pw + 1) >> 1;
    args.M = g.N * args.par_hc * args.par_wc;
    args.Kdim = ((g.kh - par_ph + 1) >> 1) * par_ns * g.K;
  }
  const int M = args.M, NC = args.Ncol, KD = args.Kdim;
  if (MODE == MODE_DGRAD && args.par && (int)(blockIdx.x * BM) >= M) return;   // class rows done
  // (kernel tap of a class-local K tap: rows ph, ph + 2, ..; columns pw, pw + 2, ..)
  auto class_tap = [&](int tl, int& rr, int& cc) {
    const int q = par_ns > 0 ? tl / par_ns : 0;
    rr = par_ph + 2 * q;
    cc = par_pw + 2 * (tl - q * par_ns);
  };
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tm = blockIdx.x, tn = blockIdx.y;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  // Input-channel count of the A operand's gather (C for fwd, K for dgrad).
  const int Acin = (MODE == MODE_FWD) ? g.C : g.K;


  // ---- per-thread loader state (row decomposition is K-invariant) ----
  const int kg = tid & 7;  // fixed 16-B k-group of every chunk this thread stages
  // 1x1 / stride 1 / no padding: output row m reads A row m (fwd and dgrad alike), so
  // (a_base, h, w) = (m, 0, 0) -- no per-chunk integer divisions by H*W and W, which
  // on the one-K-tile layers (64-channel 1x1) were a quarter of the kernel's VALU work
  const bool pointwise = g.kh == 1 && g.kw == 1 && g.stride == 1 && g.pad == 0;
  int a_base[A_PER_T], a_h[A_PER_T], a_w[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int q = tid + i * 256;
    const int r = q >> 3;
    const int m = m0 + r;
    a_h[i] = -(1 << 28);  // invalid row marker
    a_w[i] = 0;
    a_base[i] = 0;
    if (q < A_CHUNKS && m < M && pointwise) {
      a_base[i] = m;
      a_h[i] = 0;
    } else if (q < A_CHUNKS && m < M) {
      if constexpr (MODE == MODE_FWD) {
        const int hw = g.Ho * g.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
        a_base[i] = n * g.H * g.W;
        a_h[i] = ho * g.stride - g.pad;
        a_w[i] = wo * g.stride - g.pad;
      } else {
        int n, h, w;
        if (args.par) {   // class-local row -> (n, h0 + 2 hh, w0 + 2 ww)
          const int per = args.par_hc * args.par_wc;
          n = m / per;
          const int rem = m - n * per, hh = rem / args.par_wc;
          h = args.par_h0 + 2 * hh;
          w = args.par_w0 + 2 * (rem - hh * args.par_wc);
        } else {
          const int hw = g.H * g.W;
          n = m / hw;
          const int rem = m - n * hw;
          h = rem / g.W;
          w = rem - h * g.W;
        }
        a_base[i] = n * g.Ho * g.Wo;
        a_h[i] = h + g.pad;
        a_w[i] = w + g.pad;
      }
    }
  }

  bf16x8 ra[A_PER_T], rb[B_PER_T];
  const bf16x8 zero8 = {};

  unsigned amask = 0;   // PRE: which A chunks of the in-flight tile are real pixels
  // PRE: input channel of this thread's 8-channel group in the in-flight tile, and
  // its BN scale/shift, read from the LDS table right after the tile's loads are
  // issued so the table read overlaps the current tile's MFMAs (reading it at LDS
  // store time put an LDS round trip + integer division on every K tile's
  // critical path: +15..58 us per ImageNet conv).
  int pre_ci = 0;
  f32x4 s0, s1, b0, b1;
  auto load_pre = [&]() {
    s0 = *reinterpret_cast<const f32x4*>(pre_s + pre_ci);
    s1 = *reinterpret_cast<const f32x4*>(pre_s + pre_ci + 4);
    b0 = *reinterpret_cast<const f32x4*>(pre_s + Acin + pre_ci);
    b1 = *reinterpret_cast<const f32x4*>(pre_s + Acin + pre_ci + 4);
  };

  // Fast gather (every A channel count a multiple of BK: all ImageNet layers but
  // the stem): a K tile then lies inside ONE filter tap, so (tap, r, c) are
  // wave-uniform scalars per k-step and each chunk needs only two adds, two
  // unsigned compares and one 32-bit multiply-add -- instead of the per-chunk
  // runtime divisions and exec-mask branches of the general path (which cost as
  // many VALU cycles as the MFMAs).  Loads are buffer loads with a hardware range
  // check: an invalid (padding) chunk gets an out-of-range offset and reads 0.
  const long a_elems = (MODE == MODE_FWD) ? (long)g.N * g.H * g.W * g.C
                                          : (long)g.N * g.Ho * g.Wo * g.K;
  const long b_elems = (long)g.kh * g.kw * g.C * g.K;
  // Narrow forward operands (the ImageNet stem: 8 channels, or 16 in space-to-depth
  // form) take the same branch-free buffer-load gather with a per-thread tap: a K tile
  // then spans BK / Acin taps, one 8-channel group each (load_tile_fast).
  constexpr bool NARROW_OK = MODE == MODE_FWD && !PRE;
  const bool narrow = NARROW_OK && Acin < BK && Acin % 8 == 0 && BK % Acin == 0;
  const bool fast = ((Acin % BK) == 0 || narrow) && a_elems < (1L << 30) && b_elems < (1L << 30);
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.a), 0,
                                                      (int)(fast ? a_elems * 2 : 0), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.b), 0,
                                                      (int)(fast ? b_elems * 2 : 0), 0x00020000);
  constexpr int kOOB = 0x7ffffff0;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  auto bload = [&](const __amdgpu_buffer_rsrc_t& rs, int byte_off) -> bf16x8 {
    return __builtin_bit_cast(bf16x8, (u32x4)__builtin_amdgcn_raw_buffer_load_b128(rs, byte_off,
                                                                                   0, 0));
  };
  auto load_tile_fast = [&](int t) {
    if constexpr (PRE) amask = 0;
    const int kb = t * BK;                       // uniform
    bool kv = kb < KD;
    int tap = kv ? kb / Acin : 0;                // uniform (scalar unit)
    int ci = kb - tap * Acin + kg * 8;
    if constexpr (NARROW_OK) {
      if (narrow) {   // this thread's own tap (K tail checked per 8-channel group)
        const int k = kb + kg * 8;
        kv = k < KD;
        tap = kv ? k / Acin : 0;
        ci = k - tap * Acin;
      }
    }
    if constexpr (PRE) pre_ci = kv ? ci : 0;
    int rr = tap / g.kw, cc = tap - rr * g.kw;
    if (MODE == MODE_DGRAD && args.par) class_tap(tap, rr, cc);
    const int gtap = rr * g.kw + cc;   // kernel tap (weight layout)
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      int off = kOOB;
      if constexpr (MODE == MODE_FWD) {
        const int hi = a_h[i] + rr, wi = a_w[i] + cc;
        if (kv && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W) {
          off = ((a_base[i] + hi * g.W + wi) * g.C + ci) * 2;
          if constexpr (PRE) amask |= 1u << i;
        }
      } else {
        int hp = a_h[i] - rr, wp = a_w[i] - cc;
        bool ok = kv && hp >= 0 && wp >= 0;
        if (g.stride == 2) {
          ok = ok && ((hp | wp) & 1) == 0;
          hp >>= 1;
          wp >>= 1;
        }
        if (ok && hp < g.Ho && wp < g.Wo) off = ((a_base[i] + hp * g.Wo + wp) * g.K + ci) * 2;
      }
      ra[i] = bload(rs_a, off);
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      const int nrow = q >> 3;
      int off = kOOB;
      if (q < B_CHUNKS && n0 + nrow < NC && kv) {
        if constexpr (MODE == MODE_FWD) off = ((n0 + nrow) * KD + kb + kg * 8) * 2;
        else off = ((gtap * g.C + (n0 + nrow)) * g.K + ci) * 2;
      }
      rb[i] = bload(rs_b, off);
    }
  };
  auto load_tile = [&](int t) {
    if (fast) {
      load_tile_fast(t);
      return;
    }
    if constexpr (PRE) amask = 0;
    const int k = t * BK + kg * 8;
    const bool kvalid = k < KD;
    const int tap = kvalid ? k / Acin : 0;
    const int ci = k - tap * Acin;
    if constexpr (PRE) pre_ci = kvalid ? ci : 0;
    int rr = tap / g.kw, cc = tap - rr * g.kw;
    if (MODE == MODE_DGRAD && args.par) class_tap(tap, rr, cc);
    const int gtap = rr * g.kw + cc;   // kernel tap (weight layout)
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      bf16x8 v = zero8;
      if constexpr (MODE == MODE_FWD) {
        const int hi = a_h[i] + rr, wi = a_w[i] + cc;
        if (kvalid && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
          const long off = ((long)(a_base[i] + hi * g.W + wi)) * g.C + ci;
          v = *reinterpret_cast<const bf16x8*>(args.a + off);
          if constexpr (PRE) amask |= 1u << i;   // BN+ReLU applied at LDS store time
        }
      } else {
        int hp = a_h[i] - rr, wp = a_w[i] - cc;
        bool ok = kvalid && hp >= 0 && wp >= 0;
        if (g.stride != 1) {
          ok = ok && (hp % g.stride == 0) && (wp % g.stride == 0);
          hp /= g.stride;
          wp /= g.stride;
        }
        if (ok && hp < g.Ho && wp < g.Wo) {
          const long off = ((long)(a_base[i] + hp * g.Wo + wp)) * g.K + ci;
          v = *reinterpret_cast<const bf16x8*>(args.a + off);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      const int nrow = q >> 3;
      bf16x8 v = zero8;
      if (q < B_CHUNKS && n0 + nrow < NC && kvalid) {
        long off;
        if constexpr (MODE == MODE_FWD) {
          off = (long)(n0 + nrow) * KD + k;                    // W[co][r][c][ci]
        } else {
          off = ((long)gtap * g.C + (n0 + nrow)) * g.K + ci;   // W[r][c][ci][co]
        }
        v = *reinterpret_cast<const bf16x8*>(args.b + off);
      }
      rb[i] = v;
    }
  };

  // PRE is applied here, after the MFMAs of the previous tile, so the prefetched
  // loads stay in flight across them (applying it in load_tile forced the wait).
  auto store_tile = [&](int buf) {
    bf16* A = As + buf * BM * BK;
    bf16* B = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * 256;
      if (q < A_CHUNKS) {
        const int r = q >> 3;
        bf16x8 v = ra[i];
        if constexpr (PRE) {
          if ((amask >> i) & 1u) v = affine_relu8_reg(v, s0, s1, b0, b1);
        }
        *reinterpret_cast<bf16x8*>(A + r * BK + ((kg ^ (r & 7)) << 3)) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      if (q < B_CHUNKS) {
        const int r = q >> 3;
        *reinterpret_cast<bf16x8*>(B + r * BK + ((kg ^ (r & 7)) << 3)) = rb[i];
      }
    }
  };

  // ---- FAST path: two register sets (tile parity), everything branch-free ----
  bf16x8 pa[2][A_PER_T], pb[2][B_PER_T];
  unsigned pmask[2] = {0u, 0u};
  int pci[2] = {0, 0};
  // split-K slice of this workgroup: K tiles [t_beg, t_end)
  const int KT_all = (KD + BK - 1) / BK;
  const int sk_n = args.ksplit > 1 ? args.ksplit : 1, sk_z = sk_n > 1 ? (int)blockIdx.z : 0;
  const int t_beg = (int)(((long)sk_z * KT_all) / sk_n);
  const int t_end = (int)(((long)(sk_z + 1) * KT_all) / sk_n);
  auto issue = [&](int t, auto P) {   // loads of K tile t into set P (t >= t_end: zeros)
    constexpr int p = decltype(P)::value;
    const int kb = t * BK;                       // uniform
    const bool kv = kb < KD && t < t_end;
    const int tap = kv ? kb / Acin : 0;          // uniform (scalar unit)
    const int ci = kb - tap * Acin + kg * 8;
    if constexpr (PRE) pci[p] = kv ? ci : 0;
    int rr = tap / g.kw, cc = tap - rr * g.kw;
    if (MODE == MODE_DGRAD && args.par) class_tap(tap, rr, cc);
    const int gtap = rr * g.kw + cc;   // kernel tap (weight layout)
    unsigned msk = 0u;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      int off = kOOB;
      if constexpr (MODE == MODE_FWD) {
        const int hi = a_h[i] + rr, wi = a_w[i] + cc;
        const bool ok = kv && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
        off = ok ? ((a_base[i] + hi * g.W + wi) * g.C + ci) * 2 : kOOB;
        msk |= ok ? (1u << i) : 0u;
      } else {
        int hp = a_h[i] - rr, wp = a_w[i] - cc;
        bool ok = kv && hp >= 0 && wp >= 0;
        if (g.stride == 2) {
          ok = ok && ((hp | wp) & 1) == 0;
          hp >>= 1;
          wp >>= 1;
        }
        ok = ok && hp < g.Ho && wp < g.Wo;
        off = ok ? ((a_base[i] + hp * g.Wo + wp) * g.K + ci) * 2 : kOOB;
        msk |= ok ? (1u << i) : 0u;
      }
      pa[p][i] = bload(rs_a, off);
    }
    if constexpr (PRE) pmask[p] = msk;
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      const int nrow = q >> 3;
      const bool ok = (B_CHUNKS % 256 == 0 || q < B_CHUNKS) && n0 + nrow < NC && kv;
      int off;
      if constexpr (MODE == MODE_FWD) off = ((n0 + nrow) * KD + kb + kg * 8) * 2;
      else off = ((gtap * g.C + (n0 + nrow)) * g.K + ci) * 2;
      pb[p][i] = bload(rs_b, ok ? off : kOOB);
    }
  };
  auto stage = [&](int buf, auto P) {   // set P -> LDS buffer `buf` (BN+ReLU applied)
    constexpr int p = decltype(P)::value;
    bf16* A = As + buf * BM * BK;
    bf16* B = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * 256;
      if (A_CHUNKS % 256 == 0 || q < A_CHUNKS) {
        const int r = q >> 3;
        bf16x8 v = pa[p][i];
        if constexpr (PRE) {
          const unsigned sel = 0u - ((pmask[p] >> i) & 1u);   // all-ones: real pixel
          v = affine_relu8_sel(v, s0, s1, b0, b1, sel);
        }
        *reinterpret_cast<bf16x8*>(A + r * BK + ((kg ^ (r & 7)) << 3)) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int q = tid + i * 256;
      if (B_CHUNKS % 256 == 0 || q < B_CHUNKS) {
        const int r = q >> 3;
        *reinterpret_cast<bf16x8*>(B + r * BK + ((kg ^ (r & 7)) << 3)) = pb[p][i];
      }
    }
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto mma_tile = [&](int buf) {
    const bf16* A = As + buf * BM * BK;
    const bf16* B = Bs + buf * BN * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;
      bf16x8 af[MR], bfr[NR];
#pragma unroll
      for (int a = 0; a < MR; ++a) {
        const int r = wm * WTM + a * 16 + fr;
        af[a] = *reinterpret_cast<const bf16x8*>(A + r * BK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int r = wn * WTN + b * 16 + fr;
        bfr[b] = *reinterpret_cast<const bf16x8*>(B + r * BK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int b = 0; b < NR; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
  };

  const int KT = (KD + BK - 1) / BK;
  // dgrad + BN-backward sums: the epilogue's BN-input rows and coefficients are
  // GEMM-independent -> issue their loads now, off the epilogue's critical path.
  // (prefetching the forward's residual rows the same way measured 1% slower)
  using EP = EpiPre<BM, BN, WM, true>;
  EP epre;
  if constexpr (FAST) {
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    issue(t_beg, I0{});
    issue(t_beg + 1, I1{});
    if constexpr (BNB) epi_prefetch<BM, BN, WM, FLAGS, true>(args, m0, n0, epre);
    if constexpr (PRE) {
      if (args.pfin.cnt > 0) {
        bn_prefin_table(args.pfin, Acin, pre_s, pre_s + Acin, reinterpret_cast<float*>(As));
      } else {
        for (int i = tid; i < Acin; i += 256) {
          pre_s[i] = args.pre_scale[i];
          pre_s[Acin + i] = args.pre_shift[i];
        }
        __syncthreads();
      }
      pre_ci = pci[0];
      load_pre();
    }
    stage(0, I0{});
    __syncthreads();
    // iteration t (parity P): loads of t+2 into set P (its tile t is already in
    // LDS), MFMAs on buffer P, then set !P (tile t+1) -> buffer !P.
    auto body = [&](int t, auto P) {
      constexpr int p = decltype(P)::value;
      issue(t + 2, P);
      if constexpr (PRE) {
        pre_ci = pci[p ^ 1];
        load_pre();
      }
      mma_tile(p);
      stage(p ^ 1, std::integral_constant<int, p ^ 1>{});
      __syncthreads();
    };
    int t = t_beg;
    for (; t + 1 < t_end; t += 2) {
      body(t, I0{});
      body(t + 1, I1{});
    }
    if (t < t_end) body(t, I0{});
    if (sk_n > 1 && !splitk_combine<MR, NR>(args, acc, smem, tm, tn, blockIdx.z)) return;
  } else {   // general gather (runtime `fast` only for the narrow-column tiles)
  load_tile(0);
  if constexpr (BNB) epi_prefetch<BM, BN, WM, FLAGS, true>(args, m0, n0, epre);
  if constexpr (PRE) {   // BN scale/shift table (finalized here if this is the first consumer)
    if (args.pfin.cnt > 0) {
      bn_prefin_table(args.pfin, Acin, pre_s, pre_s + Acin, reinterpret_cast<float*>(As));
    } else {
      for (int i = tid; i < Acin; i += 256) {
        pre_s[i] = args.pre_scale[i];
        pre_s[Acin + i] = args.pre_shift[i];
      }
      __syncthreads();
    }
  }
  if constexpr (PRE) load_pre();
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < KT; ++t) {
    if (t + 1 < KT) {
      load_tile(t + 1);
      if constexpr (PRE) load_pre();
    }
    mma_tile(NBUF == 2 ? (t & 1) : 0);
    if constexpr (NBUF == 1) __syncthreads();   // every wave is done reading the tile
    if (t + 1 < KT) store_tile(NBUF == 2 ? ((t + 1) & 1) : 0);
    __syncthreads();
  }
  }

  if constexpr (BNB && EP::ON)
    conv_epilogue<BM, BN, WM, WN, FLAGS, true>(args, acc, smem, m0, n0, &epre, tm, tn);
  else
    conv_epilogue<BM, BN, WM, WN, FLAGS, false>(args, acc, smem, m0, n0, nullptr, tm, tn);
}

// ---------------------------------------------------------------------------
// host-side dispatch (tile / schedule parameters: tune.h)
// ---------------------------------------------------------------------------
void set_conv_pipeline(int enabled) { tune_set(T_CONV_PIPE, enabled ? 1 : 0); }

// Split-K of the FAST loop for under-filled grids (the 7x7 stage: 196 tiles of 128x128
// for 256 CUs, each a 32-72 K-tile loop at one workgroup per CU): up to `splitk` slices
// for grids of <= `splitk_tiles` tiles.  Workspace: one fp32 tile per slice and tile plus
// a ticket per tile, per device, allocated on first need (never while a graph is being
// captured -- the launch then runs unsplit) and grown, never freed.  The launches that
// use it are ordered on one stream (the training plan issues every conv_gemm on the main
// stream); the ticket of a tile is reset by its last slice.
void set_conv_splitk(int max_slices) { tune_set(T_SPLITK, max_slices < 1 ? 1 : max_slices); }

static int pick_ksplit(long tiles, int KT) {
  const long smax = tune(T_SPLITK), max_tiles = tune(T_SPLITK_TILES);
  int S = 1;
  while (S * 2 <= smax && tiles * S <= max_tiles && KT / (S * 2) >= 8) S *= 2;
  return S;
}

// FAST-path eligibility (see the kernel): must match the kernel's own `fast` test.
static bool conv_gemm_fast(const GemmArgs& a, int mode) {
  if (!tune(T_CONV_PIPE)) return false;
  const ConvGeom& g = a.g;
  const int Acin = (mode == MODE_FWD) ? g.C : g.K;
  const long a_elems = (mode == MODE_FWD) ? (long)g.N * g.H * g.W * g.C
                                          : (long)g.N * g.Ho * g.Wo * g.K;
  const long b_elems = (long)g.kh * g.kw * g.C * g.K;
  if (!(Acin % 64 == 0 && a_elems < (1L << 30) && b_elems < (1L << 30))) return false;
  // Where the deeper pipeline pays (scripts/ab_conv_gemm.py, ImageNet RN50 shapes,
  // both loops at 2 waves/SIMD): K loops of >= 4 tiles, and
  //   forward: >= 128 output channels (1.02-1.24x; the 64-column 56x56 convs
  //            run 0.81-0.83x: their single-set loop keeps more tiles per CU);
  //   dgrad:   >= 16k rows (1.06-1.16x at 14x14..56x56; the 7x7 grids of <= 200
  //            tiles run 0.88-0.95x) -- and the 7x7 dgrads once split-K doubles their grid.
  if (a.Kdim < 256) return false;
  if (mode == MODE_FWD) return a.Ncol >= 128;
  if (a.M >= 16384) return true;
  if (!tune(T_DGRAD_SPLITK) || a.Ncol < 128) return false;
  const int bm = conv_gemm_bm(a.M, a.Ncol), bn = conv_gemm_bn(a.M, a.Ncol);
  const long tiles = (long)((a.M + bm - 1) / bm) * ((a.Ncol + bn - 1) / bn);
  return pick_ksplit(tiles, (a.Kdim + 63) / 64) > 1;
}

// Split-K workspace of an immediate (non-plan) launch: grown on demand, per device.  Plan
// launches never come here -- the plan owns one workspace per stream, sized when the op is
// recorded (conv_gemm_splitk_need) and passed in GemmArgs::sk_part / sk_cnt.
struct SplitKWorkspace {
  float* part = nullptr;
  size_t part_bytes = 0;
  unsigned* cnt = nullptr;
  size_t cnt_n = 0;
};

static bool splitk_workspace(size_t part_bytes, size_t tiles, hipStream_t s, float** part,
                             unsigned** cnt) {
  static SplitKWorkspace ws[64];   // per device
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) return false;
  if (dev < 0 || dev >= 64) return false;
  SplitKWorkspace& w = ws[dev];
  if (part_bytes > w.part_bytes || tiles > w.cnt_n) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &cap);
    if (cap != hipStreamCaptureStatusNone) return false;
    (void)hipStreamSynchronize(s);   // the old buffers are no longer read in flight
    if (part_bytes > w.part_bytes) {
      void* p = nullptr;
      if (hipMalloc(&p, part_bytes) != hipSuccess) return false;
      (void)hipFree(w.part);
      w.part = static_cast<float*>(p);
      w.part_bytes = part_bytes;
    }
    if (tiles > w.cnt_n) {
      void* p = nullptr;
      const size_t n = tiles < 4096 ? 4096 : tiles;
      if (hipMalloc(&p, n * sizeof(unsigned)) != hipSuccess) return false;
      if (hipMemsetAsync(p, 0, n * sizeof(unsigned), s) != hipSuccess) return false;
      (void)hipFree(w.cnt);
      w.cnt = static_cast<unsigned*>(p);
      w.cnt_n = n;
    }
  }
  *part = w.part;
  *cnt = w.cnt;
  return true;
}

// Sizing query (conv_gemm_splitk_need): the launchers run their selection logic and
// record the split-K slab bytes and tile counters they would use, launching nothing.
struct SplitKNeed {
  size_t bytes = 0, tiles = 0;
};
static thread_local SplitKNeed* g_sk_query = nullptr;

template <int BM, int BN, int WM, int WN, int MODE, int FLAGS, int NBUF>
static void launch_nbuf(const GemmArgs& a0, hipStream_t s);

template <int BM, int BN, int WM, int WN, int MODE, int FLAGS>
static void launch_cfg(const GemmArgs& a, hipStream_t s) {
  // A one-tile K loop (the 64-channel 1x1 convs: 4 forward + 4 dgrad launches of the
  // ImageNet 56x56 stage) double-buffers nothing: one LDS buffer halves the main-loop
  // LDS, so the 128x128 tiles fit 4 workgroups per CU instead of 2 and the
  // load -> MFMA -> epilogue phases of co-resident workgroups overlap.
  if constexpr (BM * BN >= 128 * 64) {
    if ((a.Kdim + 63) / 64 <= tune(T_NBUF1_KT) && !conv_gemm_fast(a, MODE)) {
      launch_nbuf<BM, BN, WM, WN, MODE, FLAGS, 1>(a, s);
      return;
    }
  }
  launch_nbuf<BM, BN, WM, WN, MODE, FLAGS, 2>(a, s);
}

template <int BM, int BN, int WM, int WN, int MODE, int FLAGS, int NBUF>
static void launch_nbuf(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  // sizing query: only the FAST / ring split-K branch below records a need
  const bool query = g_sk_query != nullptr;
  a.wt = wt_store_enabled() && (long)a.M * a.Ncol * 2 < (1L << 31) ? 1 : 0;
  const int Acin = (MODE == MODE_FWD) ? a.g.C : a.g.K;
  size_t lds = (size_t)NBUF * (BM + BN) * 64 * sizeof(bf16);
  if (FLAGS & F_PRE) lds += (size_t)2 * Acin * sizeof(float);
  lds = std::max(lds, EpiLayout<BM, BN, WM>::BYTES);
  lds = (lds + 15) & ~(size_t)15;
  dim3 grid((a.M + BM - 1) / BM, (a.Ncol + BN - 1) / BN, a.par ? 4 : 1);
  // the pipelined FAST loop is instantiated for the wide-column (ImageNet) tiles
  if constexpr (NBUF == 1) {   // general loop only (launch_cfg: one-tile K loops)
    if (query) return;
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, MODE, FLAGS, false, 1>), grid,
                       dim3(256), lds, s, a);
    DTR_CHECK_LAUNCH();
  } else {
    if constexpr (BN >= 64) {
      const bool ring = BM == 128 && (BN == 128 || (BN == 64 && WM == 4)) && (FLAGS & F_PRE) == 0 &&
                        conv_ring_covers(a, MODE);
      if (ring || conv_gemm_fast(a, MODE)) {
        const long tiles = (long)grid.x * grid.y;
        const int S = a.par ? 1 : pick_ksplit(tiles, (a.Kdim + 63) / 64);
        const size_t need = (size_t)S * tiles * BM * BN * sizeof(float);
        if (g_sk_query) {
          if (S > 1) {
            g_sk_query->bytes = need;
            g_sk_query->tiles = (size_t)tiles;
          }
          return;
        }
        float* part = a.sk_part;
        unsigned* cnt = a.sk_cnt;
        // a plan's op brings its stream's workspace (sized at record time); an immediate
        // call uses the per-device one
        const bool ok = part != nullptr ? true
                                         : splitk_workspace(need, (size_t)tiles, s, &part, &cnt);
        if (S > 1 && ok) {
          a.ksplit = S;
          a.sk_part = part;
          a.sk_cnt = cnt;
          grid.z = S;
        }
        if (ring) {
          conv_ring(a, MODE, FLAGS, grid, s);
          return;
        }
        hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, MODE, FLAGS, true, NBUF>), grid,
                           dim3(256), lds, s, a);
        DTR_CHECK_LAUNCH();
        return;
      }
    }
    if (query) return;
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, MODE, FLAGS, false, NBUF>), grid,
                       dim3(256), lds, s, a);
    DTR_CHECK_LAUNCH();
  }
}

template <int BM, int BN, int WM, int WN, int MODE>
static void launch_flags(const GemmArgs& a, hipStream_t s) {
  const bool pre = a.pre_scale != nullptr, st = a.stat_part != nullptr;
  const bool bnb = a.bnb_part != nullptr;
  if constexpr (MODE == MODE_FWD) {
    if (pre && st) launch_cfg<BM, BN, WM, WN, MODE, F_PRE | F_STATS>(a, s);
    else if (pre) launch_cfg<BM, BN, WM, WN, MODE, F_PRE>(a, s);
    else if (st) launch_cfg<BM, BN, WM, WN, MODE, F_STATS>(a, s);
    else launch_cfg<BM, BN, WM, WN, MODE, 0>(a, s);
  } else {
    if (bnb) launch_cfg<BM, BN, WM, WN, MODE, F_BNB>(a, s);
    else launch_cfg<BM, BN, WM, WN, MODE, 0>(a, s);
  }
}

// Tile selection: one function of (rows M = images x output pixels, output columns).
// BM shrinks with M so the grid still covers the 256 CUs.  Shared by the launcher and
// by the host (the BN-stat partial buffer has one row per M tile).  The narrow-column
// rows are the CIFAR shapes, measured per per-rank batch on MI355X (CIFAR RN50 step,
// round 3; these replaced the smallc_bm16/32 and c16_mid/c32_mid keys):
//   16 columns (32x32 maps): 256 rows from 128 images (M >= 131072), 128 from 32 images
//     (bs64 1.233 -> 1.08 ms against 64), 64 below;
//   32 columns (16x16 maps): 128 rows from 32768 rows (bs128 1.303 -> 1.273 ms against
//     64), 64 below;
//   64 columns: 128 rows from 32768, else 64.
// Per-rank CIFAR batches <= 240 take the persistent step instead (train/persist.py).
int conv_gemm_bm(int M, int nc) {
  const long m = M;
  if (nc <= 16) return m >= 256L * 512 ? 256 : m >= 32768 ? 128 : 64;
  if (nc <= 32) return m >= 32768 ? 128 : 64;
  if (nc <= 64) return m >= 128L * 256 ? 128 : 64;
  return (m >= tune(T_BM128_MIN) && nc % 128 == 0) ? 128 : 64;
}

int conv_gemm_bn(int M, int nc) {
  if (nc <= 16) return 16;
  if (nc <= 32) return 32;
  if (nc <= 64) return 64;
  return conv_gemm_bm(M, nc) == 128 ? 128 : 64;
}

template <int MODE>
static void launch_mode(const GemmArgs& a, hipStream_t s) {
  const int nc = a.Ncol;
  const int bm = conv_gemm_bm(a.M, nc);
  if (nc <= 16) {
    if (bm == 256) launch_flags<256, 16, 4, 1, MODE>(a, s);
    else if (bm == 128) launch_flags<128, 16, 4, 1, MODE>(a, s);
    else launch_flags<64, 16, 4, 1, MODE>(a, s);
  } else if (nc <= 32) {
    if (bm == 128) launch_flags<128, 32, 4, 1, MODE>(a, s);
    else launch_flags<64, 32, 4, 1, MODE>(a, s);
  } else if (nc <= 64) {
    if (bm == 128) launch_flags<128, 64, 4, 1, MODE>(a, s);
    else launch_flags<64, 64, 4, 1, MODE>(a, s);
  } else {
    if (bm == 128) launch_flags<128, 128, 2, 2, MODE>(a, s);
    else launch_flags<64, 64, 4, 1, MODE>(a, s);
  }
}

void set_conv_parity(int enabled) { tune_set(T_PARITY_DGRAD, enabled ? 1 : 0); }

// Stride-2 dgrad as 4 parity classes of output pixels (one launch, blockIdx.z = class):
// a pixel with (h + pad, w + pad) = (ph, pw) mod 2 only receives the filter taps r = ph,
// ph + 2, .. and s = pw, pw + 2, .., so each class is a dense implicit GEMM over a
// quarter of the rows and its own taps -- instead of every pixel running all kh x kw
// taps with 3/4 of the (pixel, tap) pairs masked to zero (ImageNet's stride-2 dgrads
// ran 3-3.5x slower than their forward convs).  Not with tile-partial BN sums (their
// layout is per row tile of the whole output).
static bool parity_dgrad(const GemmArgs& a) {
  return tune(T_PARITY_DGRAD) && a.g.stride == 2 &&
         (a.bnb_part == nullptr || a.bnb_acc != nullptr) && a.out_f32 == nullptr &&
         a.bias == nullptr && a.residual == nullptr;
}

// Whether conv_gemm(a, mode) takes the LDS-DMA ring loop (tests, diagnostics): the
// dispatcher's own decisions -- direct kernel, parity classes, tile, ring coverage.
bool conv_gemm_uses_ring(const GemmArgs& a0, int mode) {
  if (conv_direct_covers(a0, mode)) return false;
  GemmArgs a = a0;
  if (mode == MODE_DGRAD && parity_dgrad(a)) {
    const ConvGeom& g = a.g;
    a.par = 1;
    a.M = g.N * ((g.H + 1) >> 1) * ((g.W + 1) >> 1);
    a.Kdim = ((g.kh + 1) >> 1) * ((g.kw + 1) >> 1) * g.K;
  }
  return conv_ring_covers(a, mode);
}

size_t conv_gemm_splitk_need(const GemmArgs& a, int mode, size_t* tiles) {
  SplitKNeed need;
  if (!conv_direct_covers(a, mode)) {
    g_sk_query = &need;
    try {
      conv_gemm(a, mode, nullptr);
    } catch (...) {
      g_sk_query = nullptr;
      throw;
    }
    g_sk_query = nullptr;
  }
  if (tiles) *tiles = need.tiles;
  return need.bytes;
}

void conv_gemm(const GemmArgs& a, int mode, hipStream_t s) {
  if (g_sk_query == nullptr && conv_direct(a, mode, s)) return;
  if (a.abwd.x != nullptr)
    throw std::runtime_error("conv_gemm: the fused BN backward (abwd) is direct-conv only");
  if (mode == MODE_FWD) {
    launch_mode<MODE_FWD>(a, s);
  } else if (parity_dgrad(a)) {
    GemmArgs b = a;   // tiles / FAST chosen for the largest class (the kernel derives its own)
    const ConvGeom& g = a.g;
    b.par = 1;
    b.M = g.N * ((g.H + 1) >> 1) * ((g.W + 1) >> 1);
    b.Kdim = ((g.kh + 1) >> 1) * ((g.kw + 1) >> 1) * g.K;
    launch_mode<MODE_DGRAD>(b, s);
  } else {
    launch_mode<MODE_DGRAD>(a, s);
  }
}

}  // namespace dtr
