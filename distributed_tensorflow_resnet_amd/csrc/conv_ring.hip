// LDS-DMA ring implicit-GEMM convolution for the 128x128 tiles of the ImageNet layers
// (forward without the BN+ReLU prologue, and data gradient) on gfx950.
//
// Same GEMM as conv_gemm.hip (reference: cuDNN Conv2D / Conv2DBackpropInput emitted by
// conv2d_fixed_padding, resnet_model_official.py:80-91) and the same epilogue
// (conv_epilogue.h: bias / residual / accumulate, BN statistics, BN backward sums,
// split-K combine), but a different main loop, chosen by what the per-layer PMC table
// measured (profiles/imagenet_resnet50_pmc_bytes.md): the register-staged loop of
// conv_gemm.hip keeps about one 32 KiB K tile per workgroup in flight, ~2 us per K tile
// on the 14x14 / 7x7 3x3 layers -- ~24 GB/s per CU, i.e. ~390 TF/s at the tile's
// 64 FLOP/B -- with HBM bytes at their floor and MFMA 17 % busy: a memory-level
// parallelism bound, not a byte or MFMA bound.
//
// Here both operands go global -> LDS by buffer_load ... lds (16 B per lane, no VGPR
// destination, out-of-range padding reads land as zeros) into a 2-stage LDS ring:
//
//   prologue: issue K tile 0 into stage 0
//   tile t:   s_waitcnt vmcnt(0)   this wave's DMAs of tile t have landed
//             s_barrier            ... every wave's; stage (t+1) % 2 (tile t-1) is free
//             issue tile t+1 into stage (t+1) % 2
//             MFMAs on stage t % 2
//
// Tiles BM x BN = 128 x 128 (4 waves 2 x 2, 48-64 KiB LDS: two workgroups per CU) and
// 128 x 64 (4 waves 4 x 1, the 64-channel stage-1 layers).  Measured alternatives
// (profiles/imagenet_resnet50_ring.md, in-process A/B over the RN50 layers): a ring of
// five 16 KiB operand slots (80 KiB, still two workgroups per CU, 1.5 tiles ahead) tied
// this one; 3-4 stages (one workgroup per CU, 2-3 tiles ahead) were 10-50 % slower --
// with one wave per SIMD nothing covers the LDS-read latency after each barrier or the
// epilogue.  What the ring wins over the register loop is issue work (no VGPR staging,
// no ds_write pass, no per-chunk index math), not memory-level parallelism.
//
// One raw barrier per K tile: __syncthreads() would add a vmcnt(0) that also drains the
// epilogue operands prefetched at kernel start.  The LDS image is the XOR-swizzled
// [row][64] bf16 layout of conv_gemm.hip; since a DMA's LDS destination is lane-linear
// (wave base + 16 B x lane), the swizzle goes on the SOURCE: lane l of a 1 KiB piece
// covers row l / 8, slot l % 8, and fetches k-chunk (l % 8) ^ (row % 8).
//
// Per lane and K tile the gather is one add (row offset + scalar tap offset) and a
// tap-validity bit (a per-row mask of the filter taps, built once), instead of the
// per-chunk index math of the register loop; the tap walk (tap, channel base) of the
// issue pointer advances on the scalar unit.
#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "conv_epilogue.h"

namespace dtr {

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int kRingOOB = 0x7fff0000;   // buffer offset past every operand (reads zeros)
constexpr int STAGE_A_BYTES = 128 * 64 * 2;   // the A tile (128 rows x 64 k) of a ring stage

template <int n>
__device__ __forceinline__ void ring_wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  // s_waitcnt: vmcnt n (bits 3:0 + 15:14), expcnt / lgkmcnt left at their maxima
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}

}  // namespace

template <int MODE, int FLAGS, int BN>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(2, 2)))
conv_ring_kernel(GemmArgs args) {
  constexpr int BM = 128, BK = 64;
  constexpr int WM = BN == 128 ? 2 : 4, WN = 4 / WM;
  constexpr int MR = BM / WM / 16, NR = BN / WN / 16;
  static_assert(BM * BK * 2 == STAGE_A_BYTES, "A tile bytes");   // stage: A, then B (BN x BK)
  constexpr bool BNB = (FLAGS & F_BNB) != 0;
  static_assert((FLAGS & (F_PRE | F_ABWD)) == 0, "no A-operand prologue on the ring");
  static_assert(BN == 128 || BN == 64, "128 x 128 or 128 x 64 tiles");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ConvGeom& g = args.g;
  const int tm = blockIdx.x, tn = blockIdx.y, lz = blockIdx.z;
  int par_ph = 0, par_pw = 0;
  if (MODE == MODE_DGRAD && args.par) {   // stride-2 dgrad parity class (see conv_gemm.hip)
    par_ph = lz >> 1;
    par_pw = lz & 1;
    args.par_h0 = (par_ph + g.pad) & 1;
    args.par_w0 = (par_pw + g.pad) & 1;
    args.par_hc = (g.H - args.par_h0 + 1) >> 1;
    args.par_wc = (g.W - args.par_w0 + 1) >> 1;
    args.M = g.N * args.par_hc * args.par_wc;
    args.Kdim = ((g.kh - par_ph + 1) >> 1) * ((g.kw - par_pw + 1) >> 1) * g.K;
  }
  const int M = args.M, NC = args.Ncol, KD = args.Kdim;
  if (MODE == MODE_DGRAD && args.par && tm * BM >= M) return;
  const bool par = MODE == MODE_DGRAD && args.par;
  // taps of this launch (class): rows ta < tah, columns tb < taw
  const int taw = par ? (g.kw - par_pw + 1) >> 1 : g.kw;
  const int Acin = MODE == MODE_FWD ? g.C : g.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-lane gather state: rows (wave * 4 + i) * 8 + lane / 8, chunk kg ----
  const int lr = lane >> 3;
  const int kg = (lane & 7) ^ lr;                 // source-side swizzle
  int a_off[4];                                    // bytes, valid-tap base
  unsigned a_mask[4];                              // bit tl: class-local tap tl is in range
  // B DMAs (8 rows each) per wave and tile: BN / 32 of the 4 used.  Fixed size on purpose:
  // a lambda capturing an array whose size depends on a template parameter made hipcc
  // (ROCm 7.2) silently drop the kernel's host stub -- an undefined symbol at load time.
  int b_off[4];
  const int ntap = (par ? ((g.kh - par_ph + 1) >> 1) : g.kh) * taw;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (wave * 4 + i) * 8 + lr;
    const int m = m0 + r;
    unsigned mask = 0u;
    long pix = 0;
    if (m < M) {
      if constexpr (MODE == MODE_FWD) {
        const int hw = g.Ho * g.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
        const int h0 = ho * g.stride - g.pad, w0 = wo * g.stride - g.pad;
        pix = (long)n * g.H * g.W + (long)h0 * g.W + w0;        // pixel of tap (0, 0)
        for (int tl = 0; tl < ntap; ++tl) {
          const int rr = tl / taw, cc = tl - rr * taw;
          if ((unsigned)(h0 + rr) < (unsigned)g.H && (unsigned)(w0 + cc) < (unsigned)g.W)
            mask |= 1u << tl;
        }
      } else {
        int n, h, w;
        if (par) {
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
        // dy pixel of tap (0, 0); tap (ta, tb) moves it by -(ta * Wo + tb)
        int hp0, wp0;
        if (par) {   // (h + pad - (ph + 2 ta)) / 2 = hp0 - ta  (exact: even numerator)
          hp0 = (h + g.pad - par_ph) >> 1;
          wp0 = (w + g.pad - par_pw) >> 1;
        } else {
          hp0 = h + g.pad;
          wp0 = w + g.pad;
        }
        pix = (long)n * g.Ho * g.Wo + (long)hp0 * g.Wo + wp0;
        for (int tl = 0; tl < ntap; ++tl) {
          const int ta = tl / taw, tb = tl - ta * taw;
          if ((unsigned)(hp0 - ta) < (unsigned)g.Ho && (unsigned)(wp0 - tb) < (unsigned)g.Wo)
            mask |= 1u << tl;
        }
      }
    }
    a_mask[i] = mask;
    a_off[i] = mask ? (int)((pix * Acin + kg * 8) * 2) : 0;
  }
#pragma unroll
  for (int i = 0; i < BN / 32; ++i) {
    const int nrow = n0 + (wave * (BN / 32) + i) * 8 + lr;
    if constexpr (MODE == MODE_FWD) b_off[i] = nrow < NC ? (nrow * KD + kg * 8) * 2 : kRingOOB;
    else b_off[i] = nrow < NC ? (nrow * g.K + kg * 8) * 2 : kRingOOB;
  }
  const long a_elems = MODE == MODE_FWD ? (long)g.N * g.H * g.W * g.C
                                        : (long)g.N * g.Ho * g.Wo * g.K;
  const long b_elems = (long)g.kh * g.kw * g.C * g.K;
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.a), 0,
                                                      (int)(a_elems * 2), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.b), 0,
                                                      (int)(b_elems * 2), 0x00020000);

  // ---- K range of this split-K slice; scalar tap walk of the issue pointer ----
  const int KT_all = (KD + BK - 1) / BK;
  const int sk_n = args.ksplit > 1 ? args.ksplit : 1, sk_z = sk_n > 1 ? lz : 0;
  const int t_beg = (int)(((long)sk_z * KT_all) / sk_n);
  const int t_end = (int)(((long)(sk_z + 1) * KT_all) / sk_n);
  const int cpt = Acin / BK;                       // K tiles per tap
  int it_t = t_beg;                                // issue pointer: tile, tap, channel
  int it_tl = t_beg / cpt;
  int it_c = (t_beg - it_tl * cpt) * BK;
  int it_ta = it_tl / taw, it_tb = it_tl - it_ta * taw;
  auto issue = [&](int stage) {   // tile it_t -> stage: 4 A + BN / 32 B DMAs per wave
    const int a_pix = MODE == MODE_FWD ? it_ta * g.W + it_tb : -(it_ta * g.Wo + it_tb);
    const int sa = (a_pix * Acin + it_c) * 2;
    int sb;
    if constexpr (MODE == MODE_FWD) {
      sb = (it_tl * Acin + it_c) * 2;
    } else {
      const int rr = par ? par_ph + 2 * it_ta : it_ta, cc = par ? par_pw + 2 * it_tb : it_tb;
      sb = ((rr * g.kw + cc) * g.C * g.K + it_c) * 2;
    }
    char* st = smem + stage * (STAGE_A_BYTES + BN * 128);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = (a_mask[i] >> it_tl) & 1u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_a, (lds_void*)(st + (wave * 4 + i) * 1024), 16, ok ? a_off[i] + sa : kRingOOB, 0, 0,
          0);
    }
    char* const stb = st + STAGE_A_BYTES;
#pragma unroll
    for (int i = 0; i < BN / 32; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_b, (lds_void*)(stb + (wave * (BN / 32) + i) * 1024), 16, b_off[i] + sb, 0, 0, 0);
    ++it_t;
    it_c += BK;
    if (it_c == Acin) {
      it_c = 0;
      ++it_tl;
      if (++it_tb == taw) {
        it_tb = 0;
        ++it_ta;
      }
    }
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto mma_stage = [&](int stage) {
    const bf16* A = reinterpret_cast<const bf16*>(smem + stage * (STAGE_A_BYTES + BN * 128));
    const bf16* B = reinterpret_cast<const bf16*>(smem + stage * (STAGE_A_BYTES + BN * 128) +
                                                  STAGE_A_BYTES);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;
      bf16x8 af[MR], bfr[NR];
#pragma unroll
      for (int a = 0; a < MR; ++a) {
        const int r = wm * (BM / WM) + a * 16 + fr;
        af[a] = *reinterpret_cast<const bf16x8*>(A + r * BK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int r = wn * (BN / WN) + b * 16 + fr;
        bfr[b] = *reinterpret_cast<const bf16x8*>(B + r * BK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int b = 0; b < NR; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
  };

  // dgrad + BN-backward sums: the epilogue's BN-input rows / coefficients, loaded now
  using EP = EpiPre<BM, BN, WM, true>;
  EP epre;
  if constexpr (BNB) epi_prefetch<BM, BN, WM, FLAGS, true>(args, m0, n0, epre);

  // ---- 2-stage ring: tile t+1 in flight during the MFMAs of tile t ----
  issue(0);
  int rd = 0;
  for (int t = t_beg; t < t_end; ++t) {
    ring_wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < t_end) issue(rd ^ 1);
    mma_stage(rd);
    rd ^= 1;
  }
  __syncthreads();   // every wave's MFMA reads are done: the epilogue reuses the LDS

  if (sk_n > 1 && !splitk_combine<MR, NR>(args, acc, smem, tm, tn, lz)) return;
  if constexpr (BNB && EP::ON)
    conv_epilogue<BM, BN, WM, WN, FLAGS, true>(args, acc, smem, m0, n0, &epre, tm, tn);
  else
    conv_epilogue<BM, BN, WM, WN, FLAGS, false>(args, acc, smem, m0, n0, nullptr, tm, tn);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool conv_ring_covers(const GemmArgs& a, int mode) {
  if (!tune(T_RING)) return false;
  const ConvGeom& g = a.g;
  const int Acin = mode == MODE_FWD ? g.C : g.K;
  if (a.pre_scale != nullptr || a.abwd.x != nullptr) return false;
  if (Acin % 64 != 0 || a.Ncol % 64 != 0 || conv_gemm_bm(a.M, a.Ncol) != 128) return false;
  const int bn = conv_gemm_bn(a.M, a.Ncol);
  if (bn != 128 && bn != 64) return false;
  const long a_elems = mode == MODE_FWD ? (long)g.N * g.H * g.W * g.C
                                        : (long)g.N * g.Ho * g.Wo * g.K;
  const long b_elems = (long)g.kh * g.kw * g.C * g.K;
  if (a_elems >= (1L << 30) || b_elems >= (1L << 30) || g.kh * g.kw > 32) return false;
  if (mode == MODE_DGRAD && g.stride != 1 && !a.par) return false;   // non-linear taps
  const long kt_min = mode == MODE_FWD ? tune(T_RING_KT) : tune(T_RING_KT_DGRAD);
  return (a.Kdim + 63) / 64 >= kt_min;
}

template <int MODE, int FLAGS, int BN>
static void ring_launch(GemmArgs a, dim3 grid, hipStream_t s) {
  constexpr int WM = BN == 128 ? 2 : 4;
  const size_t lds = std::max((size_t)2 * (128 + BN) * 64 * 2, EpiLayout<128, BN, WM>::BYTES);
  hipLaunchKernelGGL((conv_ring_kernel<MODE, FLAGS, BN>), grid, dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

template <int BN>
static void ring_flags(const GemmArgs& a, int mode, int flags, dim3 grid, hipStream_t s) {
  if (mode == MODE_FWD) {
    if (flags & F_STATS) ring_launch<MODE_FWD, F_STATS, BN>(a, grid, s);
    else ring_launch<MODE_FWD, 0, BN>(a, grid, s);
  } else {
    if (flags & F_BNB) ring_launch<MODE_DGRAD, F_BNB, BN>(a, grid, s);
    else ring_launch<MODE_DGRAD, 0, BN>(a, grid, s);
  }
}

void conv_ring(const GemmArgs& a, int mode, int flags, dim3 grid, hipStream_t s) {
  if (conv_gemm_bn(a.M, a.Ncol) == 128) ring_flags<128>(a, mode, flags, grid, s);
  else ring_flags<64>(a, mode, flags, grid, s);
}

}  // namespace dtr
