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
// destination, out-of-range padding reads land as zeros) into a ring of SLOTS 16 KiB
// operand slots (one slot = the A or the B tile of one 64-deep K step); operand load j
// (A of tile j / 2 for even j, B for odd j) goes to slot j % SLOTS:
//
//   prologue: issue operand loads 0 .. SLOTS-3
//   tile t:   s_waitcnt vmcnt(4 (SLOTS-4))  this wave's DMAs of A_t and B_t have landed
//             s_barrier                      ... every wave's; tile t-1's two slots are free
//             issue the next two operand loads into them
//             32 MFMA per wave on tile t's slots
//
// so (SLOTS - 2) / 2 K tiles are in flight beside the one being multiplied.  Built with
// SLOTS = 4 (64 KiB, two workgroups per CU, one tile ahead).  Measured alternatives
// (profiles/imagenet_resnet50_ring.md, in-process A/B over the RN50 layers): 5 slots
// (80 KiB, still two workgroups per CU, 1.5 tiles ahead) tie; 6 and 8 slots (one
// workgroup per CU, 2-3 tiles ahead) are 10-50 % slower -- with one wave per SIMD
// nothing covers the LDS-read latency after each barrier or the epilogue.  What the
// ring wins over the register loop is issue work (no VGPR staging, ds_write pass or
// per-chunk index math), not memory-level parallelism.
//
// One raw barrier per K tile and counted waits only: __syncthreads() would add the
// vmcnt(0) that drains the ring (cdna_hip_programming.md, "Pipelining across
// barriers").  Every wave issues exactly 4 DMAs per operand load (loads past the end
// are issued out of range), so the count is exact.  The LDS image is the XOR-swizzled
// [row][64] bf16 layout of conv_gemm.hip; since a DMA's LDS destination is lane-linear
// (wave base + 16 B x lane), the swizzle goes on the SOURCE: lane l of a 1 KiB piece
// covers row l / 8, slot l % 8, and fetches k-chunk (l % 8) ^ (row % 8).
//
// Per lane and K tile the gather is one add (row offset + scalar tap offset) and a
// tap-validity bit (a per-row mask of the filter taps, built once), instead of the
// per-chunk index math of the register loop; the tap walks (tap, channel base) of the
// A and B issue pointers advance on the scalar unit.
#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "conv_epilogue.h"

namespace dtr {

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int kRingOOB = 0x7fff0000;   // buffer offset past every operand (reads zeros)

template <int n>
__device__ __forceinline__ void ring_wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  // s_waitcnt: vmcnt n (bits 3:0 + 15:14), expcnt / lgkmcnt left at their maxima
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}

}  // namespace

template <int MODE, int FLAGS, int SLOTS>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(SLOTS <= 5 ? 2 : 1, SLOTS <= 5 ? 2 : 1)))
conv_ring_kernel(GemmArgs args) {
  constexpr int BM = 128, BN = 128, WM = 2, WN = 2, BK = 64;
  constexpr int MR = BM / WM / 16, NR = BN / WN / 16;
  constexpr int OP_B = BM * BK * 2;      // bytes of one operand tile (one slot)
  constexpr bool BNB = (FLAGS & F_BNB) != 0;
  static_assert((FLAGS & (F_PRE | F_ABWD)) == 0, "no A-operand prologue on the ring");
  static_assert(SLOTS >= 4 && SLOTS <= 8, "4-8 operand slots");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ConvGeom& g = args.g;
  int par_ph = 0, par_pw = 0;
  if (MODE == MODE_DGRAD && args.par) {   // stride-2 dgrad parity class (see conv_gemm.hip)
    par_ph = blockIdx.z >> 1;
    par_pw = blockIdx.z & 1;
    args.par_h0 = (par_ph + g.pad) & 1;
    args.par_w0 = (par_pw + g.pad) & 1;
    args.par_hc = (g.H - args.par_h0 + 1) >> 1;
    args.par_wc = (g.W - args.par_w0 + 1) >> 1;
    args.M = g.N * args.par_hc * args.par_wc;
    args.Kdim = ((g.kh - par_ph + 1) >> 1) * ((g.kw - par_pw + 1) >> 1) * g.K;
  }
  const int M = args.M, NC = args.Ncol, KD = args.Kdim;
  if (MODE == MODE_DGRAD && args.par && (int)(blockIdx.x * BM) >= M) return;
  const bool par = MODE == MODE_DGRAD && args.par;
  // taps of this launch (class): rows ta < tah, columns tb < taw
  const int taw = par ? (g.kw - par_pw + 1) >> 1 : g.kw;
  const int Acin = MODE == MODE_FWD ? g.C : g.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tm = blockIdx.x, tn = blockIdx.y;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-lane gather state: rows (wave * 4 + i) * 8 + lane / 8, chunk kg ----
  const int lr = lane >> 3;
  const int kg = (lane & 7) ^ lr;                 // source-side swizzle
  int a_off[4];                                    // bytes, valid-tap base
  unsigned a_mask[4];                              // bit tl: class-local tap tl is in range
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
    const int nrow = n0 + r;
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
  const int sk_n = args.ksplit > 1 ? args.ksplit : 1, sk_z = sk_n > 1 ? (int)blockIdx.z : 0;
  const int t_beg = (int)(((long)sk_z * KT_all) / sk_n);
  const int t_end = (int)(((long)(sk_z + 1) * KT_all) / sk_n);
  const int cpt = Acin / BK;                       // K tiles per tap
  struct Walk {                                    // issue pointer: tile, tap, channel base
    int t, tl, c, ta, tb;
  };
  Walk wa, wb;
  wa.t = t_beg;
  wa.tl = t_beg / cpt;
  wa.c = (t_beg - wa.tl * cpt) * BK;
  wa.ta = wa.tl / taw;
  wa.tb = wa.tl - wa.ta * taw;
  wb = wa;
  auto advance = [&](Walk& w) {
    ++w.t;
    w.c += BK;
    if (w.c == Acin) {
      w.c = 0;
      ++w.tl;
      if (++w.tb == taw) {
        w.tb = 0;
        ++w.ta;
      }
    }
  };
  // operand load j -> slot j % SLOTS: A of tile wa.t (even j) or B of tile wb.t (odd j)
  auto issue_a = [&](int slot) {
    const bool live = wa.t < t_end;
    const int a_pix = MODE == MODE_FWD ? wa.ta * g.W + wa.tb : -(wa.ta * g.Wo + wa.tb);
    const int sa = live ? (a_pix * Acin + wa.c) * 2 : kRingOOB;
    char* st = smem + slot * OP_B;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = (a_mask[i] >> (wa.tl & 31)) & 1u;   // (tail tiles: sa is out of range)
      const int off = ok ? a_off[i] + sa : kRingOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_a, (lds_void*)(st + (wave * 4 + i) * 1024), 16, off, 0, 0, 0);
    }
    advance(wa);
  };
  auto issue_b = [&](int slot) {
    const bool live = wb.t < t_end;
    int b_bytes;
    if constexpr (MODE == MODE_FWD) {
      b_bytes = (wb.tl * Acin + wb.c) * 2;
    } else {
      const int rr = par ? par_ph + 2 * wb.ta : wb.ta, cc = par ? par_pw + 2 * wb.tb : wb.tb;
      b_bytes = ((rr * g.kw + cc) * g.C * g.K + wb.c) * 2;
    }
    const int sb = live ? b_bytes : kRingOOB;
    char* st = smem + slot * OP_B;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_b, (lds_void*)(st + (wave * 4 + i) * 1024), 16, b_off[i] + sb, 0, 0, 0);
    advance(wb);
  };
  int j_issue = 0, slot_issue = 0;
  auto issue_next = [&]() {
    if (j_issue & 1) issue_b(slot_issue);
    else issue_a(slot_issue);
    ++j_issue;
    slot_issue = slot_issue + 1 == SLOTS ? 0 : slot_issue + 1;
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto mma_slots = [&](int sa, int sb) {
    const bf16* A = reinterpret_cast<const bf16*>(smem + sa * OP_B);
    const bf16* B = reinterpret_cast<const bf16*>(smem + sb * OP_B);
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

  // ---- prologue: SLOTS - 2 operand loads in flight ----
#pragma unroll
  for (int j = 0; j < SLOTS - 2; ++j) issue_next();
  int rd = 0;   // slot of A_t (B_t in the next)
  for (int t = t_beg; t < t_end; ++t) {
    ring_wait_vm<4 * (SLOTS - 4)>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue_next();
    issue_next();
    const int rb = rd + 1 == SLOTS ? 0 : rd + 1;
    mma_slots(rd, rb);
    rd = rb + 1 == SLOTS ? 0 : rb + 1;
  }
  // drain the ring (the over-issued tail DMAs too) before the epilogue reuses the LDS
  ring_wait_vm<0>();
  __syncthreads();

  if (sk_n > 1 && !splitk_combine<MR, NR>(args, acc, smem, tm, tn)) return;
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
  if (Acin % 64 != 0 || a.Ncol % 128 != 0 || conv_gemm_bm(a.M, a.Ncol) != 128) return false;
  const long a_elems = mode == MODE_FWD ? (long)g.N * g.H * g.W * g.C
                                        : (long)g.N * g.Ho * g.Wo * g.K;
  const long b_elems = (long)g.kh * g.kw * g.C * g.K;
  if (a_elems >= (1L << 30) || b_elems >= (1L << 30) || g.kh * g.kw > 32) return false;
  if (mode == MODE_DGRAD && g.stride != 1 && !a.par) return false;   // non-linear taps
  return (a.Kdim + 63) / 64 >= tune(T_RING_KT);
}

template <int MODE, int FLAGS, int SLOTS>
static void ring_launch(GemmArgs a, dim3 grid, hipStream_t s) {
  size_t lds = std::max((size_t)SLOTS * 16 * 1024, EpiLayout<128, 128, 2>::BYTES);
  hipLaunchKernelGGL((conv_ring_kernel<MODE, FLAGS, SLOTS>), grid, dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

void conv_ring(const GemmArgs& a, int mode, int flags, dim3 grid, hipStream_t s) {
  if (mode == MODE_FWD) {
    if (flags & F_STATS) ring_launch<MODE_FWD, F_STATS, 4>(a, grid, s);
    else ring_launch<MODE_FWD, 0, 4>(a, grid, s);
  } else {
    if (flags & F_BNB) ring_launch<MODE_DGRAD, F_BNB, 4>(a, grid, s);
    else ring_launch<MODE_DGRAD, 0, 4>(a, grid, s);
  }
}

}  // namespace dtr
