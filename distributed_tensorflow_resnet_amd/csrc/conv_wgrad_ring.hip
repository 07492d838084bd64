// Weight gradient on an LDS-DMA ring (128 x 128 output tiles: every ImageNet ResNet-50
// layer with >= 128 output channels and >= 128 (tap, channel) columns).
//
// Same GEMM, LDS image, transposed fragment reads, split-K partial slabs and reduce as
// conv_wgrad.hip (dW[co][tap][ci] = sum_p DY[p][co] * X[p shifted by tap][ci]; replaces
// cuDNN Conv2DBackpropFilter), but both operands go global -> LDS by
// buffer_load ... lds (16 B per lane, no VGPR destination), as in conv_ring.hip:
//
//   tile t:  s_waitcnt vmcnt(0)            this thread's DMAs of K tile t have landed
//            [PRE] BN+ReLU in place on this thread's own B chunks (padding stays 0)
//            s_barrier                     every thread's chunks are in LDS
//            issue K tile t+1 into the other stage
//            MFMAs on tile t (ds_read_b64_tr_b16 fragments)
//
// Why: the backward pass is throughput-bound -- skipping the weight gradients (timing
// only) takes the RN50 bs128 backward from 7.92 to 5.91 ms -- so the side-stream wgrads'
// issue work (VGPR staging, per-chunk index math, ds_write pass) costs the critical path.
//
// LDS image (per stage, A then B): [64 pixel rows][128 columns] bf16, 32-byte units XOR
// row % 8 (conv_wgrad.hip unit_swz<8>).  A DMA's destination is lane-linear (wave base
// + 16 B x lane: 4 rows of 256 B), so the swizzle goes on the SOURCE: lane l covers row
// l / 16, slot l % 16, and fetches the 16-B chunk whose 32-B unit is (slot / 2) ^ (row %
// 8).  Rows (wave * 4 + i) * 4 + l / 16 have row % 8 = (4 i + l / 16) % 8, so a lane's
// B chunks use two columns only: their (tap, channel) and BN coefficients are fixed.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace dtr {

namespace {

typedef __attribute__((address_space(3))) void lds_void;
constexpr int kWrOOB = 0x7fff0000;   // buffer offset past every operand (reads zeros)
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Raw buffer descriptor (base, 0 stride, num_records bytes, the same dword3 as
// __builtin_amdgcn_make_buffer_rsrc's 0x00020000) for the inline-asm DMA below.
__device__ __forceinline__ i32x4 buf_rsrc(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32) & 0xffff);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000;
  return r;
}

// buffer_load_dwordx4 ... lds (16 B per lane, lane-linear at M0 = the wave's LDS base) as
// inline asm.  Through the builtin, hipcc treats the DMA as a pending LDS write that may
// alias every ds_read: it waited vmcnt(0) right after each K tile's issue, before the
// ds_reads of the tile being computed -- no DMA ever overlapped this wave's MFMAs (only
// the second workgroup on the CU's).  Invisible to the compiler's counters, the DMAs are
// waited for only by this kernel's own counted vmcnt at the top of the K loop (no other
// vector-memory load is in flight in the loop).
__device__ __forceinline__ void dma16(const i32x4& rsrc, unsigned lds_base, int voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds_base), "v"(voff), "s"(rsrc) : "m0");
}

}  // namespace

// Two LDS stages (each K tile's A and B images, 32 KiB): one tile in flight beside the
// MFMAs, two workgroups per CU.  Tiles past the slice's end are issued all out-of-range
// (zeros, never read), so every wait is the same vmcnt and the loop body has no branch.
// (3 / 4 stages at one workgroup per CU for the grids of <= one workgroup per CU measured
// slower standalone and 1-2 % slower in-step: a 128 KiB workgroup keeps every other
// kernel off its CU; profiles/imagenet_wgrad_r6.md.)
template <bool PRE>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(2, 2)))
conv_wgrad_ring_kernel(WgradArgs args) {
  constexpr int NST = 2;
  constexpr int BM = 128, BN = 128, BK = 64, WN = 2;
  constexpr int WTM = 64, WTN = 64, MR = 4, NR = 4;
  constexpr int OP_B = BK * BM * 2;          // 16 KiB per operand tile
  constexpr int UA = BM / 16, UB = BN / 16;  // 32-byte units per row (8)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ConvGeom& g = args.g;
  const int Cout = g.K, Cin = g.C;
  const int NT = g.kh * g.kw * Cin;
  const int P = g.N * g.Ho * g.Wo;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const unsigned pblk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned lblk = args.xcd ? xcd_logical_block(pblk, gridDim.x * gridDim.y * gridDim.z) : pblk;
  const int n0 = (int)(lblk % gridDim.x) * BN, m0 = (int)((lblk / gridDim.x) % gridDim.y) * BM;
  const int split = (int)(lblk / (gridDim.x * gridDim.y));
  const int p_begin = split * args.px_per_split;
  const int p_end = min(P, p_begin + args.px_per_split);
  const int KT = (p_end - p_begin + BK - 1) / BK;

  const long x_elems = (long)g.N * g.H * g.W * Cin;
  const long dy_elems = (long)P * Cout;
  const i32x4 rs_x = buf_rsrc(args.x, (int)(x_elems * 2));
  const i32x4 rs_dy = buf_rsrc(args.dy, (int)(dy_elems * 2));
  const unsigned lds0 = (unsigned)(unsigned long long)(lds_void*)smem;   // LDS byte address

  // ---- per-lane DMA state: rows r_i = (wave * 4 + i) * 4 + lr, slot sl ----
  const int sl = lane & 15, lr = lane >> 4;
  // 16-B column chunk fetched for rows with row % 8 = lr (even i) / 4 + lr (odd i)
  int cc[2];
  cc[0] = (((sl >> 1) ^ lr) << 1) | (sl & 1);
  cc[1] = (((sl >> 1) ^ (4 + lr)) << 1) | (sl & 1);
  // A: dy channel of each column parity (invalid -> out of range)
  int a_col[2];
  // B: (tap row, tap col, channel) of each column parity
  int b_r[2], b_c[2], b_ci[2];
  bool b_ok[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + cc[j] * 8;
    a_col[j] = m < Cout ? m : -1;
    const int n = n0 + cc[j] * 8;
    b_ok[j] = n < NT;
    const int tap = b_ok[j] ? n / Cin : 0;
    b_ci[j] = n - tap * Cin;
    b_r[j] = tap / g.kw;
    b_c[j] = tap - b_r[j] * g.kw;
  }
  f32x4 ps0[2], ps1[2], pb0[2], pb1[2];   // PRE: BN scale / shift of the two columns
  if constexpr (PRE) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      ps0[j] = b_ok[j] ? *reinterpret_cast<const f32x4*>(args.pre_scale + b_ci[j]) : z;
      ps1[j] = b_ok[j] ? *reinterpret_cast<const f32x4*>(args.pre_scale + b_ci[j] + 4) : z;
      pb0[j] = b_ok[j] ? *reinterpret_cast<const f32x4*>(args.pre_shift + b_ci[j]) : z;
      pb1[j] = b_ok[j] ? *reinterpret_cast<const f32x4*>(args.pre_shift + b_ci[j] + 4) : z;
    }
  }
  // Each of the lane's 4 rows is one pixel, stepped by BK per issued tile.  Its source
  // offsets are kept incrementally in bytes -- A: p * Cout * 2; B: the 3x3 window origin
  // ((img * H + hs) * W + ws) * Cin * 2 with hs = ho * stride - pad, ws = wo * stride - pad
  // -- so a tile's 8 DMA addresses cost adds and selects, no multiply: with one workgroup
  // per CU (the slab-capped deep-K grids) the per-tile address chain (quarter-rate 32-bit
  // multiplies and 64-bit mads, one dependent on the next) ran ~0.65 us per K tile,
  // longer than the tile's MFMAs and DMAs together.
  const int S = g.stride;
  const int HoWo = g.Ho * g.Wo;
  const int d_ho = BK / g.Wo, d_wo = BK - d_ho * g.Wo;
  const int Cb = Cin * 2;   // bytes per input pixel
  int prow[4], pa[4], hs[4], ws[4], xb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = p_begin + (wave * 4 + i) * 4 + lr;
    const int img = p / HoWo;
    const int rem = p - img * HoWo;
    const int ho = rem / g.Wo, wo = rem - (rem / g.Wo) * g.Wo;
    prow[i] = p;
    pa[i] = p * Cout * 2;
    hs[i] = ho * S - g.pad;
    ws[i] = wo * S - g.pad;
    xb[i] = ((img * g.H + hs[i]) * g.W + ws[i]) * Cb;
  }
  // per column parity j: A channel bytes, B tap offset bytes from the window origin
  int ta[2], tb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ta[j] = a_col[j] * 2;
    tb[j] = (b_r[j] * g.W + b_c[j]) * Cb + b_ci[j] * 2;
  }
  // stepping constants (uniform): +BK pixels, the row wrap, the image wrap
  const int st_pa = BK * Cout * 2;
  const int st_ws = d_wo * S, st_hs = d_ho * S, st_xb = (d_ho * S * g.W + d_wo * S) * Cb;
  const int w_lim = g.Wo * S - g.pad, w_ws = g.Wo * S, w_xb = (S * g.W - g.Wo * S) * Cb;
  const int h_lim = g.Ho * S - g.pad, h_hs = g.Ho * S, h_xb = (g.H * g.W - g.Ho * S * g.W) * Cb;
  // PRE: which of this lane's 4 B chunks of each issued, unconsumed tile are real, 4 bits
  // per tile in issue order (the oldest in bits 3:0)
  unsigned pend = 0u;

  auto issue = [&](int stage) {   // the rows' next K tile -> stage (4 A + 4 B DMAs per wave)
    const unsigned st = lds0 + stage * 2 * OP_B;
    unsigned msk = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = i & 1;
      // (masks, not ?: on the offsets: hipcc sank those selects into exec-masked
      // branches, one DMA per side)
      const int pok = prow[i] < p_end;
      const int aok = pok & (a_col[j] >= 0);
      const int aoff = kWrOOB + ((pa[i] + ta[j] - kWrOOB) & -aok);
      dma16(rs_dy, st + (wave * 4 + i) * 1024, aoff);
      const int ok = pok & (int)b_ok[j] & ((unsigned)(hs[i] + b_r[j]) < (unsigned)g.H) &
                     ((unsigned)(ws[i] + b_c[j]) < (unsigned)g.W);
      const int boff = kWrOOB + ((xb[i] + tb[j] - kWrOOB) & -ok);
      dma16(rs_x, st + OP_B + (wave * 4 + i) * 1024, boff);
      msk |= (unsigned)ok << i;
      // advance this row's pixel by BK (host: BK / Wo + 1 <= 3 Ho)
      prow[i] += BK;
      pa[i] += st_pa;
      ws[i] += st_ws;
      hs[i] += st_hs;
      xb[i] += st_xb;
      const bool wrap = ws[i] >= w_lim;
      ws[i] -= wrap ? w_ws : 0;
      hs[i] += wrap ? S : 0;
      xb[i] += wrap ? w_xb : 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const bool nxt = hs[i] >= h_lim;
        hs[i] -= nxt ? h_hs : 0;
        xb[i] += nxt ? h_xb : 0;
      }
    }
    pend |= msk << (4 * (NST - 2));
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int gq = lane >> 4, li = lane & 15;
  const int qr = li >> 2, pc = li & 3;
  auto mma_stage = [&](int stage) {
    const bf16* A = reinterpret_cast<const bf16*>(smem + stage * 2 * OP_B);
    const bf16* B = reinterpret_cast<const bf16*>(smem + stage * 2 * OP_B + OP_B);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r1 = ks * 32 + 4 * gq + qr;   // pixel row of elements 0..3
      const int r2 = r1 + 16;                 // ... 4..7
      bf16x8 af[MR], bfr[NR];
#pragma unroll
      for (int a = 0; a < MR; ++a) {
        const int unit = (wm * WTM + a * 16) >> 4;
        const s16x4 lo = lds_read_tr16(A + r1 * BM + ((unit ^ (r1 & (UA - 1))) << 4) + 4 * pc);
        const s16x4 hi = lds_read_tr16(A + r2 * BM + ((unit ^ (r2 & (UA - 1))) << 4) + 4 * pc);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[a] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int unit = (wn * WTN + b * 16) >> 4;
        const s16x4 lo = lds_read_tr16(B + r1 * BN + ((unit ^ (r1 & (UB - 1))) << 4) + 4 * pc);
        const s16x4 hi = lds_read_tr16(B + r2 * BN + ((unit ^ (r2 & (UB - 1))) << 4) + 4 * pc);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[b] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int b = 0; b < NR; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
  };

  // prologue: tiles 0 .. NST-2 in flight
  if (KT > 0) {
#pragma unroll
    for (int i = 0; i < NST - 1; ++i) {
      pend >>= 4;   // (each issue lands at the FIFO's tail, NST - 2)
      issue(i);
    }
  }
  constexpr int kAfter = (NST - 2) * 8;   // this thread's DMAs issued after tile t's
  int rd = 0;
  for (int t = 0; t < KT; ++t) {
    // own DMAs of tile t landed (the NST - 2 newer tiles' may still be in flight)
    __builtin_amdgcn_s_waitcnt((kAfter & 15) | ((kAfter >> 4) << 14) | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");
    const unsigned cur = pend & 15u;
    pend >>= 4;
    if constexpr (PRE) {   // BN+ReLU on this thread's own B chunks (the ones it fetched)
      bf16* Bst = reinterpret_cast<bf16*>(smem + rd * 2 * OP_B + OP_B);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if ((cur >> i) & 1u) {
          bf16x8* q = reinterpret_cast<bf16x8*>(Bst + ((wave * 4 + i) * 1024 + lane * 16) / 2);
          const int j = i & 1;
          *q = affine_relu8_reg(*q, ps0[j], ps1[j], pb0[j], pb1[j]);
        }
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // into the stage consumed at t - 1 (every wave passed this barrier after its
    // MFMAs); past the slice's end all out of range, so the issue needs no branch and
    // its address adds can interleave with the MFMAs
    issue(rd == 0 ? NST - 1 : rd - 1);
    mma_stage(rd);
    rd = rd == NST - 1 ? 0 : rd + 1;
  }
  // the out-of-range tail DMAs land before the LDS is released
  __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8));

  float* out = args.part + (long)split * Cout * NT;
#pragma unroll
  for (int b = 0; b < NR; ++b) {
    const int n = n0 + wn * WTN + b * 16 + li;
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * WTM + a * 16 + gq * 4 + i;
        if (m < Cout && n < NT) out[(long)m * NT + n] = acc[a][b][i];
      }
  }
}

// Ring eligibility: 128 x 128 tiles (Cout > 64, >= 128 columns), 32-bit buffer offsets,
// 16-B channel chunks, and the 3-round pixel stepping covers BK = 64 pixels.
bool conv_wgrad_ring_covers(const WgradArgs& a) {
  if (!tune(T_RING_WGRAD)) return false;
  const ConvGeom& g = a.g;
  const long x_elems = (long)g.N * g.H * g.W * g.C;
  const long dy_elems = (long)g.N * g.Ho * g.Wo * g.K;
  const long NT = (long)g.kh * g.kw * g.C;
  return g.K > 64 && NT > 64 && g.C % 8 == 0 && x_elems < (1L << 30) && dy_elems < (1L << 30) &&
         64 / g.Wo + 1 <= 3 * g.Ho;
}

void conv_wgrad_ring(const WgradArgs& a, hipStream_t s) {
  const int NT = a.g.kh * a.g.kw * a.g.C;
  dim3 grid((NT + 127) / 128, (a.g.K + 127) / 128, a.splits);
  const size_t lds = (size_t)2 * 2 * 64 * 128 * sizeof(bf16);
  if (a.pre_scale)
    hipLaunchKernelGGL(conv_wgrad_ring_kernel<true>, grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(conv_wgrad_ring_kernel<false>, grid, dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
