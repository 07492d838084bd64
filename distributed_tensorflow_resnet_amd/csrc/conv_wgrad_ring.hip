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

}  // namespace

template <bool PRE>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(2, 2)))
conv_wgrad_ring_kernel(WgradArgs args) {
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
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.x), 0,
                                                      (int)(x_elems * 2), 0x00020000);
  const auto rs_dy = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(args.dy), 0,
                                                       (int)(dy_elems * 2), 0x00020000);

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
  // pixel of each of the lane's 4 rows, stepped by BK per issued tile
  const int HoWo = g.Ho * g.Wo;
  const int d_ho = BK / g.Wo, d_wo = BK - d_ho * g.Wo;
  int px_img[4], px_ho[4], px_wo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = p_begin + (wave * 4 + i) * 4 + lr;
    px_img[i] = p / HoWo;
    const int rem = p - px_img[i] * HoWo;
    px_ho[i] = rem / g.Wo;
    px_wo[i] = rem - px_ho[i] * g.Wo;
  }
  unsigned pend = 0u;   // PRE: which of this lane's 4 B chunks of the pending tile are real
  int it_pbase = p_begin;

  auto issue = [&](int stage) {   // K tile at it_pbase -> stage (4 A + 4 B DMAs per wave)
    char* st = smem + stage * 2 * OP_B;
    unsigned msk = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (wave * 4 + i) * 4 + lr;
      const int p = it_pbase + row;
      const int j = i & 1;
      const bool pok = p < p_end;
      const int aoff = (pok && a_col[j] >= 0) ? (p * Cout + a_col[j]) * 2 : kWrOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_dy, (lds_void*)(st + (wave * 4 + i) * 1024), 16, aoff, 0, 0, 0);
      const int hi = px_ho[i] * g.stride - g.pad + b_r[j];
      const int wi = px_wo[i] * g.stride - g.pad + b_c[j];
      const bool ok = pok && b_ok[j] && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const int boff = ok ? (((px_img[i] * g.H + hi) * g.W + wi) * Cin + b_ci[j]) * 2 : kWrOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_x, (lds_void*)(st + OP_B + (wave * 4 + i) * 1024), 16, boff, 0, 0, 0);
      msk |= ok ? (1u << i) : 0u;
      // advance this row's pixel by BK for the next tile (host: BK / Wo + 1 <= 3 Ho)
      px_wo[i] += d_wo;
      px_ho[i] += d_ho;
      const bool wrap = px_wo[i] >= g.Wo;
      px_wo[i] -= wrap ? g.Wo : 0;
      px_ho[i] += wrap ? 1 : 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const bool nxt = px_ho[i] >= g.Ho;
        px_ho[i] -= nxt ? g.Ho : 0;
        px_img[i] += nxt ? 1 : 0;
      }
    }
    pend = msk;
    it_pbase += BK;
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

  if (KT > 0) issue(0);
  int rd = 0;
  for (int t = 0; t < KT; ++t) {
    __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8));   // vmcnt(0): own DMAs landed
    asm volatile("" ::: "memory");
    if constexpr (PRE) {   // BN+ReLU on this thread's own B chunks (the ones it fetched)
      bf16* Bst = reinterpret_cast<bf16*>(smem + rd * 2 * OP_B + OP_B);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if ((pend >> i) & 1u) {
          bf16x8* q = reinterpret_cast<bf16x8*>(Bst + ((wave * 4 + i) * 1024 + lane * 16) / 2);
          const int j = i & 1;
          *q = affine_relu8_reg(*q, ps0[j], ps1[j], pb0[j], pb1[j]);
        }
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < KT) issue(rd ^ 1);
    mma_stage(rd);
    rd ^= 1;
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
