// 8-wave LDS-DMA ring implicit-GEMM convolution for the deep-K ImageNet layers (the
// bottlenecks' 3x3 convs at 28x28 / 14x14 / 7x7 and the stride-2 3x3 transitions:
// K >= 1024, a stride-2 dgrad by its largest parity class), forward and data gradient, on gfx950.
//
// Same GEMM, gather and epilogue as conv_ring.hip (reference: the Conv2D /
// Conv2DBackpropInput of conv2d_fixed_padding, resnet_model_official.py:80-91, inside the
// bottleneck block :153-175), but shaped for the compute-bound layers, where the 4-wave
// 128x128 ring measured 340-410 TF/s (profiles/imagenet_resnet50_roofline.md): with two
// 64 KiB workgroups per CU and a 2-stage ring, only ONE K tile (512 MFMA cycles per wave)
// is in flight behind the MFMAs, so every tile waits on a DMA round trip.  Here:
//   * 512 threads (8 waves, 2 per SIMD), one workgroup per CU, a 256 x 128 tile: each
//     wave a 64 x 64 sub-tile (4 x 4 16x16x32 MFMA fragments), so each 64-deep K tile is
//     32 MFMAs per wave, 1024 MFMA cycles per SIMD;
//   * a 3-stage ring (3 x 48 KiB): tile t+2 is issued while tile t is multiplied, two
//     tiles (~2000 SIMD cycles) cover the DMA latency;
//   * counted waits: `s_waitcnt vmcnt(6)` (this wave's 6 DMAs of tile t+1 stay in flight)
//     then a raw s_barrier -- never __syncthreads() in the loop, whose vmcnt(0) would
//     drain the ring (cdna_hip_programming.md "Pipelining across barriers");
//   * one barrier per K tile: the stage written at tile t (t+2 mod 3) was last read at
//     tile t-1, before every wave passed this tile's barrier.
// MFMA shape: 16x16x32 bf16, which on random operands delivers ~1.15x the FLOP/s of
// 32x32x16 at equal cycles (MI355X_MICROARCH.md, MFMA shape vs clock) and keeps the
// shared epilogue's fragment layout.
//
// Epilogue: the two 128-row halves of the tile run the shared 256-thread epilogue side
// by side (waves 0-3 and 4-7, conv_epilogue.h ep_tid / SYNC_ALL), each as the 128 x 128
// tile 2 tm + h; split-K slices combine the whole 256 x 128 tile behind ONE ticket so
// both halves take the same last-arriver decision.
#include <algorithm>
#include <stdexcept>

#include "conv_epilogue.h"

namespace dtr {

namespace {

typedef __attribute__((address_space(3))) void lds_void8;

constexpr int R8_BM = 256, R8_BN = 128, R8_BK = 64, R8_NSTAGE = 3;
constexpr int R8_A_BYTES = R8_BM * R8_BK * 2;                 // 32 KiB
constexpr int R8_STAGE = (R8_BM + R8_BN) * R8_BK * 2;         // 48 KiB
constexpr int R8_OOB = 0x7fff0000;
using R8Epi = EpiLayout<128, 128, 2>;
constexpr size_t R8_EPI_HALF = (R8Epi::BYTES + 255) & ~(size_t)255;
constexpr size_t R8_LDS = (size_t)R8_NSTAGE * R8_STAGE > 2 * R8_EPI_HALF
                              ? (size_t)R8_NSTAGE * R8_STAGE : 2 * R8_EPI_HALF;
static_assert(R8_LDS <= 160 * 1024, "LDS");

template <int n>
__device__ __forceinline__ void r8_wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}

// split-K: slice z of the 256 x 128 tile publishes its fp32 fragments (write-through,
// thread-native order) and takes ONE ticket; the last slice sums all slices in slice
// order (bitwise independent of arrival order) and alone returns true.
__device__ __forceinline__ bool r8_splitk_combine(const GemmArgs& args, f32x4 (&acc)[4][4],
                                                  char* smem, int tile, int z) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int S = args.ksplit;
  const long slab = 16L * 512 * 4;   // floats per slice tile
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + (long)tile * S * slab, 0,
                                                    0x7fffffff, 0x00020000);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4_t, acc[a][b]), rs,
          (int)((((long)z * slab) + ((long)(a * 4 + b) * 512 + tid) * 4) * 4), 0, 16);
  int* flag = reinterpret_cast<int*>(smem);
  if (!last_arriver(args.sk_cnt + tile, (unsigned)S, flag)) return false;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int zz = 0; zz < S; ++zz) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        acc[a][b] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
            rs, (int)((((long)zz * slab) + ((long)(a * 4 + b) * 512 + tid) * 4) * 4), 0, 16));
  }
  reset_counter(args.sk_cnt + tile);
  __syncthreads();   // the flag word's LDS is the epilogue's
  return true;
}

}  // namespace

template <int MODE, int FLAGS>
__global__ void __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_ring8_kernel(GemmArgs args) {
  constexpr int BM = R8_BM, BN = R8_BN, BK = R8_BK;
  constexpr int WN = 2, MR = 4, NR = 4;   // 8 waves as 4 (M) x 2 (N), 64 x 64 each
  constexpr bool BNB = (FLAGS & F_BNB) != 0;
  static_assert((FLAGS & (F_PRE | F_ABWD)) == 0, "no A-operand prologue on the ring");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ConvGeom& g = args.g;
  // diagnostics (set_ring8_probe): workgroup (0, 0, 0)'s lane 0 stamps the wall clock at
  // start [0], after the prologue [1], after each K tile's MFMAs [2 + t] (t < 48), after
  // the loop [50], after the split-K combine [51] and at the end [52]
  long long* const kp = (args.kprobe != nullptr && blockIdx.x == 0 && blockIdx.y == 0 &&
                         blockIdx.z == 0 && threadIdx.x == 0) ? args.kprobe : nullptr;
  if (kp) kp[0] = wall_clock64();
  // XCD-aware order (T1): consecutive tiles of one column block land on one XCD (whose
  // L2 then holds its B columns and neighbouring A rows).  Bijective for any count.
  const int nx = gridDim.x, ny = gridDim.y, nwg = nx * ny;
  const int orig = blockIdx.y * nx + blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tm = lin % nx, tn = lin / nx, lz = blockIdx.z;
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
  if (MODE == MODE_DGRAD && args.par && tm * BM >= M) return;   // (block-uniform)
  const bool par = MODE == MODE_DGRAD && args.par;
  const int taw = par ? (g.kw - par_pw + 1) >> 1 : g.kw;
  const int Acin = MODE == MODE_FWD ? g.C : g.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-lane gather state: A rows (wave * 4 + i) * 8 + lane / 8, B rows
  //      (wave * 2 + i) * 8 + lane / 8; 16-B chunk (lane % 8) ^ (row % 8) (source swizzle)
  const int lr = lane >> 3;
  const int kg = (lane & 7) ^ lr;
  int a_off[4];
  unsigned a_mask[4];
  int b_off[2];
  const int ntap = (par ? ((g.kh - par_ph + 1) >> 1) : g.kh) * taw;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (wave * 4 + i) * 8 + lr;
    unsigned mask = 0u;
    long pix = 0;
    if (m < M) {
      if constexpr (MODE == MODE_FWD) {
        const int hw = g.Ho * g.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
        const int h0 = ho * g.stride - g.pad, w0 = wo * g.stride - g.pad;
        pix = (long)n * g.H * g.W + (long)h0 * g.W + w0;
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
        int hp0, wp0;
        if (par) {
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
  for (int i = 0; i < 2; ++i) {
    const int nrow = n0 + (wave * 2 + i) * 8 + lr;
    if constexpr (MODE == MODE_FWD) b_off[i] = nrow < NC ? (nrow * KD + kg * 8) * 2 : R8_OOB;
    else b_off[i] = nrow < NC ? (nrow * g.K + kg * 8) * 2 : R8_OOB;
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
  const int cpt = Acin / BK;
  int it_tl = t_beg / cpt;
  int it_c = (t_beg - it_tl * cpt) * BK;
  int it_ta = it_tl / taw, it_tb = it_tl - it_ta * taw;
  // next tile -> stage: 4 A + 2 B DMAs per wave, in two halves (part 0: A 0-1 + B 0,
  // part 1: A 2-3 + B 1, then the tap walk advances) so the loop can put each half in
  // front of one k-step's MFMAs instead of issuing all six in one burst
  auto issue_part = [&](int stage, int part) {
    const int a_pix = MODE == MODE_FWD ? it_ta * g.W + it_tb : -(it_ta * g.Wo + it_tb);
    const int sa = (a_pix * Acin + it_c) * 2;
    int sb;
    if constexpr (MODE == MODE_FWD) {
      sb = (it_tl * Acin + it_c) * 2;
    } else {
      const int rr = par ? par_ph + 2 * it_ta : it_ta, cc = par ? par_pw + 2 * it_tb : it_tb;
      sb = ((rr * g.kw + cc) * g.C * g.K + it_c) * 2;
    }
    char* st = smem + stage * R8_STAGE;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * part + j;
      const bool ok = (a_mask[i] >> it_tl) & 1u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_a, (lds_void8*)(st + (wave * 4 + i) * 1024), 16, ok ? a_off[i] + sa : R8_OOB, 0, 0,
          0);
    }
    char* const stb = st + R8_A_BYTES;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs_b, (lds_void8*)(stb + (wave * 2 + part) * 1024), 16, b_off[part] + sb, 0, 0, 0);
    if (part == 0) return;
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
  auto mma_kstep = [&](int stage, int ks) {
    const bf16* A = reinterpret_cast<const bf16*>(smem + stage * R8_STAGE);
    const bf16* B = reinterpret_cast<const bf16*>(smem + stage * R8_STAGE + R8_A_BYTES);
    {
      const int ch = ks * 4 + fq;
      bf16x8 af[MR], bfr[NR];
#pragma unroll
      for (int a = 0; a < MR; ++a) {
        const int r = wm * 64 + a * 16 + fr;
        af[a] = *reinterpret_cast<const bf16x8*>(A + r * BK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int r = wn * 64 + b * 16 + fr;
        bfr[b] = *reinterpret_cast<const bf16x8*>(B + r * BK + ((ch ^ (r & 7)) << 3));
      }
#pragma unroll
      for (int a = 0; a < MR; ++a)
#pragma unroll
        for (int b = 0; b < NR; ++b) acc[a][b] = mfma16(af[a], bfr[b], acc[a][b]);
    }
  };

  // dgrad + BN-backward sums: this half's BN-input rows / coefficients, loaded now
  const int half = wave >> 2;
  using EP = EpiPre<128, 128, 2, true>;
  EP epre;
  if constexpr (BNB) epi_prefetch<128, 128, 2, FLAGS, true>(args, m0 + half * 128, n0, epre);

  // ---- 3-stage ring: tiles t+1 and t+2 in flight during the MFMAs of tile t ----
  const int nt = t_end - t_beg;
  if (kp) kp[1] = wall_clock64();
  if (nt > 0) {
    issue_part(0, 0);
    issue_part(0, 1);
  }
  if (nt > 1) {
    issue_part(1, 0);
    issue_part(1, 1);
  }
  int rd = 0;
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) r8_wait_vm<6>();   // this wave's tile-t DMAs have landed
    else r8_wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();      // ... every wave's; stage (t+2) % 3 is free
    asm volatile("" ::: "memory");
    const bool more = t + 2 < nt;
    const int ws = rd == 0 ? 2 : rd - 1;
    if (more) issue_part(ws, 0);
    mma_kstep(rd, 0);
    if (more) issue_part(ws, 1);
    mma_kstep(rd, 1);
    rd = rd == 2 ? 0 : rd + 1;
    if (kp && t < 48) kp[2 + t] = wall_clock64();
  }
  __syncthreads();   // every wave's MFMA reads are done: the epilogue reuses the LDS
  if (kp) kp[50] = wall_clock64();

  if (sk_n > 1 && !r8_splitk_combine(args, acc, smem, tm * ny + tn, lz)) return;
  if (kp) kp[51] = wall_clock64();
  char* hs = smem + half * R8_EPI_HALF;
  if constexpr (BNB)
    conv_epilogue<128, 128, 2, 2, FLAGS, true, true>(args, acc, hs, m0 + half * 128, n0, &epre,
                                                     2 * tm + half, tn);
  else
    conv_epilogue<128, 128, 2, 2, FLAGS, false, true>(args, acc, hs, m0 + half * 128, n0,
                                                      nullptr, 2 * tm + half, tn);
  if (kp) kp[52] = wall_clock64();
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Deep-K ring convs: 3x3 with K >= 1024 (>= 16 K tiles; a stride-2 dgrad's largest
// parity class counts), 128-column tiles, and
// the statistics / BN-backward sums in accumulator mode (no per-tile partial rows, no
// last-arriver finalize: the two epilogue halves must pass the same barriers).
bool conv_ring8_covers(const GemmArgs& a, int mode) {
  if (!tune(T_RING8) || !conv_ring_covers(a, mode)) return false;
  if (a.g.kh * a.g.kw == 1 || a.Kdim < 1024 || a.Ncol % 128 != 0 ||
      conv_gemm_bn(a.M, a.Ncol) != 128)
    return false;
  if (a.fin.counters != nullptr || a.bfin.counters != nullptr) return false;
  if (a.stat_part != nullptr && a.stat_acc == nullptr) return false;
  if (a.bnb_part != nullptr && a.bnb_acc == nullptr) return false;
  if (a.out_f32 != nullptr || a.probe != nullptr) return false;
  return true;
}

size_t conv_ring8_lds() { return R8_LDS; }

static long long* g_r8_probe = nullptr;
void set_ring8_probe(long long* p) { g_r8_probe = p; }

template <int MODE, int FLAGS>
static void r8_launch(const GemmArgs& a0, dim3 grid, hipStream_t s) {
  GemmArgs a = a0;
  a.kprobe = g_r8_probe;
  hipLaunchKernelGGL((conv_ring8_kernel<MODE, FLAGS>), grid, dim3(512), R8_LDS, s, a);
  DTR_CHECK_LAUNCH();
}

void conv_ring8(const GemmArgs& a, int mode, int flags, dim3 grid, hipStream_t s) {
  if (mode == MODE_FWD) {
    if (flags & F_STATS) r8_launch<MODE_FWD, F_STATS>(a, grid, s);
    else r8_launch<MODE_FWD, 0>(a, grid, s);
  } else {
    if (flags & F_BNB) r8_launch<MODE_DGRAD, F_BNB>(a, grid, s);
    else r8_launch<MODE_DGRAD, 0>(a, grid, s);
  }
}

}  // namespace dtr
