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

#include "bn_fused.h"
#include "common.h"
#include "kernels.h"

namespace dtr {

enum { F_PRE = 1, F_STATS = 2, F_BNB = 4 };

// Epilogue staging: PR rows of the fp32 tile at a time -- the whole tile when
// it fits in 64 KiB (one phase), else one wave-row per phase (128x128 tiles).
template <int BM, int BN, int WM>
struct EpiLayout {
  static constexpr int LDC = BN + 4;              // fp32 staging row stride (floats)
  static constexpr int CPR = BN / 8;              // 8-channel chunks per row
  static constexpr int RPP = 256 / CPR;           // rows per pass
  static constexpr int RED = 2 * RPP * BN + BN;   // floats (two reduction planes + means)
  static constexpr int PHASES = ((BM * LDC + RED) * 4 <= 64 * 1024) ? 1 : WM;
  static constexpr int PR = BM / PHASES;          // rows staged per phase
  static constexpr int TILE = PR * LDC;           // floats
  static constexpr size_t BYTES = (size_t)(TILE + RED) * sizeof(float);
};

template <int BM, int BN, int WM, int WN, int MODE, int FLAGS>
__global__ void __launch_bounds__(256)
conv_gemm_kernel(GemmArgs args) {
  constexpr bool PRE = (FLAGS & F_PRE) != 0;
  constexpr bool STATS = (FLAGS & F_STATS) != 0;
  constexpr bool BNB = (FLAGS & F_BNB) != 0;
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
  bf16* As = reinterpret_cast<bf16*>(smem);                 // [2][BM][BK]
  bf16* Bs = As + 2 * BM * BK;                              // [2][BN][BK]
  float* pre_s = reinterpret_cast<float*>(Bs + 2 * BN * BK); // [2][Cin] (PRE)

  const ConvGeom& g = args.g;
  const int M = args.M, NC = args.Ncol, KD = args.Kdim;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;

  // Input-channel count of the A operand's gather (C for fwd, K for dgrad).
  const int Acin = (MODE == MODE_FWD) ? g.C : g.K;

  if constexpr (PRE) {
    for (int i = tid; i < Acin; i += 256) {
      pre_s[i] = args.pre_scale[i];
      pre_s[Acin + i] = args.pre_shift[i];
    }
  }

  // ---- per-thread loader state (row decomposition is K-invariant) ----
  const int kg = tid & 7;  // fixed 16-B k-group of every chunk this thread stages
  int a_base[A_PER_T], a_h[A_PER_T], a_w[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int q = tid + i * 256;
    const int r = q >> 3;
    const int m = m0 + r;
    a_h[i] = -(1 << 28);  // invalid row marker
    a_w[i] = 0;
    a_base[i] = 0;
    if (q < A_CHUNKS && m < M) {
      if constexpr (MODE == MODE_FWD) {
        const int hw = g.Ho * g.Wo;
        const int n = m / hw, rem = m - n * hw;
        const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
        a_base[i] = n * g.H * g.W;
        a_h[i] = ho * g.stride - g.pad;
        a_w[i] = wo * g.stride - g.pad;
      } else {
        const int hw = g.H * g.W;
        const int n = m / hw, rem = m - n * hw;
        const int h = rem / g.W, w = rem - h * g.W;
        a_base[i] = n * g.Ho * g.Wo;
        a_h[i] = h + g.pad;
        a_w[i] = w + g.pad;
      }
    }
  }

  bf16x8 ra[A_PER_T], rb[B_PER_T];
  const bf16x8 zero8 = {};

  auto load_tile = [&](int t) {
    const int k = t * BK + kg * 8;
    const bool kvalid = k < KD;
    const int tap = kvalid ? k / Acin : 0;
    const int ci = k - tap * Acin;
    const int rr = tap / g.kw, cc = tap - rr * g.kw;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      bf16x8 v = zero8;
      if constexpr (MODE == MODE_FWD) {
        const int hi = a_h[i] + rr, wi = a_w[i] + cc;
        if (kvalid && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
          const long off = ((long)(a_base[i] + hi * g.W + wi)) * g.C + ci;
          v = *reinterpret_cast<const bf16x8*>(args.a + off);
          if constexpr (PRE) v = affine_relu8(v, pre_s + ci, pre_s + Acin + ci);
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
          off = ((long)tap * g.C + (n0 + nrow)) * g.K + ci;    // W[r][c][ci][co]
        }
        v = *reinterpret_cast<const bf16x8*>(args.b + off);
      }
      rb[i] = v;
    }
  };

  auto store_tile = [&](int buf) {
    bf16* A = As + buf * BM * BK;
    bf16* B = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int q = tid + i * 256;
      if (q < A_CHUNKS) {
        const int r = q >> 3;
        *reinterpret_cast<bf16x8*>(A + r * BK + ((kg ^ (r & 7)) << 3)) = ra[i];
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

  f32x4 acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PRE) __syncthreads();
  const int KT = (KD + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < KT; ++t) {
    if (t + 1 < KT) load_tile(t + 1);
    const bf16* A = As + (t & 1) * BM * BK;
    const bf16* B = Bs + (t & 1) * BN * BK;
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
    if (t + 1 < KT) store_tile((t + 1) & 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  // Processed in EL::PHASES phases of EL::PR rows (1 phase unless the tile is 128x128):
  //  (a) the waves owning those rows write their fragments (+bias) to an fp32 LDS tile
  //      (the K loop ended with a barrier: staging buffers/PRE table are dead);
  //  (b) all 256 threads sweep it as 16-byte row vectors (8 channels per lane):
  //      residual / accumulate, ONE bf16 rounding, 16-B store, BN partials;
  //  (c) STATS: per-phase two-pass (mean, M2) folded across phases with Chan's
  //      formula in fixed order; BNB: sums carried in registers.
  using EL = EpiLayout<BM, BN, WM>;
  float* cs = reinterpret_cast<float*>(smem);
  float* red = cs + EL::TILE;
  float* red2 = red + EL::RPP * BN;
  float* mean_s = red + 2 * EL::RPP * BN;
  const int cc = tid % EL::CPR, r0 = tid / EL::CPR;
  const int col0 = n0 + cc * 8;
  const bool colok = col0 < NC;  // NC % 16 == 0 -> a chunk is all-in or all-out
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  float bsc[8], bsh[8], bmu[8], brs[8];
  if constexpr (BNB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsc[j] = colok ? args.bnb_scale[col0 + j] : 0.f;
      bsh[j] = colok ? args.bnb_shift[col0 + j] : 0.f;
      bmu[j] = colok ? args.bnb_mean[col0 + j] : 0.f;
      brs[j] = colok ? args.bnb_rstd[col0 + j] : 0.f;
    }
  }
  float wn_run = 0.f, wmean_run = 0.f, wm2_run = 0.f;  // STATS, thread tid < BN owns column tid

#pragma unroll 1
  for (int ph = 0; ph < EL::PHASES; ++ph) {
    const int prow0 = m0 + ph * EL::PR;
    const int nph = min(EL::PR, M - prow0);   // block-uniform
    if (nph <= 0) break;
    if ((wm * WTM) / EL::PR == ph) {
      const int rbase = wm * WTM - ph * EL::PR;
#pragma unroll
      for (int b = 0; b < NR; ++b) {
        const int cl = wn * WTN + b * 16 + fr;
        const int col = n0 + cl;
        const float bias = (args.bias != nullptr && col < args.nbias) ? args.bias[col] : 0.f;
#pragma unroll
        for (int a = 0; a < MR; ++a)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            cs[(rbase + a * 16 + fq * 4 + i) * EL::LDC + cl] = acc[a][b][i] + bias;
      }
    }
    __syncthreads();
    float p1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) p1[j] = 0.f;
    for (int r = r0; r < nph; r += EL::RPP) {
      if (!colok) break;
      const int row = prow0 + r;
      float* cp = cs + r * EL::LDC + cc * 8;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(cp);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(cp + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const long o = (long)row * NC + col0;
      if (args.residual) {
        const bf16x8 rv = *reinterpret_cast<const bf16x8*>(args.residual + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += (float)rv[j];
      }
      if (args.out_f32) {
        float* op = args.out_f32 + o;
        if (args.accumulate) {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(op);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(op + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] += a0[j];
            v[4 + j] += a1[j];
          }
        }
        *reinterpret_cast<f32x4*>(op) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(op + 4) = f32x4{v[4], v[5], v[6], v[7]};
      } else {
        if (args.accumulate) {
          const bf16x8 av = *reinterpret_cast<const bf16x8*>(args.out + o);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += (float)av[j];
        }
        bf16x8 ob;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ob[j] = (bf16)v[j];
          v[j] = (float)ob[j];
        }
        *reinterpret_cast<bf16x8*>(args.out + o) = ob;
      }
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) p1[j] += v[j];
        *reinterpret_cast<f32x4*>(cp) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(cp + 4) = f32x4{v[4], v[5], v[6], v[7]};
      }
      if constexpr (BNB) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(args.bnb_x + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = (float)xv[j];
          const float gg = (xf * bsc[j] + bsh[j] > 0.f) ? v[j] : 0.f;
          s1[j] += gg;
          s2[j] += gg * (xf - bmu[j]) * brs[j];
        }
      }
    }
    if constexpr (STATS) {
      // phase mean
#pragma unroll
      for (int j = 0; j < 8; ++j) red[r0 * BN + cc * 8 + j] = p1[j];
      __syncthreads();
      if (tid < BN) {
        float t = 0.f;
        for (int k = 0; k < EL::RPP; ++k) t += red[k * BN + tid];
        mean_s[tid] = t / (float)nph;
      }
      __syncthreads();
      float mu[8], q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mu[j] = mean_s[cc * 8 + j];
        q[j] = 0.f;
      }
      for (int r = r0; r < nph; r += EL::RPP) {
        if (!colok) break;
        const float* cp = cs + r * EL::LDC + cc * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = cp[j] - mu[j];
          q[j] += d * d;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) red2[r0 * BN + cc * 8 + j] = q[j];
      __syncthreads();
      if (tid < BN) {
        float m2 = 0.f;
        for (int k = 0; k < EL::RPP; ++k) m2 += red2[k * BN + tid];
        const float nb = (float)nph, mb = mean_s[tid];
        const float n = wn_run + nb;
        const float d = mb - wmean_run;
        wmean_run += d * nb / n;
        wm2_run += m2 + d * d * wn_run * nb / n;
        wn_run = n;
      }
    }
    __syncthreads();  // the next phase overwrites the staging tile
  }

  if constexpr (STATS) {
    if (tid < BN && n0 + tid < NC) {
      float* tile_out = args.stat_part + (long)blockIdx.x * 2 * NC;
      if (args.fin.counters != nullptr) {   // handed to the last arriver: write-through (sc1)
        publish_f32(tile_out + n0 + tid, wmean_run);
        publish_f32(tile_out + NC + n0 + tid, wm2_run);
      } else {
        tile_out[n0 + tid] = wmean_run;     // tile mean
        tile_out[NC + n0 + tid] = wm2_run;  // tile M2
      }
    }
    const BnFwdFin& F = args.fin;
    if (F.counters != nullptr &&
        last_arriver(F.counters + blockIdx.y, gridDim.x, reinterpret_cast<int*>(mean_s))) {
      // Chan-combine all tiles of columns [n0, n0+BN): thread = (column, tile group)
      constexpr int G = 256 / BN;
      const int c = tid % BN, gq2 = tid / BN;
      const int col = n0 + c;
      float n = 0.f, mu = 0.f, m2 = 0.f;
      const int T = gridDim.x;
      if (col < NC) {   // host guarantees T <= G * FIN_UNROLL: all loads in flight at once
        float mbv[FIN_UNROLL], qbv[FIN_UNROLL];
#pragma unroll
        for (int u = 0; u < FIN_UNROLL; ++u) {
          const int t = gq2 + u * G;
          mbv[u] = t < T ? args.stat_part[(long)t * 2 * NC + col] : 0.f;
          qbv[u] = t < T ? args.stat_part[(long)t * 2 * NC + NC + col] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < FIN_UNROLL; ++u) {
          const int t = gq2 + u * G;
          if (t < T) {
            const float nb = (float)min(BM, M - t * BM);
            const float nn = n + nb, d = mbv[u] - mu;
            mu += d * nb / nn;
            m2 += qbv[u] + d * d * n * nb / nn;
            n = nn;
          }
        }
      }
      red[gq2 * BN + c] = n;
      red2[gq2 * BN + c] = mu;
      cs[gq2 * BN + c] = m2;                // staging tile is free now
      __syncthreads();
      if (gq2 == 0 && col < NC) {
        float fn_ = red[c], fmu = red2[c], fm2 = cs[c];
        for (int k = 1; k < G; ++k) {
          const float nb = red[k * BN + c], mb = red2[k * BN + c], qb = cs[k * BN + c];
          const float nn = fn_ + nb;
          if (nn > 0.f) {
            const float d = mb - fmu;
            fmu += d * nb / nn;
            fm2 += qb + d * d * fn_ * nb / nn;
            fn_ = nn;
          }
        }
        const float var = fm2 / fn_;
        const float rs = rsqrtf(var + F.eps);
        const float sc = F.gamma[col] * rs;
        F.mean[col] = fmu;
        F.rstd[col] = rs;
        F.scale[col] = sc;
        F.shift[col] = F.beta[col] - fmu * sc;
        if (F.update_moving) {
          const float uvar = fn_ > 1.f ? fm2 / (fn_ - 1.f) : fm2;
          F.mmean[col] -= (1.f - F.momentum) * (F.mmean[col] - fmu);
          F.mvar[col] -= (1.f - F.momentum) * (F.mvar[col] - uvar);
        }
      }
      reset_counter(F.counters + blockIdx.y);
    }
  }
  if constexpr (BNB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[r0 * BN + cc * 8 + j] = s1[j];
      red2[r0 * BN + cc * 8 + j] = s2[j];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < NC) {
      float t1 = 0.f, t2 = 0.f;
      for (int k = 0; k < EL::RPP; ++k) {
        t1 += red[k * BN + tid];
        t2 += red2[k * BN + tid];
      }
      float* tile_out = args.bnb_part + (long)blockIdx.x * 2 * NC;
      if (args.bfin.counters != nullptr) {
        publish_f32(tile_out + n0 + tid, t1);
        publish_f32(tile_out + NC + n0 + tid, t2);
      } else {
        tile_out[n0 + tid] = t1;        // sum g
        tile_out[NC + n0 + tid] = t2;   // sum g * xhat
      }
    }
    const BnBwdFin& F = args.bfin;
    if (F.counters != nullptr &&
        last_arriver(F.counters + blockIdx.y, gridDim.x, reinterpret_cast<int*>(mean_s))) {
      constexpr int G = 256 / BN;
      const int c = tid % BN, gq2 = tid / BN;
      const int col = n0 + c;
      float a1 = 0.f, a2 = 0.f;
      const int T = gridDim.x;
      if (col < NC) {
        float v1[FIN_UNROLL], v2[FIN_UNROLL];
#pragma unroll
        for (int u = 0; u < FIN_UNROLL; ++u) {
          const int t = gq2 + u * G;
          v1[u] = t < T ? args.bnb_part[(long)t * 2 * NC + col] : 0.f;
          v2[u] = t < T ? args.bnb_part[(long)t * 2 * NC + NC + col] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < FIN_UNROLL; ++u) {
          a1 += v1[u];
          a2 += v2[u];
        }
      }
      red[gq2 * BN + c] = a1;
      red2[gq2 * BN + c] = a2;
      __syncthreads();
      if (gq2 == 0 && col < NC) {
        float sg = 0.f, sgx = 0.f;
        for (int k = 0; k < G; ++k) {
          sg += red[k * BN + c];
          sgx += red2[k * BN + c];
        }
        F.dbeta[col] = sg;
        F.dgamma[col] = sgx;
        const float a = F.gamma[col] * F.rstd[col];
        F.coef[col] = a;
        F.coef[NC + col] = a * sg / (float)M;
        F.coef[2 * NC + col] = a * sgx / (float)M;
      }
      reset_counter(F.counters + blockIdx.y);
    }
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int MODE, int FLAGS>
static void launch_cfg(const GemmArgs& a, hipStream_t s) {
  const int Acin = (MODE == MODE_FWD) ? a.g.C : a.g.K;
  size_t lds = (size_t)2 * (BM + BN) * 64 * sizeof(bf16);
  if (FLAGS & F_PRE) lds += (size_t)2 * Acin * sizeof(float);
  lds = std::max(lds, EpiLayout<BM, BN, WM>::BYTES);
  lds = (lds + 15) & ~(size_t)15;
  dim3 grid((a.M + BM - 1) / BM, (a.Ncol + BN - 1) / BN);
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, MODE, FLAGS>), grid, dim3(256), lds, s, a);
  DTR_CHECK_LAUNCH();
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

// Tile selection by output width; BM shrinks for small M so the grid still
// covers the 256 CUs.  Shared by the launcher and by the host (the BN-stat
// partial buffer has one row per M tile).
int conv_gemm_bm(int M, int nc) {
  const long m = M;
  if (nc <= 16) return m >= 256L * 512 ? 256 : 64;
  if (nc <= 32) return m >= 128L * 512 ? 128 : 64;
  if (nc <= 64) return m >= 128L * 256 ? 128 : 64;
  return (m >= 128L * 128 && nc % 128 == 0) ? 128 : 64;
}

template <int MODE>
static void launch_mode(const GemmArgs& a, hipStream_t s) {
  const int nc = a.Ncol;
  const int bm = conv_gemm_bm(a.M, nc);
  if (nc <= 16) {
    if (bm == 256) launch_flags<256, 16, 4, 1, MODE>(a, s);
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

void conv_gemm(const GemmArgs& a, int mode, hipStream_t s) {
  if (mode == MODE_FWD) launch_mode<MODE_FWD>(a, s);
  else launch_mode<MODE_DGRAD>(a, s);
}

}  // namespace dtr
