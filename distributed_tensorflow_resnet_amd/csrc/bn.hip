// Training-mode BatchNorm + ReLU for NHWC bf16 activations (replaces TF's
// FusedBatchNorm / FusedBatchNormGrad / Relu / ReluGrad / AssignSub, SURVEY §2.5;
// semantics of `batch_norm_relu`, resnet_model_official.py:41-50: decay 0.997,
// eps 1e-5, moving variance fed with the Bessel-corrected batch variance).
//
// Forward statistics come as per-tile Welford partials (mean, M2) -- either from
// the producing convolution's epilogue (conv_gemm STATS) or from bn_stats below
// -- and are combined deterministically with Chan's parallel formula.  The
// normalisation itself is never a separate pass: consumers apply
// relu(x*scale+shift) while staging their operands.
//
// Backward: g = dy * [x*scale+shift > 0];  dbeta = sum g;  dgamma = sum g*xhat;
//   dx = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat))   (+ residual gradient).
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "bn_fused.h"

namespace dtr {

struct Welford {
  float n, mean, m2;
};

__device__ __forceinline__ Welford wcombine(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (n <= 0.f) return a;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  Welford r;
  r.n = n;
  r.mean = a.mean + d * fb;
  r.m2 = a.m2 + b.m2 + d * d * a.n * fb;
  return r;
}

// Finalize launches sit on the critical path between two convolutions (one per
// BatchNorm whose consumer cannot combine the partials itself), so they are
// built for latency: per-channel parameters loaded up front, the partials in
// ONE round of loads, division-free combines, bitwise-deterministic orders.
constexpr int FIN_BATCH = 16;

// Per-channel variant: one 256-thread block per channel; thread t holds tiles t + 256u
// (u < FIN_BATCH, loads issued together; more tiles re-read in further rounds).
// Two division-free block sums (Chan about the global mean): N and sum n*mean ->
// mean; then sum M2 + n (mean_i - mean)^2.  The per-channel parameters are loaded
// up front so their latency hides under the partial loads.
__device__ __forceinline__ float block_sum4(float v, float* red, int slot) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[slot * 4 + (threadIdx.x >> 6)] = v;
  __syncthreads();
  return (red[slot * 4] + red[slot * 4 + 1]) + (red[slot * 4 + 2] + red[slot * 4 + 3]);
}

__global__ void __launch_bounds__(256)
bn_finalize_chan_kernel(const float* __restrict__ part, int tiles, int tile_rows, int M, int C,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    float* moving_mean, float* moving_var, float momentum, float eps,
                    int update_moving, float* mean_out, float* rstd_out, float* scale_out,
                    float* shift_out) {
  __shared__ float red[12];
  const int c = blockIdx.x, tid = threadIdx.x;
  float g = 0.f, bt = 0.f, mm = 0.f, mvv = 0.f;
  if (tid == 0) {
    g = gamma[c];
    bt = beta[c];
    if (update_moving) {
      mm = moving_mean[c];
      mvv = moving_var[c];
    }
  }
  float mv[FIN_BATCH], qv[FIN_BATCH], nv[FIN_BATCH];
#pragma unroll
  for (int u = 0; u < FIN_BATCH; ++u) {
    const int t = tid + u * 256;
    const bool ok = t < tiles;
    mv[u] = ok ? part[(long)t * 2 * C + c] : 0.f;
    qv[u] = ok ? part[(long)t * 2 * C + C + c] : 0.f;
    nv[u] = ok ? (float)min(tile_rows, M - t * tile_rows) : 0.f;
  }
  float n = 0.f, sx = 0.f;
#pragma unroll
  for (int u = 0; u < FIN_BATCH; ++u) {
    n += nv[u];
    sx += nv[u] * mv[u];
  }
  for (int t = tid + FIN_BATCH * 256; t < tiles; t += 256) {   // beyond one round
    const float nt = (float)min(tile_rows, M - t * tile_rows);
    n += nt;
    sx += nt * part[(long)t * 2 * C + c];
  }
  const float N = block_sum4(n, red, 0);
  const float mean = block_sum4(sx, red, 1) / N;
  float m2 = 0.f;
#pragma unroll
  for (int u = 0; u < FIN_BATCH; ++u) {
    const float d = mv[u] - mean;
    m2 += qv[u] + nv[u] * d * d;
  }
  for (int t = tid + FIN_BATCH * 256; t < tiles; t += 256) {
    const float nt = (float)min(tile_rows, M - t * tile_rows);
    const float d = part[(long)t * 2 * C + c] - mean;
    m2 += part[(long)t * 2 * C + C + c] + nt * d * d;
  }
  m2 = block_sum4(m2, red, 2);
  if (tid == 0) {
    const float rstd = rsqrtf(m2 / N + eps);
    const float sc = g * rstd;
    mean_out[c] = mean;
    rstd_out[c] = rstd;
    scale_out[c] = sc;
    shift_out[c] = bt - mean * sc;
    if (update_moving) {
      const float uvar = N > 1.f ? m2 / (N - 1.f) : m2;
      moving_mean[c] = mm - (1.f - momentum) * (mm - mean);
      moving_var[c] = mvv - (1.f - momentum) * (mvv - uvar);
    }
  }
}

__global__ void __launch_bounds__(256)
bn_bwd_finalize_chan_kernel(const float* __restrict__ part, int tiles, int M, int C,
                        const float* __restrict__ gamma, const float* __restrict__ rstd,
                        float* dgamma, float* dbeta, float* coef) {
  __shared__ float s0[4], s1[4];
  const int c = blockIdx.x, tid = threadIdx.x;
  const float a = tid == 0 ? gamma[c] * rstd[c] : 0.f;   // issued ahead of the partials
  float sg = 0.f, sgx = 0.f;
  for (int base = tid; base < tiles; base += FIN_BATCH * 256) {
    float v1[FIN_BATCH], v2[FIN_BATCH];
#pragma unroll
    for (int u = 0; u < FIN_BATCH; ++u) {
      const int t = base + u * 256;
      v1[u] = t < tiles ? part[(long)t * 2 * C + c] : 0.f;
      v2[u] = t < tiles ? part[(long)t * 2 * C + C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < FIN_BATCH; ++u) {
      sg += v1[u];
      sgx += v2[u];
    }
  }
  sg = wave_sum(sg);
  sgx = wave_sum(sgx);
  const int wave = tid >> 6;
  if ((tid & 63) == 0) {
    s0[wave] = sg;
    s1[wave] = sgx;
  }
  __syncthreads();
  if (tid == 0) {
    const float a0 = (s0[0] + s0[1]) + (s0[2] + s0[3]);
    const float a1 = (s1[0] + s1[1]) + (s1[2] + s1[3]);
    dbeta[c] = a0;
    dgamma[c] = a1;
    coef[c] = a;
    coef[C + c] = a * a0 / (float)M;
    coef[2 * C + c] = a * a1 / (float)M;
  }
}

// Variant choice (measured, scripts/fin_bench.py): the per-channel one-round
// kernels win once there are many partials per channel; the LDS-tree kernels
// below win for few partials or many channels.  tune fin_v = 0 / 2 forces one.
void set_fin_version(int v) { tune_set(T_FIN_V, v); }
static bool fin_use_v2(int tiles, int C, bool bwd) {
  const int v = (int)tune(T_FIN_V);
  if (v != 1) return v == 2;
  return C <= 512 && tiles >= (bwd ? 256 : 1024);
}

// One block per channel: thread t folds tiles t, t+256, ... then a fixed-shape
// LDS tree -- bitwise deterministic.
__global__ void __launch_bounds__(256)
bn_finalize_kernel(const float* __restrict__ part, int tiles, int tile_rows, int M, int C,
                   const float* __restrict__ gamma, const float* __restrict__ beta,
                   float* moving_mean, float* moving_var, float momentum, float eps,
                   int update_moving, float* mean_out, float* rstd_out, float* scale_out,
                   float* shift_out) {
  __shared__ float sn[256], sm[256], s2[256];
  const int c = blockIdx.x, tid = threadIdx.x;
  float g = 0.f, bt = 0.f, mm = 0.f, mvv = 0.f;   // issued ahead of the partials
  if (tid == 0) {
    g = gamma[c];
    bt = beta[c];
    if (update_moving) {
      mm = moving_mean[c];
      mvv = moving_var[c];
    }
  }
  Welford w{0.f, 0.f, 0.f};
  for (int t = tid; t < tiles; t += 256) {
    Welford b;
    b.n = (float)min(tile_rows, M - t * tile_rows);
    b.mean = part[(long)t * 2 * C + c];
    b.m2 = part[(long)t * 2 * C + C + c];
    w = wcombine(w, b);
  }
  sn[tid] = w.n;
  sm[tid] = w.mean;
  s2[tid] = w.m2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      Welford a{sn[tid], sm[tid], s2[tid]}, b{sn[tid + o], sm[tid + o], s2[tid + o]};
      a = wcombine(a, b);
      sn[tid] = a.n;
      sm[tid] = a.mean;
      s2[tid] = a.m2;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float n = sn[0], mean = sm[0], m2 = s2[0];
    const float var = m2 / n;
    const float rstd = rsqrtf(var + eps);
    const float sc = g * rstd;
    mean_out[c] = mean;
    rstd_out[c] = rstd;
    scale_out[c] = sc;
    shift_out[c] = bt - mean * sc;
    if (update_moving) {
      const float uvar = n > 1.f ? m2 / (n - 1.f) : m2;
      moving_mean[c] = mm - (1.f - momentum) * (mm - mean);
      moving_var[c] = mvv - (1.f - momentum) * (mvv - uvar);
    }
  }
}

void bn_finalize(const float* stat_part, int tiles, int tile_rows, int M, int C,
                 const float* gamma, const float* beta, float* moving_mean, float* moving_var,
                 float momentum, float eps, int update_moving, float* mean, float* rstd,
                 float* scale, float* shift, hipStream_t s) {
  if (fin_use_v2(tiles, C, false)) {
    hipLaunchKernelGGL(bn_finalize_chan_kernel, dim3(C), dim3(256), 0, s, stat_part, tiles,
                       tile_rows, M, C, gamma, beta, moving_mean, moving_var, momentum, eps,
                       update_moving, mean, rstd, scale, shift);
    DTR_CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, s, stat_part, tiles, tile_rows,
                     M, C, gamma, beta, moving_mean, moving_var, momentum, eps, update_moving,
                     mean, rstd, scale, shift);
  DTR_CHECK_LAUNCH();
}

// Accumulator mode (GemmArgs::stat_acc): the producer's workgroups added their
// tile sums into BN_ACC_REP fp64 replicas; one thread per channel finalizes.
__global__ void bn_finalize_acc_kernel(const double* __restrict__ acc, int M, int C,
                                       const float* __restrict__ gamma,
                                       const float* __restrict__ beta, float* moving_mean,
                                       float* moving_var, float momentum, float eps,
                                       int update_moving, float* mean_out, float* rstd_out,
                                       float* scale_out, float* shift_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s1, s2;
  bn_acc_sums(acc, C, c, s1, s2);
  const double dm = s1 / (double)M;
  const double var = fmax(s2 / (double)M - dm * dm, 0.0);
  const float mean = (float)dm, fvar = (float)var;
  const float rstd = rsqrtf(fvar + eps);
  const float sc = gamma[c] * rstd;
  mean_out[c] = mean;
  rstd_out[c] = rstd;
  scale_out[c] = sc;
  shift_out[c] = beta[c] - mean * sc;
  if (update_moving) {
    const float uvar = M > 1 ? (float)(var * M / (M - 1.0)) : fvar;
    const float mm = moving_mean[c], mvv = moving_var[c];
    moving_mean[c] = mm - (1.f - momentum) * (mm - mean);
    moving_var[c] = mvv - (1.f - momentum) * (mvv - uvar);
  }
}

void bn_finalize_acc(const double* acc, int M, int C, const float* gamma, const float* beta,
                     float* moving_mean, float* moving_var, float momentum, float eps,
                     int update_moving, float* mean, float* rstd, float* scale, float* shift,
                     hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_acc_kernel, dim3((C + 255) / 256), dim3(256), 0, s, acc, M, C,
                     gamma, beta, moving_mean, moving_var, momentum, eps, update_moving, mean,
                     rstd, scale, shift);
  DTR_CHECK_LAUNCH();
}

__global__ void bn_bwd_finalize_acc_kernel(const double* __restrict__ acc, int M, int C,
                                           const float* __restrict__ gamma,
                                           const float* __restrict__ rstd, float* dgamma,
                                           float* dbeta, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s1, s2;
  bn_acc_sums(acc, C, c, s1, s2);
  const float sg = (float)s1, sgx = (float)s2;
  const float a = gamma[c] * rstd[c];
  dbeta[c] = sg;
  dgamma[c] = sgx;
  coef[c] = a;
  coef[C + c] = a * sg / (float)M;
  coef[2 * C + c] = a * sgx / (float)M;
}

void bn_bwd_finalize_acc(const double* acc, int M, int C, const float* gamma, const float* rstd,
                         float* dgamma, float* dbeta, float* coef, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_acc_kernel, dim3((C + 255) / 256), dim3(256), 0, s, acc, M,
                     C, gamma, rstd, dgamma, dbeta, coef);
  DTR_CHECK_LAUNCH();
}

__global__ void bn_eval_kernel(const float* gamma, const float* beta, const float* mm,
                               const float* mv, float eps, int C, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    const float sc = gamma[c] * rsqrtf(mv[c] + eps);
    scale[c] = sc;
    shift[c] = beta[c] - mm[c] * sc;
  }
}

void bn_scale_shift_eval(const float* gamma, const float* beta, const float* moving_mean,
                         const float* moving_var, float eps, int C, float* scale, float* shift,
                         hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_kernel, dim3((C + 255) / 256), dim3(256), 0, s, gamma, beta,
                     moving_mean, moving_var, eps, C, scale, shift);
  DTR_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Row-tiled reductions over [M][C] bf16: each thread owns one 8-channel group
// (16-B vector loads) of a subset of rows.  Tile = BN_TILE_ROWS rows.
// ---------------------------------------------------------------------------
static constexpr int BN_TILE_ROWS = 256;
static constexpr int BN_ROW_BATCH = 8;   // rows whose loads are in flight together

int bn_bwd_tiles(int M, int C) { return (M + BN_TILE_ROWS - 1) / BN_TILE_ROWS; }
int bn_stats_tile_rows() { return BN_TILE_ROWS; }

// Standalone forward stats (for BN inputs not produced by a conv, e.g. after
// max-pool).  Two passes over the tile (the second from L1/L2) -> (mean, M2).
__global__ void __launch_bounds__(256)
bn_stats_kernel(const bf16* __restrict__ x, int M, int C, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [256/groups][C]... reused
  const int G = C / 8;                 // channel groups
  const int tid = threadIdx.x;
  const int rows_per_iter = 256 / G;   // C <= 2048 -> G <= 256
  const int grp = tid % G, rsub = tid / G;
  const int r0 = blockIdx.x * BN_TILE_ROWS;
  const int r1 = min(M, r0 + BN_TILE_ROWS);
  const bool active = rsub < rows_per_iter;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    int r = r0 + rsub;
    for (; r + (BN_ROW_BATCH - 1) * rows_per_iter < r1; r += BN_ROW_BATCH * rows_per_iter) {
      bf16x8 v[BN_ROW_BATCH];
#pragma unroll
      for (int u = 0; u < BN_ROW_BATCH; ++u)
        v[u] = *reinterpret_cast<const bf16x8*>(x + (long)(r + u * rows_per_iter) * C + grp * 8);
#pragma unroll
      for (int u = 0; u < BN_ROW_BATCH; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (float)v[u][j];
    }
    for (; r < r1; r += rows_per_iter) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (long)r * C + grp * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
    }
  }
  // reduce over rsub via LDS: red[rsub][C]
  float* buf = red;
  if (active)
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[rsub * C + grp * 8 + j] = s[j];
  __syncthreads();
  const float n = (float)(r1 - r0);
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int k = 0; k < rows_per_iter; ++k) t += buf[k * C + c];
    buf[rows_per_iter * C + c] = t / n;   // mean stored after the partial rows
  }
  __syncthreads();
  float mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) mu[j] = buf[rows_per_iter * C + grp * 8 + j];
  float q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    int r = r0 + rsub;
    for (; r + (BN_ROW_BATCH - 1) * rows_per_iter < r1; r += BN_ROW_BATCH * rows_per_iter) {
      bf16x8 v[BN_ROW_BATCH];
#pragma unroll
      for (int u = 0; u < BN_ROW_BATCH; ++u)
        v[u] = *reinterpret_cast<const bf16x8*>(x + (long)(r + u * rows_per_iter) * C + grp * 8);
#pragma unroll
      for (int u = 0; u < BN_ROW_BATCH; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)v[u][j] - mu[j];
          q[j] += d * d;
        }
    }
    for (; r < r1; r += rows_per_iter) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (long)r * C + grp * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)v[j] - mu[j];
        q[j] += d * d;
      }
    }
  }
  __syncthreads();
  if (active)
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[rsub * C + grp * 8 + j] = q[j];
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int k = 0; k < rows_per_iter; ++k) t += buf[k * C + c];
    part[(long)blockIdx.x * 2 * C + c] = buf[rows_per_iter * C + c];
    part[(long)blockIdx.x * 2 * C + C + c] = t;
  }
}

void bn_stats(const bf16* x, int M, int C, float* part, hipStream_t s) {
  const int G = C / 8;
  const int rpi = 256 / G;
  const size_t lds = (size_t)(rpi + 1) * C * sizeof(float);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(bn_bwd_tiles(M, C)), dim3(256), lds, s, x, M, C,
                     part);
  DTR_CHECK_LAUNCH();
}

// Backward reduction: per tile sums of g and g*xhat, g = dy*[relu active].
__global__ void __launch_bounds__(256)
bn_bwd_reduce_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                     const float* __restrict__ mean, const float* __restrict__ rstd,
                     const float* __restrict__ scale, const float* __restrict__ shift, int M,
                     int C, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int G = C / 8, tid = threadIdx.x;
  const int rows_per_iter = 256 / G;
  const int grp = tid % G, rsub = tid / G;
  const int r0 = blockIdx.x * BN_TILE_ROWS, r1 = min(M, r0 + BN_TILE_ROWS);
  const bool active = rsub < rows_per_iter;
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], rs[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = grp * 8 + j;
    mu[j] = active ? mean[c] : 0.f;
    rs[j] = active ? rstd[c] : 0.f;
    sc[j] = active ? scale[c] : 0.f;
    sh[j] = active ? shift[c] : 0.f;
  }
  // Rows in batches of BN_ROW_BATCH with every load issued before the math: with
  // C = 2048 a thread owns all 256 rows of its tile, and one round trip per row
  // made this 25-workgroup launch ~110 us.  Same accumulation order as row by row.
  auto acc_row = [&](const bf16x8& d, const bf16x8& v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = (float)v[j];
      const float gg = (xv * sc[j] + sh[j] > 0.f) ? (float)d[j] : 0.f;
      sg[j] += gg;
      sgx[j] += gg * (xv - mu[j]) * rs[j];
    }
  };
  if (active) {
    int r = r0 + rsub;
    for (; r + (BN_ROW_BATCH - 1) * rows_per_iter < r1; r += BN_ROW_BATCH * rows_per_iter) {
      bf16x8 d[BN_ROW_BATCH], v[BN_ROW_BATCH];
#pragma unroll
      for (int u = 0; u < BN_ROW_BATCH; ++u) {
        const long o = (long)(r + u * rows_per_iter) * C + grp * 8;
        d[u] = *reinterpret_cast<const bf16x8*>(dy + o);
        v[u] = *reinterpret_cast<const bf16x8*>(x + o);
      }
#pragma unroll
      for (int u = 0; u < BN_ROW_BATCH; ++u) acc_row(d[u], v[u]);
    }
    for (; r < r1; r += rows_per_iter) {
      const long o = (long)r * C + grp * 8;
      acc_row(*reinterpret_cast<const bf16x8*>(dy + o), *reinterpret_cast<const bf16x8*>(x + o));
    }
  }
  if (active)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[rsub * 2 * C + grp * 8 + j] = sg[j];
      red[rsub * 2 * C + C + grp * 8 + j] = sgx[j];
    }
  __syncthreads();
  for (int c = tid; c < 2 * C; c += 256) {
    float t = 0.f;
    for (int k = 0; k < rows_per_iter; ++k) t += red[k * 2 * C + c];
    part[(long)blockIdx.x * 2 * C + c] = t;
  }
}

void bn_relu_bwd_reduce(const bf16* dy, const bf16* x, const float* mean, const float* rstd,
                        const float* scale, const float* shift, int M, int C, float* part,
                        int* tiles_out, hipStream_t s) {
  const int G = C / 8, rpi = 256 / G;
  const size_t lds = (size_t)rpi * 2 * C * sizeof(float);
  const int tiles = bn_bwd_tiles(M, C);
  if (tiles_out) *tiles_out = tiles;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(tiles), dim3(256), lds, s, dy, x, mean, rstd,
                     scale, shift, M, C, part);
  DTR_CHECK_LAUNCH();
}

// dgamma/dbeta (written into the flat gradient) + apply coefficients.
// Block = 64 channels x 16 tile-rows: each thread folds every 16th tile
// (coalesced over channels, independent loads in flight), then a fixed-order
// LDS combine -- deterministic, and ~100x faster than one serial thread per
// channel over 500-1600 partial tiles.
__global__ void __launch_bounds__(1024)
bn_bwd_finalize_kernel(const float* __restrict__ part, int tiles, int M, int C,
                       const float* __restrict__ gamma, const float* __restrict__ rstd,
                       float* dgamma, float* dbeta, float* coef) {
  __shared__ float s0[16][64], s1[16][64];
  const int cx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cx;
  const float a = (ty == 0 && c < C) ? gamma[c] * rstd[c] : 0.f;   // ahead of the partials
  float sg = 0.f, sgx = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int t = ty; t < tiles; t += 16) {
      sg += part[(long)t * 2 * C + c];
      sgx += part[(long)t * 2 * C + C + c];
    }
  }
  s0[ty][cx] = sg;
  s1[ty][cx] = sgx;
  __syncthreads();
  if (ty == 0 && c < C) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a0 += s0[k][cx];
      a1 += s1[k][cx];
    }
    dbeta[c] = a0;
    dgamma[c] = a1;
    coef[c] = a;
    coef[C + c] = a * a0 / (float)M;
    coef[2 * C + c] = a * a1 / (float)M;
  }
}

void bn_bwd_finalize(const float* part, int tiles, int M, int C, const float* gamma,
                     const float* rstd, float* dgamma, float* dbeta, float* coef,
                     hipStream_t s) {
  if (fin_use_v2(tiles, C, true)) {
    hipLaunchKernelGGL(bn_bwd_finalize_chan_kernel, dim3(C), dim3(256), 0, s, part, tiles, M, C,
                       gamma, rstd, dgamma, dbeta, coef);
    DTR_CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, part, tiles,
                     M, C, gamma, rstd, dgamma, dbeta, coef);
  DTR_CHECK_LAUNCH();
}

// Streaming BN+ReLU backward apply, dx = a*g - b - c*xhat (+ add), g = dy*[x*scale+shift > 0].
// The grid stride is a multiple of the channel-group count G = C/8 (G divides the
// 256-thread block), so each thread owns ONE fixed 8-channel group: its 7 x 8
// per-channel parameters are loaded once into registers instead of 56 scalar
// loads + a 64-bit modulo per vector, and U vectors per thread are in flight at
// once (the per-vector load->store chain measured ~2 TB/s).
template <int U>
__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                    const float* __restrict__ mean, const float* __restrict__ rstd,
                    const float* __restrict__ scale, const float* __restrict__ shift,
                    const float* __restrict__ coef, const bf16* __restrict__ add,
                    bf16* __restrict__ dx, long nvec, int C, BwdAccFin fin) {
  const int G = C / 8;
  const long T = (long)gridDim.x * 256;
  const int c0 = (int)(threadIdx.x % G) * 8;
  float sc[8], sh[8], mu[8], rs[8], ca[8], cb[8], cc[8];
  extern __shared__ float cf[];   // acc mode: [3][C] coefficients
  const float* cfp = coef;
  if (fin.acc != nullptr) {   // accumulator mode: this launch is also the finalize
    for (int c = threadIdx.x; c < C; c += 256) {
      double s1, s2;
      bn_acc_sums(fin.acc, C, c, s1, s2);
      const float sg = (float)s1, sgx = (float)s2;
      const float a = fin.gamma[c] * rstd[c];
      const float b = a * sg / (float)fin.M, d = a * sgx / (float)fin.M;
      cf[c] = a;
      cf[C + c] = b;
      cf[2 * C + c] = d;
      if (blockIdx.x == 0) {
        fin.dbeta[c] = sg;
        fin.dgamma[c] = sgx;
        fin.coef[c] = a;
        fin.coef[C + c] = b;
        fin.coef[2 * C + c] = d;
      }
    }
    __syncthreads();
    cfp = cf;
  }
  const int ld = C;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    sc[j] = scale[c];
    sh[j] = shift[c];
    mu[j] = mean[c];
    rs[j] = rstd[c];
    ca[j] = cfp[c];
    cb[j] = cfp[ld + c];
    cc[j] = cfp[2 * ld + c];
  }
  const bf16x8 zero8 = {};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nvec; i += U * T) {
    bf16x8 d[U], v[U], ad[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long iu = i + u * T;
      const bool ok = iu < nvec;
      d[u] = ok ? *reinterpret_cast<const bf16x8*>(dy + iu * 8) : zero8;
      v[u] = ok ? *reinterpret_cast<const bf16x8*>(x + iu * 8) : zero8;
      ad[u] = (ok && add) ? *reinterpret_cast<const bf16x8*>(add + iu * 8) : zero8;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long iu = i + u * T;
      if (iu >= nvec) break;
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = (float)v[u][j];
        const float gg = (xv * sc[j] + sh[j] > 0.f) ? (float)d[u][j] : 0.f;
        const float xh = (xv - mu[j]) * rs[j];
        r[j] = (bf16)(ca[j] * gg - cb[j] - cc[j] * xh + (float)ad[u][j]);
      }
      *reinterpret_cast<bf16x8*>(dx + iu * 8) = r;
    }
  }
}

void bn_relu_bwd_apply(const bf16* dy, const bf16* x, const float* mean, const float* rstd,
                       const float* scale, const float* shift, const float* coef,
                       const bf16* add, bf16* dx, int M, int C, hipStream_t s) {
  const int G = C / 8;
  if (C % 8 != 0 || 256 % G != 0)
    throw std::runtime_error("bn_relu_bwd_apply: C/8 must divide 256");
  const long nvec = (long)M * C / 8;
  constexpr int U = 2;
  long blocks = (nvec + 256L * U - 1) / (256L * U);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(bn_bwd_apply_kernel<U>, dim3((unsigned)blocks), dim3(256), 0, s, dy, x,
                     mean, rstd, scale, shift, coef, add, dx, nvec, C, BwdAccFin{});
  DTR_CHECK_LAUNCH();
}

// Grid of the finalize-fused apply: every workgroup re-reads 16 fp64 per channel, so
// the grid is capped (BWD_FIN_BLOCKS, 4 vectors in flight per thread instead of 2).
// (256: the RN50 shapes stream at 4.9-5.9 TB/s; caps of 512-2048 measured no faster,
// profiles/bn_bwd_apply_bandwidth.md)
constexpr int BWD_FIN_U = 4;
constexpr long BWD_FIN_BLOCKS = 256;
static long bwd_fin_blocks(long nvec) {
  const long b = (nvec + 256L * BWD_FIN_U - 1) / (256L * BWD_FIN_U);
  return b < BWD_FIN_BLOCKS ? b : BWD_FIN_BLOCKS;
}

// round-1 rule (the CIFAR shapes): C <= 64 on the uncapped U = 2 grid of <= 1024 blocks
static bool bwd_fin_small(int M, int C) {
  return C <= BWD_ACC_FIN_MAXC && ((long)M * C / 8 + 511) / 512 <= 1024;
}

// tune bwd_apply_fin: 0 = only C <= 64 (round-1 rule), 1 (default) = when the grid's
// redundant finalize reads stay <= 1/4 of the apply's streamed bytes, 2 = always.
bool bn_bwd_apply_acc_fits(int M, int C) {
  const long mode = tune(T_BWD_APPLY_FIN);
  const long nvec = (long)M * C / 8;
  if (C % 8 != 0 || 256 % (C / 8) != 0 || C > 2048) return false;
  if (bwd_fin_small(M, C)) return true;
  if (mode == 0) return false;
  if (mode >= 2) return true;
  return bwd_fin_blocks(nvec) * C * 16L * 8 <= nvec * 48 / 4;
}

void bn_relu_bwd_apply_acc(const bf16* dy, const bf16* x, const float* mean, const float* rstd,
                           const float* scale, const float* shift, const BwdAccFin& fin,
                           const bf16* add, bf16* dx, int M, int C, hipStream_t s) {
  if (!bn_bwd_apply_acc_fits(M, C))
    throw std::runtime_error("bn_relu_bwd_apply_acc: shape exceeds the fused-finalize bound");
  const long nvec = (long)M * C / 8;
  if (bwd_fin_small(M, C)) {   // measured: CIFAR keeps its wider U = 2 grid
    hipLaunchKernelGGL(bn_bwd_apply_kernel<2>, dim3((unsigned)((nvec + 511) / 512)), dim3(256),
                       (size_t)3 * C * sizeof(float), s, dy, x, mean, rstd, scale, shift, fin.coef,
                       add, dx, nvec, C, fin);
    DTR_CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL(bn_bwd_apply_kernel<BWD_FIN_U>, dim3((unsigned)bwd_fin_blocks(nvec)),
                     dim3(256), (size_t)3 * C * sizeof(float), s, dy, x, mean, rstd, scale, shift,
                     fin.coef, add, dx, nvec, C, fin);
  DTR_CHECK_LAUNCH();
}

__global__ void bn_relu_apply_kernel(const bf16* __restrict__ x, const float* __restrict__ scale,
                                     const float* __restrict__ shift, bf16* __restrict__ y,
                                     unsigned nvec, int C) {
  const unsigned G = (unsigned)C / 8;   // 32-bit index math (host: nvec < 2^31)
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % G) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (size_t)i * 8);
    *reinterpret_cast<bf16x8*>(y + (size_t)i * 8) = affine_relu8(v, scale + c0, shift + c0);
  }
}

// Accumulator-mode finalize fused into the materializing BN+ReLU pass (the inner
// bottleneck BatchNorms of the 14x14 / 7x7 stages, Engine._materialize_bn): every
// workgroup finalizes the channels from the fp64 replicas into an LDS scale/shift table
// (the bn_finalize_acc math; block 0 also writes mean/rstd/scale/shift and the moving
// averages for the BN's later users), then streams U vectors per thread per round.
// <= 256 workgroups keep the redundant finalize reads (16 fp64 per channel per
// workgroup) at a few MB of L2 traffic; one launch instead of finalize + apply.
template <int U>
__global__ void __launch_bounds__(256)
bn_relu_apply_acc_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, unsigned nvec, int M,
                         int C, const double* __restrict__ acc, const float* __restrict__ gamma,
                         const float* __restrict__ beta, float* moving_mean, float* moving_var,
                         float momentum, float eps, int update_moving, float* mean_out,
                         float* rstd_out, float* scale_out, float* shift_out) {
  extern __shared__ __attribute__((aligned(16))) float tab[];   // [2][C]: scale, shift
  for (int c = threadIdx.x; c < C; c += 256) {
    double s1, s2;
    bn_acc_sums(acc, C, c, s1, s2);
    const double dm = s1 / (double)M;
    const double var = fmax(s2 / (double)M - dm * dm, 0.0);
    const float mean = (float)dm, fvar = (float)var;
    const float rstd = rsqrtf(fvar + eps);
    const float sc = gamma[c] * rstd, sh = beta[c] - mean * sc;
    tab[c] = sc;
    tab[C + c] = sh;
    if (blockIdx.x == 0) {
      mean_out[c] = mean;
      rstd_out[c] = rstd;
      scale_out[c] = sc;
      shift_out[c] = sh;
      if (update_moving) {
        const float uvar = M > 1 ? (float)(var * M / (M - 1.0)) : fvar;
        const float mm = moving_mean[c], mvv = moving_var[c];
        moving_mean[c] = mm - (1.f - momentum) * (mm - mean);
        moving_var[c] = mvv - (1.f - momentum) * (mvv - uvar);
      }
    }
  }
  __syncthreads();
  const unsigned G = (unsigned)C / 8, T = gridDim.x * 256u;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < nvec; i += U * T) {
    bf16x8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned iu = i + u * T;
      if (iu < nvec) v[u] = *reinterpret_cast<const bf16x8*>(x + (size_t)iu * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned iu = i + u * T;
      if (iu >= nvec) break;
      const int c0 = (int)(iu % G) * 8;
      *reinterpret_cast<bf16x8*>(y + (size_t)iu * 8) = affine_relu8(v[u], tab + c0, tab + C + c0);
    }
  }
}

void bn_relu_apply_acc(const bf16* x, bf16* y, int M, int C, const double* acc,
                       const float* gamma, const float* beta, float* moving_mean,
                       float* moving_var, float momentum, float eps, int update_moving,
                       float* mean, float* rstd, float* scale, float* shift, hipStream_t s) {
  const long nvec = (long)M * C / 8;
  if (C % 8 != 0 || C > 4096 || nvec >= (1L << 31))
    throw std::runtime_error("bn_relu_apply_acc: C % 8, C <= 4096, M*C/8 < 2^31");
  constexpr int U = 4;
  long blocks = (nvec + 256L * U - 1) / (256L * U);
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(bn_relu_apply_acc_kernel<U>, dim3((unsigned)blocks), dim3(256),
                     (size_t)2 * C * sizeof(float), s, x, y, (unsigned)nvec, M, C, acc, gamma, beta,
                     moving_mean, moving_var, momentum, eps, update_moving, mean, rstd, scale,
                     shift);
  DTR_CHECK_LAUNCH();
}

void bn_relu_apply(const bf16* x, const float* scale, const float* shift, bf16* y, int M, int C,
                   hipStream_t s) {
  const long nvec = (long)M * C / 8;
  if (nvec >= (1L << 31)) throw std::runtime_error("bn_relu_apply: tensor too large");
  long blocks = (nvec + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bn_relu_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, scale,
                     shift, y, (unsigned)nvec, C);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
