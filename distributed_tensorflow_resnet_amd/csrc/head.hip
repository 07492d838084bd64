// Network head and stem helpers:
//   * final BN-ReLU fused with the global average pool
//     (resnet_model_official.py:268-271 / 335-339: batch_norm_relu -> average_pooling2d)
//   * softmax cross-entropy, mean over the batch, fused with the training
//     precision (argmax == label, resnet_cifar_main.py:284-286) and the dense
//     bias gradient (resnet_model.py:77-80)
//   * 3x3/2 SAME max-pool of the ImageNet stem (resnet_model_official.py:314-316;
//     TF SAME pads 0 before / 1 after for 112 -> 56); the forward records the
//     first-max window index, the backward gathers through it (deterministic).
#include <stdexcept>

#include "bn_fused.h"
#include "common.h"
#include "kernels.h"

namespace dtr {

// pooled[n][c] = mean_hw relu(x[n][hw][c]*scale[c] + shift[c]); one block per
// image, 8 channels per thread-slot, rows strided over the block.
__global__ void __launch_bounds__(256)
bnrelu_avgpool_kernel(const bf16* __restrict__ x, const float* __restrict__ scale,
                      const float* __restrict__ shift, bf16* __restrict__ pooled, int HW,
                      int C) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int n = blockIdx.x, tid = threadIdx.x;
  const int G = C / 8;
  const int rpi = max(1, 256 / G);
  const int grp = tid % G, rsub = tid / G;
  const bool active = (grp < G) && (rsub < rpi) && tid < G * rpi;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = scale[grp * 8 + j];
      sh[j] = shift[grp * 8 + j];
    }
    for (int p = rsub; p < HW; p += rpi) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((long)n * HW + p) * C + grp * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += fmaxf((float)v[j] * sc[j] + sh[j], 0.f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rsub * C + grp * 8 + j] = s[j];
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int k = 0; k < rpi; ++k) t += red[k * C + c];
    pooled[(long)n * C + c] = (bf16)(t / (float)HW);
  }
}

void bnrelu_avgpool(const bf16* x, const float* scale, const float* shift, bf16* pooled, int N,
                    int HW, int C, hipStream_t s) {
  const int G = C / 8;
  const int rpi = G >= 256 ? 1 : 256 / G;
  const size_t lds = (size_t)rpi * C * sizeof(float);
  // C > 2048 would need multiple passes; ResNet heads are 64 / 2048 channels.
  hipLaunchKernelGGL(bnrelu_avgpool_kernel, dim3(N), dim3(256), lds, s, x, scale, shift, pooled,
                     HW, C);
  DTR_CHECK_LAUNCH();
}

// d_act[n][hw][c] = dpooled[n][c] / HW  (the ReLU mask / BN backward follow in
// bn_relu_bwd_*).
__global__ void avgpool_bwd_kernel(const bf16* __restrict__ dp, bf16* __restrict__ dx, int HW,
                                   int C, long nvec) {
  const int G = C / 8;
  const float inv = 1.f / (float)HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / G;
    const int grp = (int)(i - row * G);
    const long n = row / HW;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(dp + n * C + grp * 8);
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)((float)v[j] * inv);
    *reinterpret_cast<bf16x8*>(dx + i * 8) = r;
  }
}

void avgpool_bwd(const bf16* dpooled, bf16* dx, int N, int HW, int C, hipStream_t s) {
  const long nvec = (long)N * HW * C / 8;
  long blocks = (nvec + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dpooled, dx,
                     HW, C, nvec);
  DTR_CHECK_LAUNCH();
}

// Single 1024-thread block (N <= a few thousand rows): one wave per row at a
// time, fixed reduction order -> deterministic loss / precision / dbias.
// dlogits = (softmax - onehot) * grad_scale   (grad_scale = 1/global_batch).
__global__ void __launch_bounds__(1024)
softmax_xent_kernel(const float* __restrict__ logits, int ld, const int* __restrict__ labels,
                    int N, int classes, float* loss_sum, float* correct,
                    bf16* __restrict__ dlogits, float* __restrict__ dbias, float grad_scale,
                    float* __restrict__ probs) {
  extern __shared__ __attribute__((aligned(16))) float sh[];  // [16 waves][ld] dbias partial + misc
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nw = blockDim.x >> 6;
  float* db = sh;                    // [nw][ld]
  float* wl = sh + nw * ld;          // [nw] loss
  float* wc = wl + nw;               // [nw] correct
  for (int c = lane; c < ld; c += 64) db[wave * ld + c] = 0.f;
  float lsum = 0.f, csum = 0.f;
  for (int row = wave; row < N; row += nw) {
    const float* z = logits + (long)row * ld;
    float mx = -INFINITY;
    int amax = 0;
    for (int c = lane; c < classes; c += 64) {
      const float v = z[c];
      if (v > mx) { mx = v; amax = c; }
    }
    // wave argmax (first max on ties, like tf.argmax)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(amax, o, 64);
      if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
    }
    float se = 0.f;
    for (int c = lane; c < classes; c += 64) se += __expf(z[c] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    const int y = labels[row];
    const float zy = (y >= 0 && y < classes) ? z[y] : lse;
    if (lane == 0) {
      lsum += lse - zy;
      csum += (amax == y) ? 1.f : 0.f;
    }
    for (int c = lane; c < ld; c += 64) {
      float g = 0.f;
      if (c < classes) {
        const float p = __expf(z[c] - lse);
        if (probs) probs[(long)row * ld + c] = p;
        g = (p - (c == y ? 1.f : 0.f)) * grad_scale;
      }
      if (dlogits) dlogits[(long)row * ld + c] = (bf16)g;
      db[wave * ld + c] += g;
    }
  }
  if (lane == 0) {
    wl[wave] = lsum;
    wc[wave] = csum;
  }
  __syncthreads();
  for (int c = tid; c < ld; c += blockDim.x) {
    float t = 0.f;
    for (int w = 0; w < nw; ++w) t += db[w * ld + c];
    if (dbias && c < classes) dbias[c] = t;
  }
  if (tid == 0) {
    float l = 0.f, k = 0.f;
    for (int w = 0; w < nw; ++w) {
      l += wl[w];
      k += wc[w];
    }
    if (loss_sum) *loss_sum = l;
    if (correct) *correct = k;
  }
}

// Row-parallel variant (ws != nullptr): the single-block kernel above walks the
// rows 16 at a time and each row three times from global memory -- ~100 us for
// 128 x 1000 ImageNet logits on the critical path.  Here one wave owns one row,
// holds it in registers (VPL values per lane) and writes the per-row loss /
// correct flag and the fp32 gradient row to `ws`; softmax_xent_reduce_kernel
// then folds dbias (per column, rows in fixed order) and the scalars.
// Deterministic: every sum has a fixed order independent of the grid.
template <int VPL>
__global__ void __launch_bounds__(256)
softmax_xent_rows_kernel(const float* __restrict__ logits, int ld, const int* __restrict__ labels,
                         int N, int classes, bf16* __restrict__ dlogits, float grad_scale,
                         float* __restrict__ probs, float* __restrict__ ws, bool want_g) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;   // wave-uniform
  const float* z = logits + (long)row * ld;
  float v[VPL];
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int c = lane + 64 * k;
    v[k] = c < classes ? z[c] : -INFINITY;
  }
  float mx = -INFINITY;
  int amax = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < VPL; ++k)
    if (v[k] > mx) { mx = v[k]; amax = lane + 64 * k; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {   // first max on ties, like tf.argmax
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) se += (lane + 64 * k < classes) ? __expf(v[k] - mx) : 0.f;
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const int y = labels[row];
  float* gw = ws + (long)row * ld;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int c = lane + 64 * k;
    if (c >= ld) break;
    float g = 0.f;
    if (c < classes) {
      const float p = __expf(v[k] - lse);
      if (probs) probs[(long)row * ld + c] = p;
      g = (p - (c == y ? 1.f : 0.f)) * grad_scale;
    }
    if (dlogits) dlogits[(long)row * ld + c] = (bf16)g;
    if (want_g) gw[c] = g;
  }
  if (lane == 0) {
    const float zy = (y >= 0 && y < classes) ? z[y] : lse;
    float* rs = ws + (long)N * ld + 2 * row;
    rs[0] = lse - zy;
    rs[1] = (amax == y) ? 1.f : 0.f;
  }
}

// grid = ceil(classes / 64) blocks of 256: thread (column c, row slice q = tid / 64)
// sums rows q, q + 4, ... ; the 4 slices are added in fixed order.  Block 0 also
// folds the per-row loss / correct flags.
__global__ void __launch_bounds__(256)
softmax_xent_reduce_kernel(const float* __restrict__ ws, int ld, int N, int classes,
                           float* loss_sum, float* correct, float* __restrict__ dbias) {
  __shared__ float red[4][64];
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  const int c = blockIdx.x * 64 + lane;
  if (dbias) {
    float t = 0.f;
    if (c < classes) {
#pragma unroll 8
      for (int r = q; r < N; r += 4) t += ws[(long)r * ld + c];
    }
    red[q][lane] = t;
    __syncthreads();
    if (q == 0 && c < classes) dbias[c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  }
  if (blockIdx.x == 0 && q == 0) {
    const float* rs = ws + (long)N * ld;
    float l = 0.f, k = 0.f;
    for (int r = lane; r < N; r += 64) {
      l += rs[2 * r];
      k += rs[2 * r + 1];
    }
    l = wave_sum(l);
    k = wave_sum(k);
    if (lane == 0) {
      if (loss_sum) *loss_sum = l;
      if (correct) *correct = k;
    }
  }
}

long softmax_xent_ws_floats(int N, int ld) { return (long)N * ld + 2L * N; }

void softmax_xent_reduce(const float* ws, int ld, int N, int classes, float* loss_sum,
                         float* correct, float* dbias, hipStream_t s) {
  const int cb = dbias ? (classes + 63) / 64 : 1;
  hipLaunchKernelGGL(softmax_xent_reduce_kernel, dim3((unsigned)cb), dim3(256), 0, s, ws, ld, N,
                     classes, loss_sum, correct, dbias);
  DTR_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Fused training head (HeadArgs, kernels.h): one workgroup per image.  Thread t owns
// the 8-channel group t % G of pixels t / G, t / G + 256 / G, ...; per-channel sums
// over the image fold the wave by xor-shuffles (lanes G apart share a group) and
// the 4 waves through LDS in fixed order.  Numerics follow the unfused chain: bf16
// pooled, fp32 logits + bias, bf16 dlogits, fp32-accumulated dense dgrad rounded to
// bf16, avg-pool backward rounded to bf16, BN backward sums of that bf16 gradient.
template <int C>
__device__ __forceinline__ void head_colsum(float (&v)[8], float (*red)[C]) {
  constexpr int G = C / 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int off = G; off < 64; off <<= 1) v[j] += __shfl_xor(v[j], off, 64);
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = v[j];
  }
}

template <int C, int UPT>
__global__ void __launch_bounds__(256) head_fused_kernel(HeadArgs a) {
  constexpr int G = C / 8;
  __shared__ float sc_s[C], sh_s[C], mu_s[C], rs_s[C], pool_s[C], dp_s[C], g_s[64];
  __shared__ float red[4][C], red2[4][C];
  __shared__ float w_s[C * 64];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = tid % G;
  const int HW = a.HW, kpad = a.kpad, nunits = HW * G;
  const bf16x8 zero8 = {};
  // ---- loads: this image's activations (registers), dense weights (LDS) ----
  bf16x8 xv[UPT];
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    const int u = tid + i * 256;
    xv[i] = u < nunits ? *reinterpret_cast<const bf16x8*>(a.x + ((long)n * nunits + u) * 8)
                       : zero8;
  }
  for (int e = tid; e < C * kpad; e += 256) w_s[e] = (float)a.w[e];
  // ---- final BN statistics from the accumulators (block 0 publishes them) ----
  if (tid < C) {
    const int c = tid;
    double s1, s2;
    bn_acc_sums(a.acc, C, c, s1, s2);
    const double M = (double)a.N * HW;
    const double dm = s1 / M;
    const double var = fmax(s2 / M - dm * dm, 0.0);
    const float fmu = (float)dm, fvar = (float)var;
    const float rs = rsqrtf(fvar + a.eps);
    const float sc = a.gamma[c] * rs;
    const float sh = a.beta[c] - fmu * sc;
    sc_s[c] = sc;
    sh_s[c] = sh;
    mu_s[c] = fmu;
    rs_s[c] = rs;
    if (n == 0) {
      a.mean[c] = fmu;
      a.rstd[c] = rs;
      a.scale[c] = sc;
      a.shift[c] = sh;
      if (a.update_moving) {
        const float uvar = M > 1.0 ? (float)(var * M / (M - 1.0)) : fvar;
        const float mm = a.mmean[c], mv = a.mvar[c];
        a.mmean[c] = mm - (1.f - a.momentum) * (mm - fmu);
        a.mvar[c] = mv - (1.f - a.momentum) * (mv - uvar);
      }
    }
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = sc_s[grp * 8 + j];
    sh[j] = sh_s[grp * 8 + j];
  }
  // ---- BN + ReLU + global average pool ----
  {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      if (tid + i * 256 >= nunits) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += fmaxf((float)xv[i][j] * sc[j] + sh[j], 0.f);
    }
    head_colsum<C>(s, red);
  }
  __syncthreads();
  if (tid < C) {
    const float t = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    const bf16 pb = (bf16)(t / (float)HW);
    a.pooled[(long)n * C + tid] = pb;
    pool_s[tid] = (float)pb;
  }
  __syncthreads();
  // ---- dense + softmax cross-entropy row (wave 0, one class per lane) ----
  if (wave == 0) {
    const int y = a.labels[n];
    float z = -INFINITY;
    if (lane < a.classes) {
      float acc = 0.f;
#pragma unroll 8
      for (int c = 0; c < C; ++c) acc += pool_s[c] * w_s[c * kpad + lane];
      z = acc + a.bias[lane];
    }
    float mx = z;
    int amax = lane < a.classes ? lane : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {   // first max on ties, like tf.argmax
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(amax, o, 64);
      if (om > mx || (om == mx && oa < amax)) {
        mx = om;
        amax = oa;
      }
    }
    const float se = wave_sum(lane < a.classes ? __expf(z - mx) : 0.f);
    const float lse = mx + __logf(se);
    const float zy = __shfl(z, (y >= 0 && y < a.classes) ? y : 0, 64);
    float g = 0.f;
    if (lane < a.classes) g = (__expf(z - lse) - (lane == y ? 1.f : 0.f)) * a.grad_scale;
    if (lane < kpad) {
      const bf16 gb = (bf16)g;
      a.dlogits[(long)n * kpad + lane] = gb;
      a.ws[(long)n * kpad + lane] = g;
      g_s[lane] = (float)gb;
    }
    if (lane == 0) {
      float* rs = a.ws + (long)a.N * kpad + 2 * n;
      rs[0] = lse - ((y >= 0 && y < a.classes) ? zy : lse);
      rs[1] = (amax == y) ? 1.f : 0.f;
    }
  }
  __syncthreads();
  // ---- dense dgrad (bf16 out) -> average-pool backward (bf16) ----
  if (tid < C) {
    float d = 0.f;
    for (int k = 0; k < kpad; ++k) d += g_s[k] * w_s[tid * kpad + k];
    const float db = (float)(bf16)d;
    dp_s[tid] = (float)(bf16)(db * (1.f / (float)HW));
  }
  __syncthreads();
  // ---- dact rows + the final BN's backward sums (g = dact * relu mask) ----
  {
    float dv[8], mu[8], rs[8], s1[8], s2[8];
    bf16x8 dvb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dv[j] = dp_s[grp * 8 + j];
      dvb[j] = (bf16)dv[j];
      mu[j] = mu_s[grp * 8 + j];
      rs[j] = rs_s[grp * 8 + j];
      s1[j] = s2[j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int u = tid + i * 256;
      if (u >= nunits) continue;
      *reinterpret_cast<bf16x8*>(a.dact + ((long)n * nunits + u) * 8) = dvb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xf = (float)xv[i][j];
        const float gg = (xf * sc[j] + sh[j] > 0.f) ? dv[j] : 0.f;
        s1[j] += gg;
        s2[j] += gg * (xf - mu[j]) * rs[j];
      }
    }
    head_colsum<C>(s1, red);
    head_colsum<C>(s2, red2);
  }
  __syncthreads();
  if (tid < C) {
    const float t1 = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    const float t2 = (red2[0][tid] + red2[1][tid]) + (red2[2][tid] + red2[3][tid]);
    bn_acc_add(a.bacc, C, tid, (double)t1, (double)t2);
  }
}

bool head_fused_supported(int N, int HW, int C, int classes, int kpad) {
  return N > 0 && (C == 16 || C == 32 || C == 64) && HW >= 1 && HW * (C / 8) <= 4 * 256 &&
         kpad <= 64 && classes <= kpad && classes >= 1;
}

void head_fused(const HeadArgs& a, hipStream_t s) {
  if (!head_fused_supported(a.N, a.HW, a.C, a.classes, a.kpad))
    throw std::invalid_argument("head_fused: unsupported head shape");
  const int units = a.HW * (a.C / 8);
  const dim3 grid((unsigned)a.N);
#define DTR_HEAD(C_)                                                                        \
  if (a.C == C_) {                                                                          \
    if (units <= 256) hipLaunchKernelGGL((head_fused_kernel<C_, 1>), grid, dim3(256), 0, s, a); \
    else if (units <= 512) hipLaunchKernelGGL((head_fused_kernel<C_, 2>), grid, dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((head_fused_kernel<C_, 4>), grid, dim3(256), 0, s, a);           \
  }
  DTR_HEAD(16)
  DTR_HEAD(32)
  DTR_HEAD(64)
#undef DTR_HEAD
  DTR_CHECK_LAUNCH();
}

void softmax_xent(const float* logits, int ld, const int* labels, int N, int classes,
                  float* loss_sum, float* correct, bf16* dlogits, float* dbias, float grad_scale,
                  float* probs, float* ws, hipStream_t s) {
  if (ws != nullptr && ld <= 1024) {
    const dim3 grid((unsigned)((N + 3) / 4));
    const bool want_g = dbias != nullptr;
    if (ld <= 64)
      hipLaunchKernelGGL(softmax_xent_rows_kernel<1>, grid, dim3(256), 0, s, logits, ld, labels,
                         N, classes, dlogits, grad_scale, probs, ws, want_g);
    else if (ld <= 256)
      hipLaunchKernelGGL(softmax_xent_rows_kernel<4>, grid, dim3(256), 0, s, logits, ld, labels,
                         N, classes, dlogits, grad_scale, probs, ws, want_g);
    else
      hipLaunchKernelGGL(softmax_xent_rows_kernel<16>, grid, dim3(256), 0, s, logits, ld, labels,
                         N, classes, dlogits, grad_scale, probs, ws, want_g);
    DTR_CHECK_LAUNCH();
    const int cb = dbias ? (classes + 63) / 64 : 1;
    hipLaunchKernelGGL(softmax_xent_reduce_kernel, dim3((unsigned)cb), dim3(256), 0, s, ws, ld, N,
                       classes, loss_sum, correct, dbias);
    DTR_CHECK_LAUNCH();
    return;
  }
  const int threads = 1024, nw = threads / 64;
  const size_t lds = ((size_t)nw * ld + 2 * nw) * sizeof(float);
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(1), dim3(threads), lds, s, logits, ld, labels, N,
                     classes, loss_sum, correct, dlogits, dbias, grad_scale, probs);
  DTR_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// max pool (NHWC), window k, stride s, pad_top=pad_left=pad; out-of-range taps
// are excluded (TF SAME semantics).  The forward records, per output element,
// the window position (r*k+c) of the FIRST maximum in row-major window order;
// the backward is then a gather: every input element sums dy over the <= 4
// windows whose recorded argmax is itself (deterministic, no atomics), with
// 8 channels per thread (16-B bf16 loads, 8-B index loads).
// ---------------------------------------------------------------------------
__global__ void maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                   uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                   int Wo, int k, int st, int pad) {
  // 32-bit index math (the host checks total < 2^31): 64-bit divisions cost
  // ~3x the kernel's memory time on the ImageNet stem shapes.
  const unsigned G = (unsigned)C / 8;
  const unsigned total = (unsigned)N * Ho * Wo * G;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const int grp = (int)(i % G);
    unsigned t = i / G;
    const int wo = (int)(t % (unsigned)Wo);
    t /= (unsigned)Wo;
    const int ho = (int)(t % (unsigned)Ho);
    const int n = (int)(t / (unsigned)Ho);
    float m[8];
    int a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      a[j] = 0;
    }
    for (int r = 0; r < k; ++r) {
      const int hi = ho * st - pad + r;
      if (hi < 0 || hi >= H) continue;
      for (int c = 0; c < k; ++c) {
        const int wi = wo * st - pad + c;
        if (wi < 0 || wi >= W) continue;
        const bf16x8 v =
            *reinterpret_cast<const bf16x8*>(x + ((size_t)((n * H + hi) * W + wi)) * C + grp * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)v[j];
          if (f > m[j]) {
            m[j] = f;
            a[j] = r * k + c;
          }
        }
      }
    }
    bf16x8 r8;
    unsigned long long packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r8[j] = (bf16)m[j];
      packed |= (unsigned long long)(a[j] & 0xFF) << (8 * j);
    }
    *reinterpret_cast<bf16x8*>(y + (size_t)i * 8) = r8;
    if (idx) *reinterpret_cast<unsigned long long*>(idx + (size_t)i * 8) = packed;
  }
}

void maxpool_fwd(const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C, int Ho,
                 int Wo, int k, int stride, int pad, hipStream_t s) {
  const long total = (long)N * Ho * Wo * (C / 8);
  if (total >= (1L << 31) || (long)N * H * W * C >= (1L << 31))
    throw std::runtime_error("maxpool_fwd: tensor too large for 32-bit indexing");
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, y, idx, N, H,
                     W, C, Ho, Wo, k, stride, pad);
  DTR_CHECK_LAUNCH();
}

__global__ void maxpool_bwd_kernel(const uint8_t* __restrict__ idx, const bf16* __restrict__ dy,
                                   bf16* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                   int Wo, int k, int st, int pad) {
  const unsigned G = (unsigned)C / 8;
  const unsigned total = (unsigned)N * H * W * G;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const int grp = (int)(i % G);
    unsigned t = i / G;
    const int w = (int)(t % (unsigned)W);
    t /= (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // outputs whose window covers h: ho*st - pad <= h <= ho*st - pad + k - 1
    const int ho_lo = max(0, (h + pad - k + st) / st), ho_hi = min(Ho - 1, (h + pad) / st);
    const int wo_lo = max(0, (w + pad - k + st) / st), wo_hi = min(Wo - 1, (w + pad) / st);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int r = h - (ho * st - pad);
      if (r < 0 || r >= k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int c = w - (wo * st - pad);
        if (c < 0 || c >= k) continue;
        const size_t o = (size_t)((n * Ho + ho) * Wo + wo) * C + grp * 8;
        const unsigned long long a = *reinterpret_cast<const unsigned long long*>(idx + o);
        const bf16x8 d = *reinterpret_cast<const bf16x8*>(dy + o);
        const unsigned pos = (unsigned)(r * k + c);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((a >> (8 * j)) & 0xFF) == pos) acc[j] += (float)d[j];
      }
    }
    bf16x8 r8;
#pragma unroll
    for (int j = 0; j < 8; ++j) r8[j] = (bf16)acc[j];
    *reinterpret_cast<bf16x8*>(dx + (size_t)i * 8) = r8;
  }
}

void maxpool_bwd(const uint8_t* idx, const bf16* dy, bf16* dx, int N, int H, int W, int C, int Ho,
                 int Wo, int k, int stride, int pad, hipStream_t s) {
  const long total = (long)N * H * W * (C / 8);
  if (total >= (1L << 31) || (long)N * H * W * C >= (1L << 31))
    throw std::runtime_error("maxpool_bwd: tensor too large for 32-bit indexing");
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, idx, dy, dx, N,
                     H, W, C, Ho, Wo, k, stride, pad);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
