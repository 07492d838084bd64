// Optimizer and flat-parameter plumbing.
//
// Replaces TF's ApplyMomentum x152 + L2Loss x152 + AddN + AssignAdd(global_step)
// (resnet_model.py:85-99,120-122):
//   g'    = grad * grad_scale + wd * w          (d/dw of wd * sum 1/2 ||w||^2)
//   accum = momentum * accum + g'                (tf.train.MomentumOptimizer, non-Nesterov)
//   w    -= lr * accum
// in ONE launch over the flat fp32 master buffer, which also re-packs every conv
// kernel into the two bf16 layouts the MFMA kernels consume ([K][kh][kw][C] for
// forward, HWIO for dgrad).  The learning rate is evaluated on the device from
// the device-resident global_step with the reference's piecewise schedule
// (resnet_cifar_main.py:304-324, resnet_imagenet_main.py:306-329 incl. the
// step-0 quirk), so the whole training step can be captured in a hipGraph.
#include "common.h"
#include "kernels.h"
#include "optim.h"

namespace dtr {

__device__ __forceinline__ float lr_at(const LrSchedule& s, long step) {
  // The reference's hook feeds the rate computed after the *previous* run:
  // step 0 uses the initial value from begin(); step t>0 uses f(t-1).
  if (step <= 0) return s.init;
  const long t = step - 1;
  if (t < s.warm_steps) return s.warm_from + (s.warm_to - s.warm_from) * (float)t / (float)s.warm_steps;
  for (int i = 0; i < s.nb; ++i)
    if (t < s.bound[i]) return s.val[i];
  return s.val[s.nb];
}

__device__ __forceinline__ int find_seg(const ParamSeg* segs, int nseg, long e) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].offset <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void write_copies(const ParamSeg& sg, long e, float w, bf16* bf) {
  if (sg.bf_ohwi < 0 && sg.bf_hwio < 0) return;
  const long local = e - sg.offset;
  const int CK = sg.C * sg.K;
  const int tap = (int)(local / CK);
  const int rem = (int)(local - (long)tap * CK);
  const int ci = rem / sg.K, co = rem - ci * sg.K;
  const int taps = sg.kh * sg.kw;
  const bf16 v = (bf16)w;
  if (sg.bf_ohwi >= 0) bf[sg.bf_ohwi + ((long)co * taps + tap) * sg.cpad + ci] = v;
  if (sg.bf_hwio >= 0) bf[sg.bf_hwio + ((long)tap * sg.C + ci) * sg.kpad + co] = v;
}

__global__ void __launch_bounds__(256)
sgd_pack_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ mom,
                long n, LrSchedule sched, const long long* __restrict__ gstep, float momentum,
                float wd, float grad_scale, int use_momentum, const ParamSeg* __restrict__ segs,
                int nseg, bf16* __restrict__ bf, float* __restrict__ lr_out, int update) {
  const float lr = update ? lr_at(sched, gstep ? (long)*gstep : 0L) : 0.f;
  if (update && lr_out && blockIdx.x == 0 && threadIdx.x == 0) *lr_out = lr;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n;
       e += (long)gridDim.x * blockDim.x) {
    float wv = w[e];
    if (update) {
      const float gv = g[e] * grad_scale + wd * wv;
      if (use_momentum) {
        const float a = momentum * mom[e] + gv;
        mom[e] = a;
        wv -= lr * a;
      } else {
        wv -= lr * gv;
      }
      w[e] = wv;
    }
    if (bf) write_copies(segs[find_seg(segs, nseg, e)], e, wv, bf);
  }
}

void sgd_update_pack(float* master, const float* grad, float* mom, long n, const LrSchedule& s,
                     const long long* gstep, float momentum, float wd, float grad_scale,
                     int use_momentum, const ParamSeg* segs, int nseg, bf16* bf, float* lr_out,
                     int update, hipStream_t st) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sgd_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, st, master, grad, mom,
                     n, s, gstep, momentum, wd, grad_scale, use_momentum, segs, nseg, bf, lr_out,
                     update);
  DTR_CHECK_LAUNCH();
}

__global__ void step_incr_kernel(long long* gstep) {
  if (threadIdx.x == 0) *gstep += 1;
}
void step_increment(long long* gstep, hipStream_t s) {
  hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(64), 0, s, gstep);
  DTR_CHECK_LAUNCH();
}

// 1/2 * sum v^2 -- two-stage, fixed order (deterministic).
__global__ void __launch_bounds__(256) l2_part_kernel(const float* __restrict__ v, long n,
                                                      float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    s += v[i] * v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void __launch_bounds__(256) l2_final_kernel(const float* __restrict__ part, int np,
                                                       float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = 0.5f * (red[0] + red[1] + red[2] + red[3]);
}

static constexpr int L2_BLOCKS = 512;
int l2_workspace_floats() { return L2_BLOCKS; }

void l2_half_sum(const float* v, long n, float* ws, float* out, hipStream_t s) {
  hipLaunchKernelGGL(l2_part_kernel, dim3(L2_BLOCKS), dim3(256), 0, s, v, n, ws);
  hipLaunchKernelGGL(l2_final_kernel, dim3(1), dim3(256), 0, s, ws, L2_BLOCKS, out);
  DTR_CHECK_LAUNCH();
}

__global__ void fill_kernel(float* p, long n, float a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    p[i] = a;
}
void fill_f32(float* p, long n, float a, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, n, a);
  DTR_CHECK_LAUNCH();
}

__global__ void cast_f2b_kernel(const float* a, bf16* b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    b[i] = (bf16)a[i];
}
__global__ void cast_b2f_kernel(const bf16* a, float* b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    b[i] = (float)a[i];
}
void cast_f32_bf16(const float* a, bf16* b, long n, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cast_f2b_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, n);
  DTR_CHECK_LAUNCH();
}
void cast_bf16_f32(const bf16* a, float* b, long n, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cast_b2f_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, n);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
