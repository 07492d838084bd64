// On-device input pipeline pieces.
//
// cifar_augment reproduces the reference CIFAR training preprocessing
// (resnet_cifar_main.py:201-216: pad to 40x40, random 32x32 crop, random
// left-right flip, tf.image.per_image_standardization) and the eval path
// (cifar_input.py:71-76: standardization only) on raw CIFAR-binary uint8 images
// ([N][3][32][32], the record layout of resnet_cifar_main.py:173-198), writing
// bf16 NHWC with the channel dim zero-padded to Cpad (the stem conv consumes 8
// channels so every 16-B fragment is one tap).  Crop/flip randomness comes from
// a counter-based hash of (seed, global_step, image) read on the device, so the
// augmentation is part of the captured hipGraph and replays with fresh crops.
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "data.h"

namespace dtr {

__device__ __forceinline__ unsigned long long splitmix(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// One workgroup per image: the 3 KB record is staged in LDS with 16-B loads, every
// thread keeps its 4 output pixels' 3 channels in registers across the
// per-image statistics, and writes each pixel as ONE 16-B NHWC row (3 channels +
// zero padding).  Optionally zeroes a buffer in the same launch (the step's
// BatchNorm accumulators), so the step needs no separate memset.
template <int CPAD>
__global__ void __launch_bounds__(256)
cifar_augment_kernel(const uint8_t* __restrict__ img, bf16* __restrict__ out, int pad,
                     unsigned long long seed, const long long* gstep, int train, int* crop_log,
                     uint4* __restrict__ zero, long zero_vec) {
  constexpr int H = 32, W = 32, HW = H * W, CHW = 3 * HW, PPT = HW / 256;
  __shared__ __attribute__((aligned(16))) uint8_t im[CHW];
  __shared__ float red[8];
  const int n = blockIdx.x, tid = threadIdx.x;
  for (long i = blockIdx.x * 256L + tid; i < zero_vec; i += (long)gridDim.x * 256)
    zero[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < CHW / 16)
    reinterpret_cast<uint4*>(im)[tid] = reinterpret_cast<const uint4*>(img + (long)n * CHW)[tid];
  int oy = pad, ox = pad, flip = 0;
  if (train) {
    const unsigned long long step = gstep ? (unsigned long long)*gstep : 0ull;
    const unsigned long long h = splitmix(seed ^ splitmix(step * 0x100000001B3ull + n));
    oy = (int)(h % (2 * pad + 1));
    ox = (int)((h >> 16) % (2 * pad + 1));
    flip = (int)((h >> 32) & 1);
  }
  if (crop_log && tid == 0) {
    crop_log[n * 3 + 0] = oy;
    crop_log[n * 3 + 1] = ox;
    crop_log[n * 3 + 2] = flip;
  }
  __syncthreads();
  // pixel (y,x) of the crop = padded-image pixel (y+oy, x'+ox), x' = flip ? W-1-x : x
  float v[PPT][3];
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int p = tid + k * 256;
    const int y = p / W, x = p - y * W;
    const int xs = flip ? (W - 1 - x) : x;
    const int py = y + oy - pad, px = xs + ox - pad;
    const bool in = py >= 0 && py < H && px >= 0 && px < W;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      v[k][c] = in ? (float)im[c * HW + py * W + px] : 0.f;
      s += v[k][c];
      q += v[k][c] * v[k][c];
    }
  }
  s = wave_sum(s);
  q = wave_sum(q);
  if ((tid & 63) == 0) {
    red[tid >> 6] = s;
    red[4 + (tid >> 6)] = q;
  }
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float totq = red[4] + red[5] + red[6] + red[7];
  const float nel = (float)CHW;
  const float mean = tot / nel;
  const float var = fmaxf(totq / nel - mean * mean, 0.f);
  const float adj = fmaxf(sqrtf(var), rsqrtf(nel));
  const float inv = 1.f / adj;
  bf16* o = out + (long)n * HW * CPAD;
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int p = tid + k * 256;
    bf16x8 r = {};
#pragma unroll
    for (int c = 0; c < 3; ++c) r[c] = (bf16)((v[k][c] - mean) * inv);
    *reinterpret_cast<bf16x8*>(o + (long)p * CPAD) = r;
  }
}

// Generic-shape fallback (any H, W, Cpad): one element per thread iteration.
__global__ void __launch_bounds__(256)
cifar_augment_generic_kernel(const uint8_t* __restrict__ img, bf16* __restrict__ out, int H,
                             int W, int Cpad, int pad, unsigned long long seed,
                             const long long* gstep, int train, int* crop_log,
                             uint4* __restrict__ zero, long zero_vec) {
  __shared__ float red[8];
  const int n = blockIdx.x, tid = threadIdx.x;
  for (long i = blockIdx.x * 256L + tid; i < zero_vec; i += (long)gridDim.x * 256)
    zero[i] = make_uint4(0u, 0u, 0u, 0u);
  const int HW = H * W, CHW = 3 * HW;
  const uint8_t* src = img + (long)n * CHW;
  int oy = pad, ox = pad, flip = 0;
  if (train) {
    const unsigned long long step = gstep ? (unsigned long long)*gstep : 0ull;
    const unsigned long long h = splitmix(seed ^ splitmix(step * 0x100000001B3ull + n));
    oy = (int)(h % (2 * pad + 1));
    ox = (int)((h >> 16) % (2 * pad + 1));
    flip = (int)((h >> 32) & 1);
  }
  if (crop_log && tid == 0) {
    crop_log[n * 3 + 0] = oy;
    crop_log[n * 3 + 1] = ox;
    crop_log[n * 3 + 2] = flip;
  }
  auto val = [&](int p, int c) -> float {
    const int y = p / W, x = p - y * W;
    const int xs = flip ? (W - 1 - x) : x;
    const int py = y + oy - pad, px = xs + ox - pad;
    if (py < 0 || py >= H || px < 0 || px >= W) return 0.f;
    return (float)src[c * HW + py * W + px];
  };
  float s = 0.f, q = 0.f;
  for (int i = tid; i < CHW; i += 256) {
    const float v = val(i / 3, i % 3);
    s += v;
    q += v * v;
  }
  s = wave_sum(s);
  q = wave_sum(q);
  if ((tid & 63) == 0) {
    red[tid >> 6] = s;
    red[4 + (tid >> 6)] = q;
  }
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float totq = red[4] + red[5] + red[6] + red[7];
  const float nel = (float)CHW;
  const float mean = tot / nel;
  const float var = fmaxf(totq / nel - mean * mean, 0.f);
  const float adj = fmaxf(sqrtf(var), rsqrtf(nel));
  const float inv = 1.f / adj;
  bf16* o = out + (long)n * HW * Cpad;
  for (int i = tid; i < HW * Cpad; i += 256) {
    const int p = i / Cpad, c = i - p * Cpad;
    o[i] = (bf16)(c < 3 ? (val(p, c) - mean) * inv : 0.f);
  }
}

void cifar_augment(const uint8_t* img, bf16* out, int N, int H, int W, int Cpad, int pad,
                   unsigned long long seed, const long long* gstep, int train, int* crop_log,
                   void* zero, long zero_bytes, hipStream_t s) {
  if (zero_bytes % 16) throw std::invalid_argument("cifar_augment: zero_bytes % 16 != 0");
  uint4* z = reinterpret_cast<uint4*>(zero);
  const long zv = zero ? zero_bytes / 16 : 0;
  if (H == 32 && W == 32 && Cpad == 8)
    hipLaunchKernelGGL(cifar_augment_kernel<8>, dim3(N), dim3(256), 0, s, img, out, pad, seed,
                       gstep, train, crop_log, z, zv);
  else
    hipLaunchKernelGGL(cifar_augment_generic_kernel, dim3(N), dim3(256), 0, s, img, out, H, W,
                       Cpad, pad, seed, gstep, train, crop_log, z, zv);
  DTR_CHECK_LAUNCH();
}

__global__ void pad_channels_kernel(const float* __restrict__ x, bf16* __restrict__ out, long npix,
                                    int C, int Cpad) {
  const long total = npix * Cpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / Cpad;
    const int c = (int)(i - p * Cpad);
    out[i] = (bf16)(c < C ? x[p * C + c] : 0.f);
  }
}

void nhwc_pad_channels(const float* x, bf16* out, long npix, int C, int Cpad, hipStream_t s) {
  long blocks = (npix * Cpad + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pad_channels_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, out, npix,
                     C, Cpad);
  DTR_CHECK_LAUNCH();
}

// Gaussian-ish synthetic activations (sum of 4 uniforms, unit variance) in
// NHWC with the padded channels kept zero.
__global__ void synth_kernel(bf16* out, long npix, int C, int Cpad, unsigned long long seed) {
  const long total = npix * Cpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cpad);
    float v = 0.f;
    if (c < C) {
      const unsigned long long h = splitmix(seed + (unsigned long long)i);
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += (float)((h >> (16 * k)) & 0xFFFF) * (1.f / 65535.f);
      v = (s - 2.f) * 1.7320508f;
    }
    out[i] = (bf16)v;
  }
}

void synthetic_images(bf16* out, long npix, int C, int Cpad, unsigned long long seed,
                      hipStream_t s) {
  long blocks = (npix * Cpad + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, npix, C, Cpad,
                     seed);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr

namespace dtr {

// ImageNet real-data feed (resnet_imagenet_main.py:122-192 with VGG preprocessing,
// vgg_preprocessing.py:284-333): CPU workers decode the JPEG, do the
// aspect-preserving resize and the random (train) / central (eval) 224x224 crop
// and ship the crop as uint8 HWC -- 4x fewer host->device bytes than float32.
// This kernel does the rest on the device: the random left-right flip (hash of
// (seed, global_step, image), like cifar_augment), the per-channel mean
// subtraction (R,G,B = 123.68, 116.78, 103.94, vgg_preprocessing.py:37-39) and the
// bf16 NHWC packing with the channel dim padded to 8 (one 16-B row per pixel,
// the stem conv's operand layout).  Optionally clears a buffer in the same launch
// (the step's BatchNorm accumulators).  One thread per output pixel.
__global__ void __launch_bounds__(256)
imagenet_u8_pack_kernel(const uint8_t* __restrict__ img, bf16* __restrict__ out, int H, int W,
                        unsigned long long seed, const long long* gstep, int train,
                        uint4* __restrict__ zero, long zero_vec, long npix, int s2d) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < zero_vec; i += (long)gridDim.x * 256)
    zero[i] = make_uint4(0u, 0u, 0u, 0u);
  const long p = blockIdx.x * 256L + threadIdx.x;
  if (p >= npix) return;
  const long HW = (long)H * W;
  const long n = p / HW;
  const int rem = (int)(p - n * HW);
  const int y = rem / W, x = rem - y * W;
  int flip = 0;
  if (train) {
    const unsigned long long step = gstep ? (unsigned long long)*gstep : 0ull;
    flip = (int)((splitmix(seed ^ splitmix(step * 0x100000001B3ull + (unsigned long long)n)) >> 32) & 1);
  }
  const int xs = flip ? W - 1 - x : x;
  const uint8_t* src = img + ((n * H + y) * (long)W + xs) * 3;
  const bf16 c0 = (bf16)((float)src[0] - 123.68f);
  const bf16 c1 = (bf16)((float)src[1] - 116.78f);
  const bf16 c2 = (bf16)((float)src[2] - 103.94f);
  if (s2d) {   // space-to-depth stem operand [N][H/2][W/2][16] (stem_s2d_pack below)
    bf16x4 r = {c0, c1, c2, (bf16)0.f};
    const long q = (n * (H >> 1) + (y >> 1)) * (long)(W >> 1) + (x >> 1);
    *reinterpret_cast<bf16x4*>(out + q * 16 + ((y & 1) * 2 + (x & 1)) * 4) = r;
    return;
  }
  bf16x8 r = {};
  r[0] = c0;
  r[1] = c1;
  r[2] = c2;
  *reinterpret_cast<bf16x8*>(out + p * 8) = r;
}

void imagenet_u8_pack(const uint8_t* img, bf16* out, int N, int H, int W,
                      unsigned long long seed, const long long* gstep, int train, void* zero,
                      long zero_bytes, int s2d, hipStream_t s) {
  if (zero_bytes % 16 != 0) throw std::invalid_argument("imagenet_u8_pack: zero_bytes % 16");
  if (s2d && ((H | W) & 1)) throw std::invalid_argument("imagenet_u8_pack: s2d needs even H, W");
  const long npix = (long)N * H * W;
  const int grid = (int)((npix + 255) / 256);
  hipLaunchKernelGGL(imagenet_u8_pack_kernel, dim3(grid), dim3(256), 0, s, img, out, H, W, seed,
                     gstep, train, reinterpret_cast<uint4*>(zero), zero ? zero_bytes / 16 : 0,
                     npix, s2d);
  DTR_CHECK_LAUNCH();
}

// Space-to-depth ImageNet stem.  The 7x7 / stride-2 conv (TF fixed padding 3) over
// a 224x224x3 image equals a 4x4 / stride-1 conv (padding 2 before, 1 after) over
// the 112x112x16 space-to-depth image S[q][p][(rh*2 + rw)*4 + c] = X[2q+rh][2p+rw][c]
// (c = 3 zero): out(o) = sum_th S(o - 2 + th) reads rows 2o - 4 + 2th + rh, i.e.
// tap kh = 2th + rh - 1 of the 7x7 filter (kh = -1 is a zero row).  K = 4*4*16 = 256
// instead of 7*7*8 = 392 (57 % of the MACs real instead of 37 %), stride-1 gathers of
// 32-B pixel rows, and a weight gradient of 256 columns (two 128-wide tiles instead of
// four, the last 94 % empty).  The fp32 master weight stays the 7x7x3 HWIO of the
// checkpoint; these two kernels map it to the bf16 4x4x16 OHWI operand and the 4x4x16
// HWIO weight gradient back.
__global__ void stem_s2d_pack_kernel(const float* __restrict__ w7, bf16* __restrict__ w4, int K) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // [K][4][4][16]
  if (i >= K * 256) return;
  const int o = i >> 8, r = i & 255;
  const int th = r >> 6, tw = (r >> 4) & 3, ch = r & 15;
  const int kh = 2 * th + (ch >> 3) - 1, kw = 2 * tw + ((ch >> 2) & 1) - 1, c = ch & 3;
  float v = 0.f;
  if (c < 3 && kh >= 0 && kh < 7 && kw >= 0 && kw < 7) v = w7[((kh * 7 + kw) * 3 + c) * K + o];
  w4[i] = (bf16)v;
}

__global__ void stem_s2d_grad_kernel(const float* __restrict__ g4, float* __restrict__ g7, int K) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // [7][7][3][K]
  if (i >= 147 * K) return;
  const int o = i % K, t = i / K;
  const int c = t % 3, tap = t / 3;
  const int kh = tap / 7 + 1, kw = tap % 7 + 1;   // +1: row / column of the 8x8 grid
  const int ch = ((kh & 1) * 2 + (kw & 1)) * 4 + c;
  g7[i] = g4[(((kh >> 1) * 4 + (kw >> 1)) * 16 + ch) * K + o];
}

void stem_s2d_pack(const float* w7, bf16* w4, int K, hipStream_t s) {
  hipLaunchKernelGGL(stem_s2d_pack_kernel, dim3(K), dim3(256), 0, s, w7, w4, K);
  DTR_CHECK_LAUNCH();
}

void stem_s2d_grad(const float* g4, float* g7, int K, hipStream_t s) {
  hipLaunchKernelGGL(stem_s2d_grad_kernel, dim3((147 * K + 255) / 256), dim3(256), 0, s, g4, g7, K);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
