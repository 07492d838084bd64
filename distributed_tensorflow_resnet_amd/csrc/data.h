// On-device input-pipeline declarations (see data.hip).
#pragma once
#include "kernels.h"

namespace dtr {

void cifar_augment(const uint8_t* img, bf16* out, int N, int H, int W, int Cpad, int pad,
                   unsigned long long seed, const long long* gstep, int train, int* crop_log,
                   void* zero, long zero_bytes, hipStream_t s);   // zero: optional buffer to clear
void imagenet_u8_pack(const uint8_t* img, bf16* out, int N, int H, int W,
                      unsigned long long seed, const long long* gstep, int train, void* zero,
                      long zero_bytes, int s2d,
                      hipStream_t s);   // uint8 HWC crops -> bf16 NHWC-8 (s2d: [N][H/2][W/2][16])
// space-to-depth stem: 7x7x3xK fp32 HWIO master -> bf16 [K][4][4][16]; 4x4x16xK fp32
// HWIO gradient -> 7x7x3xK (data.hip)
void stem_s2d_pack(const float* w7, bf16* w4, int K, hipStream_t s);
void stem_s2d_grad(const float* g4, float* g7, int K, hipStream_t s);
void nhwc_pad_channels(const float* x, bf16* out, long npix, int C, int Cpad, hipStream_t s);
void synthetic_images(bf16* out, long npix, int C, int Cpad, unsigned long long seed,
                      hipStream_t s);

}  // namespace dtr
