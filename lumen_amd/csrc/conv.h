// Host-visible declarations of the convolution / CNN-support kernels (conv.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lumen {

struct GemmEpi;

struct ConvArgs {
  const uint16_t* x;   // NHWC [N, H, W, Cin] (pixel stride ldx >= Cin)
  const uint16_t* w;   // [Cout, KH, KW, Cin]
  void* out;           // NHWC [N, Ho, Wo, *] pixel stride ldo
  int64_t ldx, ldo;
  int N, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo;
};

hipError_t conv2d_igemm(const ConvArgs& a, const GemmEpi& ep, int tile, hipStream_t stream);
hipError_t conv2d_depthwise(const uint16_t* x, const uint16_t* w, const void* bias, int bias_f32, void* out,
                            int N, int H, int W, int C, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw,
                            int Ho, int Wo, int act, int out_f32, hipStream_t stream);
hipError_t channel_affine(const uint16_t* x, const float* scale, const float* shift, uint16_t* out, int64_t rows,
                          int C, int act, const uint16_t* prelu, hipStream_t stream);
hipError_t pool2d(const uint16_t* x, uint16_t* out, int N, int H, int W, int C, int KH, int KW, int sh, int sw,
                  int ph, int pw, int Ho, int Wo, int is_max, hipStream_t stream);
hipError_t global_avgpool(const uint16_t* x, float* out, int N, int HW, int C, hipStream_t stream);
hipError_t upsample_add(const uint16_t* x, const uint16_t* add, uint16_t* out, int N, int H, int W, int C, int f,
                        int64_t ldo, hipStream_t stream);
hipError_t channel_scale(uint16_t* x, const float* s, int N, int HW, int C, hipStream_t stream);
hipError_t pixel_shuffle_up(const uint16_t* y, uint16_t* out, int N, int H, int W, int C, int f, hipStream_t stream);

}  // namespace lumen
