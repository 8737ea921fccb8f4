// Host-visible declarations of the convolution / CNN-support kernels (conv.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lumen {

struct GemmEpi;

// Unsigned 32-bit division by a run-time constant as a multiply-high (round-up method, Hacker's Delight
// 10-8): q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(n, mul), l = ceil(log2 d); d = 1: shift -1.
// The conv kernels' per-row pixel decomposition (m -> image, row, column) ran two ~40-instruction
// integer divisions per staged row: on the small-Cin stems that prologue VALU was most of the kernel.
struct FastDiv {
  uint32_t mul;
  int shift;
};
inline FastDiv make_fastdiv(uint32_t d) {
  if (d <= 1) return FastDiv{0u, -1};
  int l = 0;
  while ((1ull << l) < d) ++l;
  return FastDiv{(uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1), l};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
  if (f.shift < 0) return n;
  const uint32_t t = __umulhi(n, f.mul);
  return (t + ((n - t) >> 1)) >> (f.shift - 1);
}

struct ConvArgs {
  const uint16_t* x;   // NHWC [N, H, W, Cin] (pixel stride ldx >= Cin)
  const uint16_t* w;   // [Cout, KH, KW, Cin]
  void* out;           // NHWC [N, Ho, Wo, *] pixel stride ldo
  int64_t ldx, ldo;
  int N, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo;
  FastDiv div_hw, div_w, div_kw;   // by Ho * Wo, by Wo and by KW (filled by conv2d_igemm)
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
hipError_t db_head_up(const uint16_t* h, const uint16_t* w1, const float* b1, const uint16_t* w2p, const float* b2,
                      float* out, int N, int H4, int W4, int C, hipStream_t stream);

}  // namespace lumen
