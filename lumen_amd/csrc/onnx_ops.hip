// Generic-node kernels of the ONNX graph executor (runtime/onnx_graph.py) so the GPU path of
// the reference's face / OCR ONNX packs does not fall back to torch ops:
//
//   ew_binary     Add / Sub / Mul / Div / Pow / Max / Min with numpy broadcasting over up to
//                 6 dims (per-operand strides, 0 on broadcast dims), f32 / bf16 in, f32 / bf16 out
//   softmax_rows  softmax over the last axis, one wave per row (fp32 math)
//   resize_bilinear_nhwc  NHWC bilinear resize (half_pixel / align_corners / asymmetric /
//                 pytorch_half_pixel coordinate maps), 8 channels per thread
//   bmm           strided batched C[b] = A[b] . B[b] for activation x activation MatMuls
//                 (attention scores / context in SVTR blocks): 16x16 LDS tiles, fp32 accumulate
//
// Reference runtime being replaced: onnxruntime's CPU / CUDA EPs behind
// packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py:123-129 and
// packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py.
#include "common.h"

namespace lumen {

constexpr int EW_DIMS = 6;

struct EwArgs {
  const void* a;
  const void* b;
  void* out;
  int64_t shape[EW_DIMS];     // output shape (leading dims padded with 1)
  int64_t sa[EW_DIMS];        // element strides of a / b per output dim (0 = broadcast)
  int64_t sb[EW_DIMS];
  int64_t n;
  int op;                     // 0 add 1 sub 2 mul 3 div 4 pow 5 max 6 min
  int a_bf16, b_bf16, out_bf16;
};

__device__ __forceinline__ float ew_ld(const void* p, int64_t i, int bf) {
  return bf ? bf2f(((const uint16_t*)p)[i]) : ((const float*)p)[i];
}

__global__ void ew_binary_kernel(EwArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  int64_t r = i, ia = 0, ib = 0;
#pragma unroll
  for (int d = EW_DIMS - 1; d >= 0; --d) {
    const int64_t c = r % a.shape[d];
    r /= a.shape[d];
    ia += c * a.sa[d];
    ib += c * a.sb[d];
  }
  const float x = ew_ld(a.a, ia, a.a_bf16), y = ew_ld(a.b, ib, a.b_bf16);
  float v;
  switch (a.op) {
    case 0: v = x + y; break;
    case 1: v = x - y; break;
    case 2: v = x * y; break;
    case 3: v = x / y; break;
    case 4: v = powf(x, y); break;
    case 5: v = fmaxf(x, y); break;
    default: v = fminf(x, y);
  }
  if (a.out_bf16) ((uint16_t*)a.out)[i] = f2bf(v);
  else ((float*)a.out)[i] = v;
}

hipError_t ew_binary(const EwArgs& a, hipStream_t stream) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ew_binary_kernel, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// unary elementwise over a contiguous tensor: 0 relu 1 sigmoid 2 tanh 3 exp 4 log 5 sqrt 6 neg
// 7 abs 8 reciprocal 9 hardswish 10 hardsigmoid(p0 = alpha, p1 = beta) 11 leaky(p0) 12 clip(p0, p1)
// 13 floor 14 ceil 15 erf 16 identity (dtype conversion)
__global__ void ew_unary_kernel(const void* __restrict__ x, int x_bf16, void* __restrict__ out, int out_bf16,
                                int64_t n, int op, float p0, float p1) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = ew_ld(x, i, x_bf16);
  float y;
  switch (op) {
    case 0: y = fmaxf(v, 0.f); break;
    case 1: y = 1.f / (1.f + __expf(-v)); break;
    case 2: y = tanhf(v); break;
    case 3: y = __expf(v); break;
    case 4: y = __logf(v); break;
    case 5: y = sqrtf(v); break;
    case 6: y = -v; break;
    case 7: y = fabsf(v); break;
    case 8: y = 1.f / v; break;
    case 9: y = v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f); break;
    case 10: y = fminf(fmaxf(v * p0 + p1, 0.f), 1.f); break;
    case 11: y = v > 0.f ? v : v * p0; break;
    case 12: y = fminf(fmaxf(v, p0), p1); break;
    case 13: y = floorf(v); break;
    case 14: y = ceilf(v); break;
    case 15: y = erff(v); break;
    default: y = v;
  }
  if (out_bf16) ((uint16_t*)out)[i] = f2bf(y);
  else ((float*)out)[i] = y;
}

hipError_t ew_unary(const void* x, int x_bf16, void* out, int out_bf16, int64_t n, int op, float p0, float p1,
                    hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ew_unary_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, x_bf16, out,
                     out_bf16, n, op, p0, p1);
  return hipGetLastError();
}

// softmax over rows of length D (contiguous), one wave per row
__global__ void __launch_bounds__(256) softmax_rows_kernel(const void* __restrict__ x, int x_bf16,
                                                           void* __restrict__ out, int out_bf16, int64_t rows, int D) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t base = row * D;
  float m = -INFINITY;
  for (int j = lane; j < D; j += 64) m = fmaxf(m, ew_ld(x, base + j, x_bf16));
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < D; j += 64) s += __expf(ew_ld(x, base + j, x_bf16) - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < D; j += 64) {
    const float v = __expf(ew_ld(x, base + j, x_bf16) - m) * inv;
    if (out_bf16) ((uint16_t*)out)[base + j] = f2bf(v);
    else ((float*)out)[base + j] = v;
  }
}

hipError_t softmax_rows(const void* x, int x_bf16, void* out, int out_bf16, int64_t rows, int D, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, x, x_bf16, out,
                     out_bf16, rows, D);
  return hipGetLastError();
}

// NHWC bf16 bilinear resize; C % 8 == 0, 8 channels per thread.  mode: 0 half_pixel,
// 1 align_corners, 2 asymmetric, 3 pytorch_half_pixel
__global__ void resize_bilinear_nhwc_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out, int N, int H,
                                            int W, int C, int Ho, int Wo, int mode) {
  const int cg = C / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)N * Ho * Wo * cg;
  if (i >= total) return;
  const int g = (int)(i % cg);
  int64_t r = i / cg;
  const int ox = (int)(r % Wo);
  r /= Wo;
  const int oy = (int)(r % Ho);
  const int n = (int)(r / Ho);
  auto src = [&](int o, int osz, int isz) -> float {
    const float s = (float)isz / (float)osz;
    switch (mode) {
      case 1: return osz > 1 ? o * (float)(isz - 1) / (float)(osz - 1) : 0.f;
      case 2: return o * s;
      case 3: return osz > 1 ? (o + 0.5f) * s - 0.5f : 0.f;
      default: return (o + 0.5f) * s - 0.5f;
    }
  };
  float fy = fminf(fmaxf(src(oy, Ho, H), 0.f), (float)(H - 1));
  float fx = fminf(fmaxf(src(ox, Wo, W), 0.f), (float)(W - 1));
  const int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
  const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
  const float wy = fy - y0, wx = fx - x0;
  const uint16_t* b = x + (int64_t)n * H * W * C + g * 8;
  float p00[8], p01[8], p10[8], p11[8];
  unpack8(*(const u32x4_t*)(b + ((int64_t)y0 * W + x0) * C), p00);
  unpack8(*(const u32x4_t*)(b + ((int64_t)y0 * W + x1) * C), p01);
  unpack8(*(const u32x4_t*)(b + ((int64_t)y1 * W + x0) * C), p10);
  unpack8(*(const u32x4_t*)(b + ((int64_t)y1 * W + x1) * C), p11);
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    v[q] = (p00[q] * (1.f - wx) + p01[q] * wx) * (1.f - wy) + (p10[q] * (1.f - wx) + p11[q] * wx) * wy;
  *(u32x4_t*)(out + (((int64_t)n * Ho + oy) * Wo + ox) * C + g * 8) = pack8(v);
}

hipError_t resize_bilinear_nhwc(const uint16_t* x, uint16_t* out, int N, int H, int W, int C, int Ho, int Wo, int mode,
                                hipStream_t stream) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(resize_bilinear_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, out,
                     N, H, W, C, Ho, Wo, mode);
  return hipGetLastError();
}

// C[b] (M x N, f32) = A[b] (M x K) . B[b] (K x N); element strides (batch, row, col) per operand;
// 16 x 16 output tiles through LDS, fp32 accumulation
struct BmmArgs {
  const void* a;
  const void* b;
  float* c;
  int64_t sab, sam, sak, sbb, sbk, sbn, scb, scm, scn;
  int B, M, N, K, a_bf16, b_bf16;
};

__global__ void __launch_bounds__(256) bmm_kernel(BmmArgs p) {
  __shared__ float ta[16][17], tb[16][17];
  const int bz = blockIdx.z;
  const int m = blockIdx.y * 16 + (threadIdx.x >> 4), n = blockIdx.x * 16 + (threadIdx.x & 15);
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  float acc = 0.f;
  for (int k0 = 0; k0 < p.K; k0 += 16) {
    const int ka = k0 + tx, kb = k0 + ty;
    const int am = blockIdx.y * 16 + ty, bn = blockIdx.x * 16 + tx;
    ta[ty][tx] = (am < p.M && ka < p.K) ? ew_ld(p.a, bz * p.sab + am * p.sam + ka * p.sak, p.a_bf16) : 0.f;
    tb[ty][tx] = (kb < p.K && bn < p.N) ? ew_ld(p.b, bz * p.sbb + kb * p.sbk + bn * p.sbn, p.b_bf16) : 0.f;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += ta[ty][k] * tb[k][tx];
    __syncthreads();
  }
  if (m < p.M && n < p.N) p.c[bz * p.scb + m * p.scm + n * p.scn] = acc;
}

hipError_t bmm(const BmmArgs& p, hipStream_t stream) {
  if (p.B <= 0 || p.M <= 0 || p.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(bmm_kernel, dim3((p.N + 15) / 16, (p.M + 15) / 16, p.B), dim3(256), 0, stream, p);
  return hipGetLastError();
}

}  // namespace lumen
