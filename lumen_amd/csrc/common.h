// Shared device helpers for the lumen_amd CDNA4 (gfx950) kernel library.
//
// Everything here is wave64 / MFMA-first: operand fragments are the
// v_mfma_f32_16x16x32_bf16 and v_mfma_f32_32x32x16_bf16 layouts, bf16 is
// moved in 16-byte vectors (8 elements per lane), and reductions are
// 64-lane shuffles.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LUMEN_WAVE 64

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint16_t bf16_raw;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

namespace lumen {

// Compile-time unrolled loop: f(I) for I in [B, E) with I a literal after
// inlining (keeps register-array indices static so arrays never hit scratch).
template <int B, int E>
struct Unroll {
  template <typename F>
  __device__ __forceinline__ static void run(F&& f) {
    f(B);
    Unroll<B + 1, E>::run(f);
  }
};
template <int E>
struct Unroll<E, E> {
  template <typename F>
  __device__ __forceinline__ static void run(F&&) {}
};

// ---- bf16 <-> f32 -------------------------------------------------------
__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even; lets hipcc emit v_cvt_pk_bf16_f32 where it can.
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 16-byte vector of 8 bf16 <-> 8 floats
__device__ __forceinline__ void unpack8(const u32x4_t v, float* f) {
  f[0] = __uint_as_float(v[0] << 16); f[1] = __uint_as_float(v[0] & 0xffff0000u);
  f[2] = __uint_as_float(v[1] << 16); f[3] = __uint_as_float(v[1] & 0xffff0000u);
  f[4] = __uint_as_float(v[2] << 16); f[5] = __uint_as_float(v[2] & 0xffff0000u);
  f[6] = __uint_as_float(v[3] << 16); f[7] = __uint_as_float(v[3] & 0xffff0000u);
}
__device__ __forceinline__ u32x4_t pack8(const float* f) {
  u32x4_t v;
  v[0] = pack2bf(f[0], f[1]); v[1] = pack2bf(f[2], f[3]);
  v[2] = pack2bf(f[4], f[5]); v[3] = pack2bf(f[6], f[7]);
  return v;
}

// ---- wave reductions (64 lanes) -----------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- activations ---------------------------------------------------------
enum Act : int { ACT_NONE = 0, ACT_GELU = 1, ACT_QUICK_GELU = 2, ACT_RELU = 3,
                 ACT_SILU = 4, ACT_GELU_TANH = 5, ACT_HARDSWISH = 6, ACT_SIGMOID = 7,
                 ACT_LEAKY = 8 /* slope 0.1 */, ACT_HARDSIGMOID = 9 };

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case ACT_GELU: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
    case ACT_QUICK_GELU: return x / (1.0f + __expf(-1.702f * x));
    case ACT_RELU: return fmaxf(x, 0.0f);
    case ACT_SILU: return x / (1.0f + __expf(-x));
    case ACT_GELU_TANH: {
      float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.0f + tanhf(u));
    }
    case ACT_HARDSWISH: return x * fminf(fmaxf(x + 3.0f, 0.0f), 6.0f) * (1.0f / 6.0f);
    case ACT_SIGMOID: return 1.0f / (1.0f + __expf(-x));
    case ACT_LEAKY: return x > 0.0f ? x : 0.1f * x;
    case ACT_HARDSIGMOID: return fminf(fmaxf(x * (1.0f / 6.0f) + 0.5f, 0.0f), 1.0f);
    default: return x;
  }
}

// Bijective XCD-aware remap of a flat workgroup id: blocks b and b+8 share an
// XCD (round-robin dealing), so give each XCD group a contiguous run of
// logical tiles (cdna guide T1, bijective form for nwg % 8 != 0).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8, idx = orig / 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace lumen
