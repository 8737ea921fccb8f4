// Shared device helpers for the lumen_amd CDNA4 (gfx950) kernel library.
//
// Everything here is wave64 / MFMA-first: operand fragments are the
// v_mfma_f32_16x16x32_bf16 and v_mfma_f32_32x32x16_bf16 layouts, bf16 is
// moved in 16-byte vectors (8 elements per lane), and reductions are
// 64-lane shuffles.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LM_WAVE 64

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint16_t bf16_raw;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// 16-byte load with the non-temporal hint (global_load_dwordx4 ... nt): for weight bytes that ONE
// CU reads once per launch (decode GEMV streams).  The lines do not displace the L2 / MALL working
// set the next kernel wants (activations, KV) and land ~18 % sooner (MI355X_MICROARCH nt-weights).
__device__ __forceinline__ u32x4_t ld_nt16(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
}

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

// ---- OCP e4m3fn (fp8) <-> bf16 / f32 ---------------------------------------
// fp8 bytes 0,1 (lo) or 2,3 (hi) of a dword -> 2 bf16 packed in a dword
__device__ __forceinline__ uint32_t fp8x2_lo(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.0f, false));
}
__device__ __forceinline__ uint32_t fp8x2_hi(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.0f, true));
}
// 8 fp8 (two dwords) -> 8 bf16 (16 bytes)
__device__ __forceinline__ u32x4_t fp8x8_to_bf16(uint32_t w0, uint32_t w1) {
  return (u32x4_t){fp8x2_lo(w0), fp8x2_hi(w0), fp8x2_lo(w1), fp8x2_hi(w1)};
}
// one float -> one e4m3fn byte (saturated to +-448, round to nearest even)
__device__ __forceinline__ uint8_t f2fp8(float v) {
  v = fminf(fmaxf(v, -448.f), 448.f);
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
}

// ---- MX fp8 blocks (OCP microscaling): 32 e4m3fn values sharing one E8M0 exponent --------
// The producers of a W8A8 GEMM operand (GEMM epilogues, attention) quantise each 32-value
// block with its own power-of-two scale and the consumer feeds that byte straight into the
// scale operand of v_mfma_scale_f32_16x16x128_f8f6f4 (one byte per lane = per 32 k-values).
// mx_exp: the smallest e with amax / 2^e <= 448 (the E8M0 byte is e + 127), clamped so 2^-e
// stays a normal float; amax = 0 gives the smallest scale.
__device__ __forceinline__ int mx_exp(float amax) {
  const uint32_t b = __float_as_uint(amax * (1.f / 448.f));
  int e = (int)((b >> 23) & 0xff) - 127 + ((b & 0x7fffff) != 0);
  return min(max(e, -127), 126);
}
__device__ __forceinline__ float mx_inv(int e) { return __uint_as_float((uint32_t)(127 - e) << 23); }   // 2^-e
// 8 floats * inv -> 8 e4m3fn bytes, saturated to +-448
__device__ __forceinline__ uint2 fp8x8_scaled(const float* f, float inv) {
  float t[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) t[q] = fminf(fmaxf(f[q] * inv, -448.f), 448.f);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(t[0], t[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(t[2], t[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(t[4], t[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(t[6], t[7], hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
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

__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// erf via Abramowitz & Stegun 7.1.26 (|err| < 1.5e-7): one exp + one rcp,
// ~12 VALU instead of the ~40 of the libm erff.
__device__ __forceinline__ float fast_erf(float x) {
  const float ax = fabsf(x);
  const float t = fast_rcp(1.0f + 0.3275911f * ax);
  const float y = 1.0f - (((((1.061405429f * t - 1.453152027f) * t) + 1.421413741f) * t - 0.284496736f) * t +
                          0.254829592f) * t * __expf(-ax * ax);
  return copysignf(y, x);
}

template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if constexpr (ACT == ACT_GELU) return 0.5f * x * (1.0f + fast_erf(x * 0.70710678118654752f));
  else if constexpr (ACT == ACT_QUICK_GELU) return x * fast_rcp(1.0f + __expf(-1.702f * x));
  else if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.0f);
  else if constexpr (ACT == ACT_SILU) return x * fast_rcp(1.0f + __expf(-x));
  else if constexpr (ACT == ACT_GELU_TANH) {
    const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    // tanh(u) = 1 - 2 / (1 + e^{2u})
    return 0.5f * x * (2.0f - 2.0f * fast_rcp(1.0f + __expf(2.0f * u)));
  } else if constexpr (ACT == ACT_HARDSWISH) return x * fminf(fmaxf(x + 3.0f, 0.0f), 6.0f) * (1.0f / 6.0f);
  else if constexpr (ACT == ACT_SIGMOID) return fast_rcp(1.0f + __expf(-x));
  else if constexpr (ACT == ACT_LEAKY) return x > 0.0f ? x : 0.1f * x;
  else if constexpr (ACT == ACT_HARDSIGMOID) return fminf(fmaxf(x * (1.0f / 6.0f) + 0.5f, 0.0f), 1.0f);
  else return x;
}

// Apply an activation to N registers with ONE wave-uniform branch (never a
// per-element switch: if-converted, that evaluates every activation).
template <int N>
__device__ __forceinline__ void apply_act_n(float* v, int act) {
#define LM_ACT_CASE(A)                                 \
  case A:                                                 \
    _Pragma("unroll") for (int q = 0; q < N; ++q) v[q] = act_fn<A>(v[q]); \
    break;
  switch (act) {
    LM_ACT_CASE(ACT_GELU)
    LM_ACT_CASE(ACT_QUICK_GELU)
    LM_ACT_CASE(ACT_RELU)
    LM_ACT_CASE(ACT_SILU)
    LM_ACT_CASE(ACT_GELU_TANH)
    LM_ACT_CASE(ACT_HARDSWISH)
    LM_ACT_CASE(ACT_SIGMOID)
    LM_ACT_CASE(ACT_LEAKY)
    LM_ACT_CASE(ACT_HARDSIGMOID)
    default: break;
  }
#undef LM_ACT_CASE
}

__device__ __forceinline__ float apply_act(float x, int act) {
  float v[1] = {x};
  apply_act_n<1>(v, act);
  return v[0];
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
