// Shared GEMM epilogue (bias / activation / periodic table / residual / row
// remap / bf16-or-f32 store of 16 consecutive columns) used by the dense GEMM
// kernels (gemm.hip) and the implicit-GEMM convolutions (conv.hip).
#pragma once
#include "common.h"

namespace lumen {

struct GemmEpi {
  const void* bias;          // [N] (f32 if bias_f32 else bf16) or null
  const uint16_t* residual;  // [*, ldr] bf16 or null (indexed by *output* row)
  const uint16_t* table;     // [*, ldt] bf16 periodic add or null
  int64_t ldr;
  int64_t ldt;
  int table_period;
  int table_offset;
  int act;
  int bias_f32;
  float alpha;
  int out_group;             // 0 = identity row map
  int64_t out_group_stride;
  int out_row_offset;
  int out_f32;
  const uint16_t* prelu;     // [N] per-channel PReLU slopes (bf16) or null; applied after act
  int post_act;              // activation applied AFTER the residual add (ResNet: relu(conv + x))
  int glu;                   // SwiGLU: columns interleaved [gate 8 | up 8] per 16; writes silu(g) * u to
                             // column n/2 .. n/2+8 of C (C has N/2 columns)
};

__device__ __forceinline__ int swz(int row, int chunk) {
  // 16-byte chunk index XOR row bits 1..3: a ds_read_b128 lane group that reads
  // the same logical chunk of 16 consecutive rows hits 16 distinct bank slots.
  return (row << 7) + (((chunk ^ ((row >> 1) & 7))) << 4);
}

__device__ __forceinline__ void add8(float* v, const uint16_t* p) {
  float f[8];
  unpack8(*(const u32x4_t*)p, f);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] += f[q];
}

// Apply the epilogue to 16 consecutive columns [n, n+16) of row m and store.
__device__ __forceinline__ void epi_store16(float* v, int m, int n, int M, int N, void* __restrict__ C,
                                            int64_t ldc, const GemmEpi& ep) {
  if (m >= M || n >= N) return;
  const bool full = (n + 16 <= N);
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] *= ep.alpha;
  if (ep.bias) {
    if (ep.bias_f32) {
      const float* b = (const float*)ep.bias + n;
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] += (full || n + q < N) ? b[q] : 0.f;
    } else {
      const uint16_t* b = (const uint16_t*)ep.bias + n;
      if (full) {
        add8(v, b);
        add8(v + 8, b + 8);
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) if (n + q < N) v[q] += bf2f(b[q]);
      }
    }
  }
  if (ep.glu) {
    float r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = v[q] * fast_rcp(1.f + __expf(-v[q])) * v[8 + q];
    uint16_t* o = (uint16_t*)C + (int64_t)m * ldc + (n >> 1);
    *(u32x4_t*)o = pack8(r);
    return;
  }
  if (ep.act) apply_act_n<16>(v, ep.act);
  if (ep.prelu) {
    float sl[16];
    if (full) {
      unpack8(*(const u32x4_t*)(ep.prelu + n), sl);
      unpack8(*(const u32x4_t*)(ep.prelu + n + 8), sl + 8);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) sl[q] = (n + q < N) ? bf2f(ep.prelu[n + q]) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = v[q] > 0.f ? v[q] : v[q] * sl[q];
  }
  int64_t orow = m;
  if (ep.out_group > 0)
    orow = (int64_t)(m / ep.out_group) * ep.out_group_stride + ep.out_row_offset + (m % ep.out_group);
  if (ep.table) {
    const uint16_t* t = ep.table + (int64_t)((m % ep.table_period) + ep.table_offset) * ep.ldt + n;
    if (full) {
      add8(v, t);
      add8(v + 8, t + 8);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) if (n + q < N) v[q] += bf2f(t[q]);
    }
  }
  if (ep.residual) {
    const uint16_t* t = ep.residual + orow * ep.ldr + n;
    if (full) {
      add8(v, t);
      add8(v + 8, t + 8);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) if (n + q < N) v[q] += bf2f(t[q]);
    }
  }
  // post-residual activation: ReLU only (ResNet tails).  A second full activation
  // switch here doubles the epilogue's live state and spills the 256x256 GEMM.
  if (ep.post_act) {
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = fmaxf(v[q], 0.f);
  }
  if (ep.out_f32) {
    float* o = (float*)C + orow * ldc + n;
    if (full) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *(f32x4_t*)(o + 4 * q) = (f32x4_t){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) if (n + q < N) o[q] = v[q];
    }
  } else {
    uint16_t* o = (uint16_t*)C + orow * ldc + n;
    if (full) {
      *(u32x4_t*)o = pack8(v);
      *(u32x4_t*)(o + 8) = pack8(v + 8);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) if (n + q < N) o[q] = f2bf(v[q]);
    }
  }
}

}  // namespace lumen
