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
  int64_t* dbg;              // profiling only: per-workgroup s_memrealtime stamps (null in production)
  int64_t split_koff;        // split-K launches (gridDim.y = splits): A, W advance by y * split_koff
  int64_t split_cstride;     // elements; C (fp32 slabs) advances by y * split_cstride
  // ---- decode (skinny) GEMMs only: RMSNorm folded into the projection.  gamma is folded
  // into W at load time (LLM.fold_norms), so rms_norm(x) . W'^T = rstd(x) * (x . W'^T): the
  // kernel runs on the raw residual-stream rows and scales row m of the accumulator by
  // rstd[m] before the bias.  rstd comes from ssq_in -- per (row, 16-column tile) sums of
  // squares of the stored bf16 rows that the producing GEMM's epilogue wrote to its
  // ssq_out, [M][ssq_tiles], summed in a fixed order -- or, when null, from A itself.
  int norm;
  float norm_eps;
  const float* ssq_in;
  float* ssq_out;
  int ssq_tiles;
  // ---- LayerNorm folded into the projection (pre-LN transformer blocks, ops.linear_lnf):
  //   LN(x) . W^T + b = rstd * (x . W'^T) - rstd * mean * colsum(W') + (b + W . beta),
  //   W' = W * gamma (prepared once on the host), so the GEMM runs on the raw residual
  //   stream and no normalised copy of x is written.  row_aff [M][2] = (rstd, -mean * rstd)
  //   per A row (ln_row_stats), col_aff [2][N] fp32 = (colsum(W'), b + W . beta).  Applied
  //   first, in place of alpha and bias (the host passes neither).
  const float* row_aff;
  const float* col_aff;
  // ---- per-channel affine of the FINAL value (after residual / post-activation), fp32 [N] scale /
  // shift, applied to the bf16-rounded output: written to aff_out (second output, ld_aff) or, when
  // aff_out is null, in place of the plain output.  IResNet: the next block's pre-conv BatchNorm
  // (it precedes a zero-padded conv, so it cannot fold into weights) produced by the conv that
  // writes the block input, instead of a separate channel-affine pass.  Honoured by the
  // implicit-GEMM convolutions (epi_store16_t<WT, true>).
  const float* aff_s;
  const float* aff_t;
  uint16_t* aff_out;
  int64_t ld_aff;
};

// MX operand / outputs of the W8A8 prefill GEMM (gemm_f8.hip::gemm_mx; fields documented there)
// MX scale bytes live in K-step planes: byte (row m, 32-column block b) at [b / 4][m][b % 4], plane
// stride ld_bs / ldqs bytes (>= 4 M) -- the consumer's per-step load of 64 rows is contiguous.
struct MxArgs {
  const uint8_t* a_bs;
  int64_t ld_bs;
  const float* ssq_in;
  int ssq_in_tiles;
  float norm_eps;
  uint8_t* q8;
  int64_t ldq;
  uint8_t* qs;
  int64_t ldqs;
  float* ssq_out;
  int ssq_out_tiles;
  int skip_c;        // SwiGLU with q8: no bf16 output
};

// Launch plan of an fp8-weight decode GEMM (gemm_w8.hip): column tiles per wave, K splits and
// the K chunk per split.  The host sizes the split-K slabs / counters from the same plan.
struct W8DecPlan {
  int tpw;
  int ks;
  int kchunk;
};
W8DecPlan w8_dec_plan(int M, int N, int K);

// rstd of the M (<= 32) A rows of a norm-folded decode GEMM into LDS (wave w: rows w, w + NWV, ...);
// the caller's next __syncthreads publishes it.  K = row length (the normalised width).
template <int NWV>
__device__ __forceinline__ void skinny_rstd(const uint16_t* __restrict__ A, int64_t lda, int M, int K,
                                            const GemmEpi& ep, float* rstd) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int m = wid; m < M; m += NWV) {
    float s = 0.f;
    if (ep.ssq_in) {
      const float* p = ep.ssq_in + (int64_t)m * ep.ssq_tiles;
      for (int j = lane; j < ep.ssq_tiles; j += 64) s += p[j];
    } else {
      const uint16_t* r = A + (int64_t)m * lda;
#pragma unroll 4
      for (int c = lane * 8; c < K; c += 512) {
        float f[8];
        unpack8(*(const u32x4_t*)(r + c), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) s += f[i] * f[i];
      }
    }
    s = wave_sum(s);
    if (lane == 0) rstd[m] = rsqrtf(s / (float)K + ep.norm_eps);
  }
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));

// ---- shared geometry of the 256x256x64 LDS-DMA kernels (gemm.hip, gemm_pp.hip)
constexpr int BK = 64;                  // K elements per tile = 128-byte LDS rows
constexpr int G_HALF = 128 * 128;       // bytes per half-tile image (128 rows x 128 B)
constexpr int G_OP = 2 * G_HALF;
constexpr int G_BUF = 2 * G_OP;

#ifndef LM_GEMM_RES_PREFETCH
#define LM_GEMM_RES_PREFETCH 4
#endif

__device__ __forceinline__ void vm_wait4() { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
__device__ __forceinline__ void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// linear tile id -> (row tile, column tile); group_m > 1 walks group_m row panels per column
__device__ __forceinline__ void tile_coords(int lin, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  if (group_m > 1) {
    const int span = group_m * tiles_n;
    const int grp = lin / span, first = grp * group_m;
    const int gsz = min(tiles_m - first, group_m);
    const int r = lin % span;
    tm = first + r % gsz;
    tn = r / gsz;
  } else {
    tm = lin / tiles_n;
    tn = lin % tiles_n;
  }
}

// ping-pong 256x256 GEMM (gemm_pp.hip); variant bit 0: persistent (interior tiles), bit 1:
// static priority for the lagging wave group, bit 2: two phases per K-tile (32 MFMAs per phase)
hipError_t gemm_pp(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                   int N, int K, const GemmEpi& ep, int group_m, int variant, hipStream_t stream);
// split-K form for a few row tiles (the tail rows of a round-split GEMM): fp32 slabs from one
// ping-pong launch over (tile, split), then one reduce + epilogue pass.  hipErrorNotSupported
// when the epilogue / shape / workspace does not allow it (caller falls back).
hipError_t gemm_tail_splitk(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc,
                            int M, int N, int K, const GemmEpi& ep, hipStream_t stream);


// 16-byte store of C: plain, or write-through (sc1) via a buffer descriptor over C.
// Write-through matters for the big-tile epilogues: every CU publishing its whole
// 128 KB C tile at once with plain (write-back) stores drains at ~1.7 TB/s chip-wide
// (MI355X_MICROARCH publish-large: 64 KB per WG 8.2 us plain vs 3.0 us sc1).
template <bool WT>
__device__ __forceinline__ void st16(void* C, __amdgpu_buffer_rsrc_t rs, int64_t byte_off, u32x4_t v) {
  if constexpr (WT) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v), rs, (int)byte_off, 0, 16);
  else *(u32x4_t*)((char*)C + byte_off) = v;
}

// 16-byte LDS-DMA through a buffer descriptor (buffer_load_dwordx4 ... offen lds): per-lane 32-bit
// byte offset, wave-uniform soffset; an offset past num_records lands as zeros.  A non-template
// wrapper: called directly from a kernel template the builtin suppresses the host-side stub.
__device__ __forceinline__ void buf_load_lds16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t c_rsrc(void* C) {
  return __builtin_amdgcn_make_buffer_rsrc(C, (short)0, -1, 0x00020000);
}

__device__ __forceinline__ int swz(int row, int chunk) {
  // 16-byte chunk index XOR row bits 1..3: a ds_read_b128 lane group that reads
  // the same logical chunk of 16 consecutive rows hits 16 distinct bank slots.
  return (row << 7) + (((chunk ^ ((row >> 1) & 7))) << 4);
}

// Direct-store ping-pong kernels (gemm_pp.hip, DS): the MFMA takes W as its first operand, so a lane's
// accumulator holds 4 consecutive OUTPUT COLUMNS of one row, and the B fragment of 16x16 block j holds
// W rows 8 * (f >> 2) + 4 * j + (f & 3) (f = lane & 15): blocks j = 0, 1 together give each lane 8
// consecutive columns -> one 16-byte store, no LDS round trip in the epilogue.  Those fragment rows
// ({0-3, 8-11, 16-19, 24-27} + 4j) hit 2-way bank conflicts under swz's XOR of row bits 1..3; this
// XOR of row bits 1, 3, 4 (searched exhaustively over linear XOR maps) keeps every ds_read_b128 lane
// group on 16 distinct bank slots.  Applied to the B half-tiles only (DMA source chunk and read).
__device__ __forceinline__ int ds_bxor(int row) {
  const int x = row >> 1;
  return (x & 1) ^ (((x >> 2) & 1) << 1) ^ (((x >> 3) & 1) << 2);
}
__device__ __forceinline__ int swzb(int row, int chunk) { return (row << 7) + ((chunk ^ ds_bxor(row)) << 4); }

__device__ __forceinline__ void add8(float* v, const uint16_t* p) {
  float f[8];
  unpack8(*(const u32x4_t*)p, f);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] += f[q];
}

// Apply the epilogue to 16 consecutive columns [n, n+16) of row m and store.  AFF: the output
// affine (GemmEpi::aff_s) is live (bf16 output, full 16-column pieces: the conv host code checks).
template <bool WT, bool AFF = false>
__device__ __forceinline__ void epi_store16_t(float* v, int m, int n, int M, int N, void* __restrict__ C,
                                              int64_t ldc, const GemmEpi& ep, __amdgpu_buffer_rsrc_t rs) {
  if (m >= M || n >= N) return;
  const bool full = (n + 16 <= N);
  if (ep.row_aff) {
    const float rs = ep.row_aff[2 * (int64_t)m], ro = ep.row_aff[2 * (int64_t)m + 1];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      v[q] = (full || n + q < N) ? v[q] * rs + ro * ep.col_aff[n + q] + ep.col_aff[N + n + q] : 0.f;
  }
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
    st16<WT>(C, rs, ((int64_t)m * ldc + (n >> 1)) * 2, pack8(r));
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
  if constexpr (AFF) {
    float w[16];
    const f32x4_t* s4 = (const f32x4_t*)(ep.aff_s + n);
    const f32x4_t* t4 = (const f32x4_t*)(ep.aff_t + n);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4_t sq = s4[q], tq = t4[q];
#pragma unroll
      for (int r = 0; r < 4; ++r) w[4 * q + r] = bf2f(f2bf(v[4 * q + r])) * sq[r] + tq[r];
    }
    if (ep.aff_out) {
      uint16_t* o2 = ep.aff_out + orow * ep.ld_aff + n;
      *(u32x4_t*)o2 = pack8(w);
      *(u32x4_t*)(o2 + 8) = pack8(w + 8);
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = w[q];
    }
  }
  if (ep.out_f32) {
    float* o = (float*)C + orow * ldc + n;
    if (full) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st16<WT>(C, rs, (orow * ldc + n + 4 * q) * 4,
                 __builtin_bit_cast(u32x4_t, (f32x4_t){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]}));
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) if (n + q < N) o[q] = v[q];
    }
  } else {
    uint16_t* o = (uint16_t*)C + orow * ldc + n;
    if (full) {
      st16<WT>(C, rs, (orow * ldc + n) * 2, pack8(v));
      st16<WT>(C, rs, (orow * ldc + n + 8) * 2, pack8(v + 8));
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) if (n + q < N) o[q] = f2bf(v[q]);
    }
  }
}

// 8-column form (no SwiGLU): [n, n+8) of row m.  Used by the row-coalesced
// 256x256 epilogue, where 16 consecutive lanes store 256 contiguous bytes.
template <bool WT>
__device__ __forceinline__ void epi_store8_t(float* v, int m, int n, int M, int N, void* __restrict__ C, int64_t ldc,
                                             const GemmEpi& ep, __amdgpu_buffer_rsrc_t rs) {
  if (m >= M || n >= N) return;
  const bool full = (n + 8 <= N);
  if (ep.row_aff) {
    const float rs = ep.row_aff[2 * (int64_t)m], ro = ep.row_aff[2 * (int64_t)m + 1];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      v[q] = (full || n + q < N) ? v[q] * rs + ro * ep.col_aff[n + q] + ep.col_aff[N + n + q] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] *= ep.alpha;
  if (ep.bias) {
    if (ep.bias_f32) {
      const float* b = (const float*)ep.bias + n;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += (full || n + q < N) ? b[q] : 0.f;
    } else {
      const uint16_t* b = (const uint16_t*)ep.bias + n;
      if (full) add8(v, b);
      else {
#pragma unroll
        for (int q = 0; q < 8; ++q) if (n + q < N) v[q] += bf2f(b[q]);
      }
    }
  }
  if (ep.act) apply_act_n<8>(v, ep.act);
  if (ep.prelu) {
    float sl[8];
    if (full) unpack8(*(const u32x4_t*)(ep.prelu + n), sl);
    else {
#pragma unroll
      for (int q = 0; q < 8; ++q) sl[q] = (n + q < N) ? bf2f(ep.prelu[n + q]) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.f ? v[q] : v[q] * sl[q];
  }
  int64_t orow = m;
  if (ep.out_group > 0)
    orow = (int64_t)(m / ep.out_group) * ep.out_group_stride + ep.out_row_offset + (m % ep.out_group);
  if (ep.table) {
    const uint16_t* t = ep.table + (int64_t)((m % ep.table_period) + ep.table_offset) * ep.ldt + n;
    if (full) add8(v, t);
    else {
#pragma unroll
      for (int q = 0; q < 8; ++q) if (n + q < N) v[q] += bf2f(t[q]);
    }
  }
  if (ep.residual) {
    const uint16_t* t = ep.residual + orow * ep.ldr + n;
    if (full) add8(v, t);
    else {
#pragma unroll
      for (int q = 0; q < 8; ++q) if (n + q < N) v[q] += bf2f(t[q]);
    }
  }
  if (ep.post_act) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
  }
  if (ep.out_f32) {
    float* o = (float*)C + orow * ldc + n;
    if (full) {
      st16<WT>(C, rs, (orow * ldc + n) * 4, __builtin_bit_cast(u32x4_t, (f32x4_t){v[0], v[1], v[2], v[3]}));
      st16<WT>(C, rs, (orow * ldc + n + 4) * 4, __builtin_bit_cast(u32x4_t, (f32x4_t){v[4], v[5], v[6], v[7]}));
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) if (n + q < N) o[q] = v[q];
    }
  } else {
    uint16_t* o = (uint16_t*)C + orow * ldc + n;
    if (full) st16<WT>(C, rs, (orow * ldc + n) * 2, pack8(v));
    else {
#pragma unroll
      for (int q = 0; q < 8; ++q) if (n + q < N) o[q] = f2bf(v[q]);
    }
  }
}

// Fast path for fully in-range 16-column pieces whose bf16 bias (2 x 8) and residual
// (2 x 8 bf16) were prefetched into registers when the tile's epilogue began: the
// generic path loads them inside each 16-row slab, exposing an L2/HBM round trip per
// slab (8 per tile; measured +8 % for bias, +22 % for bias + residual at K = 1024).
template <bool WT, bool RES>
__device__ __forceinline__ void epi_store16_fast(float* v, int64_t m, int n, void* __restrict__ C, int64_t ldc,
                                                 const GemmEpi& ep, u32x4_t b0, u32x4_t b1, u32x4_t r0, u32x4_t r1,
                                                 __amdgpu_buffer_rsrc_t rs) {
  {
    float f[8];
    unpack8(b0, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = v[q] * ep.alpha + f[q];
    unpack8(b1, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[8 + q] = v[8 + q] * ep.alpha + f[q];
  }
  if (ep.act) apply_act_n<16>(v, ep.act);
  if constexpr (RES) {
    float f[8];
    unpack8(r0, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += f[q];
    unpack8(r1, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
  }
  st16<WT>(C, rs, (m * ldc + n) * 2, pack8(v));          // bf16 output only (host-checked)
  st16<WT>(C, rs, (m * ldc + n + 8) * 2, pack8(v + 8));
}

// LN-folded fast path (FK = 5 of the ping-pong kernels): v[q] = v[q] * rs + ro * cs[q] + cb[q], then the
// activation, bf16 store of n_cols (8 or 16) columns.  cs / cb: the lane's columns of col_aff, prefetched.
template <bool WT, int NC>
__device__ __forceinline__ void epi_store_lnf(float* v, int64_t m, int n, void* __restrict__ C, int64_t ldc,
                                              const GemmEpi& ep, float rs, float ro, const float* cs, const float* cb,
                                              __amdgpu_buffer_rsrc_t r) {
#pragma unroll
  for (int q = 0; q < NC; ++q) v[q] = v[q] * rs + (ro * cs[q] + cb[q]);
  if (ep.act) apply_act_n<NC>(v, ep.act);
#pragma unroll
  for (int h = 0; h < NC / 8; ++h) st16<WT>(C, r, (m * ldc + n + 8 * h) * 2, pack8(v + 8 * h));
}

__device__ __forceinline__ void epi_store16(float* v, int m, int n, int M, int N, void* __restrict__ C, int64_t ldc,
                                            const GemmEpi& ep) {
  epi_store16_t<false>(v, m, n, M, N, C, ldc, ep, c_rsrc(C));
}
__device__ __forceinline__ void epi_store8(float* v, int m, int n, int M, int N, void* __restrict__ C, int64_t ldc,
                                           const GemmEpi& ep) {
  epi_store8_t<false>(v, m, n, M, N, C, ldc, ep, c_rsrc(C));
}
// decode GEMM epilogue: optional rstd row scale (norm folding, before the bias), the shared
// epilogue, then the producer's per-tile sum of squares of the stored bf16 values (ssq_out)
__device__ __forceinline__ void epi_store16_dec(float* v, float rs, int m, int n, int M, int N,
                                                void* __restrict__ C, int64_t ldc, const GemmEpi& ep) {
  if (ep.norm) {
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] *= rs;
  }
  epi_store16(v, m, n, M, N, C, ldc, ep);
  if (ep.ssq_out && m < M && n < N) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float f = bf2f(f2bf(v[q]));
      s += n + q < N ? f * f : 0.f;
    }
    ep.ssq_out[(int64_t)m * ep.ssq_tiles + (n >> 4)] = s;
  }
}

// In-launch split-K reduction of the skinny decode GEMMs (the counter form of the
// write-through hand-off, cdna_hip_programming.md §6 G16 / MI355X_MICROARCH.md: per-XCD
// L2s are not coherent, and a __threadfence() per block costs ~4x the whole GEMM).
// Called by every thread once `red` ([4 waves][rows][17] LDS partials) is complete:
//   1. the workgroup's summed partial tile goes to its fp32 slab with agent-scope
//      (sc1, write-through) stores, drained by every wave before the barrier;
//   2. lane 0 draws a ticket from the tile's counter (relaxed agent fetch_add); the
//      workgroup that draws nsplit-1 arrived last, resets the counter (buffer is
//      all-zero between kernels) and tells its waves through red's padding column;
//   3. the last arriver reads every slab with sc1 loads and sums them in split order
//      (deterministic, independent of arrival order) into red[1][m][c].
// No release/acquire fences: sc1 stores leave L2 before the ticket, sc1 loads bypass L1.
template <int NWV, int ROWS>
__device__ __forceinline__ bool splitk_reduce_last(float (&red)[NWV][ROWS][17], float* ws, uint32_t* cnt, int M, int N,
                                                   int n0) {
  const int tid = threadIdx.x;
  const int64_t slab = (int64_t)M * N;
  float* mine = ws + (int64_t)blockIdx.y * slab;
  for (int idx = tid; idx < ROWS * 16; idx += blockDim.x) {
    const int m = idx >> 4, c = idx & 15;
    if (m < M && n0 + c < N) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) v += red[w][m][c];
      __hip_atomic_store(mine + (int64_t)m * N + n0 + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == gridDim.y - 1;
    if (last) __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    red[0][0][16] = last ? 1.f : 0.f;
  }
  __syncthreads();
  if (red[0][0][16] == 0.f) return false;
  for (int idx = tid; idx < ROWS * 16; idx += blockDim.x) {
    const int m = idx >> 4, c = idx & 15;
    float v = 0.f;
    if (m < M && n0 + c < N) {
      const float* p = ws + (int64_t)m * N + n0 + c;
      for (int s = 0; s < (int)gridDim.y; ++s)
        v += __hip_atomic_load(p + s * slab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    red[1][m][c] = v;
  }
  __syncthreads();
  return true;
}

}  // namespace lumen
