// Weight-only FP8 GEMMs for the LLM decoder (BASELINE config 5: "fp8 CDNA4 MFMA").
//
//   C[M, N] = epi( (A[M, K] . W8[N, K]^T) * scale[n] )
//
// W8 is OCP e4m3fn (gfx950's native fp8, NOT the MI300 fnuz encoding) with one fp32
// scale per output row, A stays bf16.  Every e4m3 value is exactly representable in
// bf16, so each fp8 pair is widened with ONE v_cvt_scalef32_pk_bf16_fp8 (scale 1.0)
// and fed to the bf16 MFMA; the per-channel scale is applied once in fp32 in the
// epilogue.  Decode GEMMs are HBM-bound on W, so halving the weight bytes is the
// whole point there; prefill keeps bf16 MFMA throughput with half the weight traffic.
//
//  * gemm_skinny_w8_kernel (M <= 32, decode): the split-K skinny kernel of
//    gemm_skinny.hip with 16-byte loads of 16 fp8 weights per lane.  The MFMA k order
//    inside a 64-wide block is permuted identically for A and W (lane group g owns
//    k in [16g, 16g + 16)), so one W load feeds two MFMAs.
//  * gemm_w8_kernel (M > 32, prefill): register-staged 2-stage tile; the W tile is
//    loaded as 8 fp8 per chunk and widened to bf16 on its way into the swizzled LDS
//    image, after which the MFMA loop is the bf16 one.
#include <cstdlib>

#include "common.h"
#include "gemm_epi.h"

namespace lumen {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// row-streaming decode weights (M <= 4): read once per launch by one CU -> non-temporal
// (8B fp8 single-stream decode 428 -> 452 tok/s, r3).  The batched kernels
// (M > 4) keep the default policy: nt measured 5 % slower there (r3_w8_nt_ab_v1.txt).
template <bool NT>
__device__ __forceinline__ u32x4_t wload(const uint8_t* p) {
  if constexpr (NT) return ld_nt16(p);
  else return *(const u32x4_t*)p;
}

__device__ __forceinline__ void fp8x16_to_bf16(const u32x4_t w, bf16x8_t& f0, bf16x8_t& f1) {
  f0 = __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(w[0], w[1]));
  f1 = __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(w[2], w[3]));
}

// ============================================================================ decode, 16 < M <= 32
// Two 16-row MFMA tiles per wave (MT = 2); the K range of a 16-column tile is split over the
// 4 waves (64-wide k blocks interleaved, 4 in flight per wave) and, for narrow N, over grid.y
// with the in-launch split-K reduction.  The MFMA k order inside a 64-wide block is permuted
// identically for A and W (lane group g owns k in [16g, 16g + 16)), so one 16-byte W load
// feeds two MFMAs.
template <int MT>
__global__ void __launch_bounds__(256) gemm_skinny_w8_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                             const uint8_t* __restrict__ W, int64_t ldw,
                                                             const float* __restrict__ scale, void* __restrict__ C,
                                                             int64_t ldc, float* __restrict__ ws, uint32_t* __restrict__ cnt,
                                                             int M, int N, int K, int kchunk, GemmEpi ep) {
  constexpr int NWV = 4, UNR = 4;
  __shared__ float red[NWV][MT * 16][17];
  __shared__ float rstd_s[MT * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int k_begin = blockIdx.y * kchunk;
  const int k_end = min(K, k_begin + kchunk);
  const uint8_t* wr = W + (int64_t)min(n0 + col, N - 1) * ldw + g * 16;
  const uint16_t* ar[MT];
  bool av[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + col;
    av[t] = m < M;
    ar[t] = A + (int64_t)(av[t] ? m : 0) * lda + g * 16;
  }
  f32x4_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto mma_block = [&](const u32x4_t w8, const u32x4_t (&a)[MT][2]) {
    bf16x8_t f0, f1;
    fp8x16_to_bf16(w8, f0, f1);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[t][0]), f0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[t][1]), f1, acc[t], 0, 0, 0);
    }
  };
  auto load_a = [&](int k, u32x4_t (&a)[MT][2]) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      a[t][0] = *(const u32x4_t*)(ar[t] + k);
      a[t][1] = *(const u32x4_t*)(ar[t] + k + 8);
      if (!av[t]) a[t][0] = a[t][1] = (u32x4_t){0u, 0u, 0u, 0u};
    }
  };
  const int nblk = (k_end - k_begin) / 64;
  int s = wid;
  for (; s + NWV * (UNR - 1) < nblk; s += NWV * UNR) {
    u32x4_t wf[UNR];
    u32x4_t af[UNR][MT][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int k = k_begin + (s + NWV * u) * 64;
      wf[u] = *(const u32x4_t*)(wr + k);
      load_a(k, af[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) mma_block(wf[u], af[u]);
  }
  for (; s < nblk; s += NWV) {
    const int k = k_begin + s * 64;
    const u32x4_t wf = *(const u32x4_t*)(wr + k);
    u32x4_t af[MT][2];
    load_a(k, af);
    mma_block(wf, af);
  }
  // C fragment: row (m) = t*16 + 4g + r, column n0 + col
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][t * 16 + 4 * g + r][col] = acc[t][r];
  if (ep.norm) skinny_rstd<NWV>(A, lda, M, K, ep, rstd_s);
  __syncthreads();
  if (ws != nullptr) {   // K split over grid.y: the last split to arrive reduces + runs the epilogue
    if (!splitk_reduce_last(red, ws, cnt, M, N, n0)) return;
    if (tid < M) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = red[1][tid][c] * (n0 + c < N ? scale[n0 + c] : 0.f);
      epi_store16_dec(v, rstd_s[tid], tid, n0, M, N, C, ldc, ep);
    }
    return;
  }
  if (tid < M) {
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t += red[w][tid][c];
      v[c] = t * (n0 + c < N ? scale[n0 + c] : 0.f);
    }
    epi_store16_dec(v, rstd_s[tid], tid, n0, M, N, C, ldc, ep);
  }
}

// ============================================================================ decode, 4 < M <= 16
// Batched decode GEMV on MFMA: a workgroup owns a stripe of 16 * TPW output columns and a K
// range (grid.y splits K for narrow N); its 4 waves interleave 64-wide k blocks.  Per k block a
// wave loads the A fragment (16 rows x 32 B per lane group) ONCE and TPW weight fragments, and
// issues 2 * TPW MFMAs: the activations cost 1 / (2 TPW) of the weight bytes in load traffic
// (the one-tile kernel paid 2x the weight bytes in L2 reads of A).  k blocks run as a two-slot
// register pipeline of U-block chunks.  Norm sums of squares and the column scales are loaded
// before the weight stream (vmcnt retires in issue order).
template <int TPW, int U>
__global__ void __launch_bounds__(256) gemv_w8_mfma_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                           const uint8_t* __restrict__ W, int64_t ldw,
                                                           const float* __restrict__ scale, void* __restrict__ C,
                                                           int64_t ldc, float* __restrict__ ws, uint32_t* __restrict__ cnt,
                                                           int M, int N, int K, int kchunk, GemmEpi ep) {
  constexpr int COLS = 16 * TPW;
  __shared__ float red[4][16][COLS + 1];
  __shared__ float sc_s[COLS];
  __shared__ float rstd_s[16];
  __shared__ int last_s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * COLS;
  const int k_begin = blockIdx.y * kchunk;
  const int k_end = min(K, k_begin + kchunk);

  // ---- epilogue operands first
  const float scv = scale[min(n0 + (tid % COLS), N - 1)];
  const bool rs_pre = ep.norm && ep.ssq_in != nullptr && ep.ssq_tiles <= 16 * 16;   // K <= 4096
  f32x4_t ssq_v[4];
  if (rs_pre) {   // thread (row tid / 16, part tid % 16): float4 s part, part + 16, ...
    const f32x4_t* p = (const f32x4_t*)(ep.ssq_in + (int64_t)min(tid >> 4, M - 1) * ep.ssq_tiles);
    const int n4 = ep.ssq_tiles >> 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) ssq_v[j] = p[min((tid & 15) + 16 * j, n4 - 1)];
  }

  const uint8_t* wr[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) wr[t] = W + (int64_t)min(n0 + t * 16 + col, N - 1) * ldw + g * 16;
  const bool arow = col < M;
  const uint16_t* ar = A + (int64_t)(arow ? col : 0) * lda + g * 16;
  f32x4_t acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  u32x4_t wb[2][U][TPW];
  u32x4_t ab[2][U][2];
  const int nblk = (k_end - k_begin) >> 6;
  const int mine = wid < nblk ? (nblk - wid + 3) >> 2 : 0;   // this wave's k blocks: wid, wid + 4, ...
  auto issue = [&](const int slot, const int j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = k_begin + (int64_t)(wid + 4 * (j0 + u)) * 64;
#pragma unroll
      for (int t = 0; t < TPW; ++t) wb[slot][u][t] = *(const u32x4_t*)(wr[t] + k);
      ab[slot][u][0] = *(const u32x4_t*)(ar + k);
      ab[slot][u][1] = *(const u32x4_t*)(ar + k + 8);
    }
  };
  auto consume = [&](const int slot, const int nu) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < nu) {
        const u32x4_t a0 = arow ? ab[slot][u][0] : (u32x4_t){0u, 0u, 0u, 0u};
        const u32x4_t a1 = arow ? ab[slot][u][1] : (u32x4_t){0u, 0u, 0u, 0u};
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          bf16x8_t f0, f1;
          fp8x16_to_bf16(wb[slot][u][t], f0, f1);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0), f0, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1), f1, acc[t], 0, 0, 0);
        }
      }
    }
  };
  const int nch = mine / U;
  if (nch > 0) {
    issue(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    int c = 0;
    for (; c + 2 < nch; c += 2) {
      issue(1, (c + 1) * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(0, U);
      __builtin_amdgcn_sched_barrier(0);
      issue(0, (c + 2) * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(1, U);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < nch) {
      issue(1, (c + 1) * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(0, U);
      __builtin_amdgcn_sched_barrier(0);
      consume(1, U);
    } else {
      consume(0, U);
    }
  }
  for (int j = nch * U; j < mine; ++j) {   // remainder blocks, one at a time
    const int64_t k = k_begin + (int64_t)(wid + 4 * j) * 64;
#pragma unroll
    for (int t = 0; t < TPW; ++t) wb[0][0][t] = *(const u32x4_t*)(wr[t] + k);
    ab[0][0][0] = *(const u32x4_t*)(ar + k);
    ab[0][0][1] = *(const u32x4_t*)(ar + k + 8);
    consume(0, 1);
  }

  // ---- wave partials -> LDS (C fragment: row 4g + r, column t * 16 + col)
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][4 * g + r][t * 16 + col] = acc[t][r];
  if (tid < COLS) sc_s[tid] = scv;
  if (ep.norm) {
    if (rs_pre) {
      const int n4 = ep.ssq_tiles >> 2;
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((tid & 15) + 16 * j < n4) t += (ssq_v[j][0] + ssq_v[j][1]) + (ssq_v[j][2] + ssq_v[j][3]);
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
      if ((tid & 15) == 0 && (tid >> 4) < 16) rstd_s[tid >> 4] = rsqrtf(t / (float)K + ep.norm_eps);
    } else {
      skinny_rstd<4>(A, lda, M, K, ep, rstd_s);
    }
  }
  __syncthreads();
  // wave sum, kept in red[0] (thread-owned elements only: no race)
  for (int i = tid; i < 16 * COLS; i += 256) {
    const int m = i / COLS, c = i - m * COLS;
    red[0][m][c] = (red[0][m][c] + red[1][m][c]) + (red[2][m][c] + red[3][m][c]);
  }
  if (ws != nullptr) {
    // ---- in-launch split-K: write-through partial slab, ticket, the last split sums in order
    const int64_t slab = (int64_t)M * N;
    for (int i = tid; i < M * COLS; i += 256) {
      const int m = i / COLS, c = i - m * COLS;
      if (n0 + c < N)
        __hip_atomic_store(ws + blockIdx.y * slab + (int64_t)m * N + n0 + c, red[0][m][c], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint32_t prev = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = prev == gridDim.y - 1;
      if (last) __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_s = last ? 1 : 0;
    }
    __syncthreads();
    if (!last_s) return;
    const int S = gridDim.y;
    for (int i = tid; i < M * COLS; i += 256) {
      const int m = i / COLS, c = i - m * COLS;
      const float* p = ws + (int64_t)m * N + min(n0 + c, N - 1);
      float v = 0.f;
      for (int s0 = 0; s0 < S; s0 += 8) {   // 8 slab loads in flight; summed in split order
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          pv[j] = __hip_atomic_load(p + min(s0 + j, S - 1) * slab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int j = 0; j < 8; ++j) v += s0 + j < S ? pv[j] : 0.f;
      }
      red[1][m][c] = v;
    }
    __syncthreads();
  }
  const int src = ws != nullptr ? 1 : 0;
  __syncthreads();
  if (tid < M * TPW) {   // thread: (row m, 16-column tile t)
    const int m = tid / TPW, t = tid - m * TPW;
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = red[src][m][t * 16 + c] * sc_s[t * 16 + c];
    epi_store16_dec(v, rstd_s[m], m, n0 + t * 16, M, N, C, ldc, ep);
  }
}

// t + <8 bf16 of x, 8 bf16 of y> on v_dot2c_f32_bf16.  The pairs are taken by shuffling a
// bf16x8 view: bit-casting a u32 vector ELEMENT to bf16x2 miscompiles on ROCm 7.2 (every
// element reads lane 0's dword).
__device__ __forceinline__ float dot8_bf16(const u32x4_t x, const u32x4_t y, float t) {
  const bf16x8_t xv = __builtin_bit_cast(bf16x8_t, x), yv = __builtin_bit_cast(bf16x8_t, y);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x2_t p = {xv[2 * j], xv[2 * j + 1]}, q = {yv[2 * j], yv[2 * j + 1]};
    t = __builtin_amdgcn_fdot2_f32_bf16(p, q, t, false);
  }
  return t;
}

// ============================================================================ decode, M <= 4
// Row-streaming GEMV.  Every wave streams whole weight rows: one wave instruction reads 1 KiB
// contiguous of ONE row (lane l: bytes [16 l, 16 l + 16) of a 1024-wide k step).  The k steps
// run as a two-slot register pipeline of U-step chunks (chunk c + 1 is issued before chunk c is
// consumed: up to 2 * U * R * 16 B in flight per lane); each 16 fp8 widen to 8 bf16 pairs
// (v_cvt_scalef32_pk_bf16_fp8) and meet the bf16 activations (L1/L2-resident) in
// v_dot2c_f32_bf16; every (row, m) partial is reduced over the 64 lanes once at the end.
// A workgroup = 4 waves x 4 rows = 16 consecutive output columns, so the decode epilogue
// works on whole 16-column tiles (SwiGLU [gate 8 | up 8] pairing, ssq tiles).  Everything the
// epilogue reads -- the folded-norm sums of squares, the per-channel scales, bias and residual
// -- is loaded BEFORE the weight stream, so the tail after the last weight byte is only the
// reductions and the store (vmcnt retires in issue order: a load issued after the stream
// would wait behind it).  No MFMA: at M <= 4 the dot products use ~20-40 % of the VALU issue
// budget while HBM streams.
template <int MR, int U, bool NT>
__global__ void __launch_bounds__(256) gemv_w8_rows_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                           const uint8_t* __restrict__ W, int64_t ldw,
                                                           const float* __restrict__ scale, void* __restrict__ C,
                                                           int64_t ldc, int M, int N, int K, GemmEpi ep) {
  constexpr int R = 4;
  constexpr int SSQ_MAX = 16;   // ssq tiles per lane: K <= 16 * 64 * 16 = 16384
  __shared__ float red[16][MR];
  __shared__ float sc_s[16];
  __shared__ float rstd_s[MR];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * 16;

  // ---- epilogue operands first (see header); straight-line loads at clamped addresses, so no
  // exec-masked branch makes the compiler drain vmcnt before the weight stream is issued
  const float scv = scale[min(n0 + (lane & 15), N - 1)];
  constexpr int SSQ4 = 4;   // float4 ssq loads per lane and row: K <= 4 * 4 * 64 * 16 = 16384
  const bool rs_pre = MR <= 2 && ep.norm && ep.ssq_in != nullptr && K <= SSQ4 * 4 * 64 * 16;
  f32x4_t ssq_v[MR <= 2 ? MR : 1][SSQ4];
  if (rs_pre) {   // wave-uniform
    const int n4 = ep.ssq_tiles >> 2;
#pragma unroll
    for (int m = 0; m < (MR <= 2 ? MR : 1); ++m) {
      const f32x4_t* p = (const f32x4_t*)(ep.ssq_in + (int64_t)min(m, M - 1) * ep.ssq_tiles);
#pragma unroll
      for (int j = 0; j < SSQ4; ++j) ssq_v[m][j] = p[min(lane + j * 64, n4 - 1)];
    }
  }
  const int prow = min(lane, M - 1);
  const bool full16 = n0 + 16 <= N;
  const bool pre_bias = ep.bias && !ep.bias_f32 && full16;
  const bool pre_res = ep.residual && full16;
  u32x4_t pre_b[2] = {(u32x4_t){0u, 0u, 0u, 0u}, (u32x4_t){0u, 0u, 0u, 0u}};
  u32x4_t pre_r[2] = {(u32x4_t){0u, 0u, 0u, 0u}, (u32x4_t){0u, 0u, 0u, 0u}};
  if (pre_bias) {
    pre_b[0] = *(const u32x4_t*)((const uint16_t*)ep.bias + n0);
    pre_b[1] = *(const u32x4_t*)((const uint16_t*)ep.bias + n0 + 8);
  }
  if (pre_res) {
    pre_r[0] = *(const u32x4_t*)(ep.residual + (int64_t)prow * ep.ldr + n0);
    pre_r[1] = *(const u32x4_t*)(ep.residual + (int64_t)prow * ep.ldr + n0 + 8);
  }

  // ---- weight stream
  const int r0 = n0 + wid * R;
  const uint8_t* wp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wp[r] = W + (int64_t)min(r0 + r, N - 1) * ldw + lane * 16;
  const uint16_t* ap[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) ap[m] = A + (int64_t)(m < M ? m : 0) * lda + lane * 16;
  float acc[R][MR];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[r][m] = 0.f;

  u32x4_t wb[2][U][R];
  u32x4_t ab[2][U][MR][2];
  auto issue = [&](const int slot, const int st0) {   // U full 1024-wide steps
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t ko = (int64_t)(st0 + u) << 10;
#pragma unroll
      for (int r = 0; r < R; ++r) wb[slot][u][r] = wload<NT>(wp[r] + ko);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        ab[slot][u][m][0] = *(const u32x4_t*)(ap[m] + ko);
        ab[slot][u][m][1] = *(const u32x4_t*)(ap[m] + ko + 8);
      }
    }
  };
  auto consume = [&](const int slot, const int nu) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < nu) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const u32x4_t b0 = fp8x8_to_bf16(wb[slot][u][r][0], wb[slot][u][r][1]);
          const u32x4_t b1 = fp8x8_to_bf16(wb[slot][u][r][2], wb[slot][u][r][3]);
#pragma unroll
          for (int m = 0; m < MR; ++m)
            acc[r][m] = dot8_bf16(b1, ab[slot][u][m][1], dot8_bf16(b0, ab[slot][u][m][0], acc[r][m]));
        }
      }
    }
  };
  // Straight-line steady state (a conditional issue inside the loop makes the waitcnt pass
  // merge both paths and drain everything), and a sched_barrier after every issue: the machine
  // scheduler otherwise sinks part of chunk c's loads below chunk c + 1's.
  const int nfull = K >> 10;
  const int nch = nfull / U;
  if (nch > 0) {
    issue(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    int c = 0;
    for (; c + 2 < nch; c += 2) {
      issue(1, (c + 1) * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(0, U);
      __builtin_amdgcn_sched_barrier(0);
      issue(0, (c + 2) * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(1, U);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 1 < nch) {
      issue(1, (c + 1) * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(0, U);
      __builtin_amdgcn_sched_barrier(0);
      consume(1, U);
    } else {
      consume(0, U);
    }
  }
  // remainder: full steps past the last chunk, then the partial step (K % 1024; Qwen2: 896,
  // 4864), whose lanes past K load a clamped in-row address and zero their activations
  for (int st = nch * U; st < nfull; ++st) {
    const int64_t ko = (int64_t)st << 10;
#pragma unroll
    for (int r = 0; r < R; ++r) wb[0][0][r] = wload<NT>(wp[r] + ko);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      ab[0][0][m][0] = *(const u32x4_t*)(ap[m] + ko);
      ab[0][0][m][1] = *(const u32x4_t*)(ap[m] + ko + 8);
    }
    consume(0, 1);
  }
  if ((K & 1023) != 0) {
    const int k = (nfull << 10) + lane * 16;
    const bool ok = k < K;
    const int64_t ko = ok ? k - lane * 16 : K - 16 - lane * 16;
#pragma unroll
    for (int r = 0; r < R; ++r) wb[0][0][r] = wload<NT>(wp[r] + ko);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const u32x4_t a0 = *(const u32x4_t*)(ap[m] + ko), a1 = *(const u32x4_t*)(ap[m] + ko + 8);
      ab[0][0][m][0] = ok ? a0 : (u32x4_t){0u, 0u, 0u, 0u};
      ab[0][0][m][1] = ok ? a1 : (u32x4_t){0u, 0u, 0u, 0u};
    }
    consume(0, 1);
  }

  // ---- reductions + epilogue
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const float v = wave_sum(acc[r][m]);
      if (lane == 0) red[wid * R + r][m] = v;
    }
  if (tid < 16) sc_s[tid] = scv;
  if (ep.norm) {
    if (rs_pre) {
      if (wid == 0) {
        const int n4 = ep.ssq_tiles >> 2;
#pragma unroll
        for (int m = 0; m < (MR <= 2 ? MR : 1); ++m) {
          float t = 0.f;
#pragma unroll
          for (int j = 0; j < SSQ4; ++j)
            if (lane + j * 64 < n4) t += (ssq_v[m][j][0] + ssq_v[m][j][1]) + (ssq_v[m][j][2] + ssq_v[m][j][3]);
          t = wave_sum(t);
          if (lane == 0 && m < M) rstd_s[m] = rsqrtf(t / (float)K + ep.norm_eps);
        }
      }
    } else {
      skinny_rstd<4>(A, lda, M, K, ep, rstd_s);
    }
  }
  __syncthreads();
  if (tid < M) {
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = red[c][tid] * sc_s[c];
    if (ep.norm) {
      const float rs = rstd_s[tid];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] *= rs;
    }
    const bool fast = full16 && !ep.bias_f32 && !ep.act && !ep.out_f32 && ep.out_group == 0 && !ep.table &&
                      !ep.prelu && !ep.post_act && ep.alpha == 1.f;
    if (fast) {   // bias / residual from the prologue registers (lane tid < M loaded row tid)
      if (pre_bias) {
        float f[8];
        unpack8(pre_b[0], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += f[q];
        unpack8(pre_b[1], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
      }
      if (ep.glu) {
        float g[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) g[q] = v[q] * fast_rcp(1.f + __expf(-v[q])) * v[8 + q];
        *(u32x4_t*)((uint16_t*)C + (int64_t)tid * ldc + (n0 >> 1)) = pack8(g);
        return;
      }
      if (pre_res) {
        float f[8];
        unpack8(pre_r[0], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += f[q];
        unpack8(pre_r[1], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
      }
      const u32x4_t o0 = pack8(v), o1 = pack8(v + 8);
      uint16_t* o = (uint16_t*)C + (int64_t)tid * ldc + n0;
      *(u32x4_t*)o = o0;
      *(u32x4_t*)(o + 8) = o1;
      if (ep.ssq_out) {
        float f[16], t = 0.f;
        unpack8(o0, f);
        unpack8(o1, f + 8);
#pragma unroll
        for (int q = 0; q < 16; ++q) t += f[q] * f[q];
        ep.ssq_out[(int64_t)tid * ep.ssq_tiles + (n0 >> 4)] = t;
      }
    } else {
      GemmEpi e2 = ep;
      e2.norm = 0;   // rstd applied above
      epi_store16_dec(v, 1.f, tid, n0, M, N, C, ldc, e2);
    }
  }
}

// ============================================================================ prefill
template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_w8_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint8_t* __restrict__ W, int64_t ldw,
               const float* __restrict__ scale, void* __restrict__ C, int64_t ldc, int M, int N, int K, GemmEpi ep) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int CA = BM * 8 / NT;  // 16-byte (8-element) chunks per thread
  constexpr int CB = BN * 8 / NT;
  static_assert(CA >= 1 && CB >= 1 && BM * 8 % NT == 0 && BN * 8 % NT == 0, "bad tiling");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;                 // [2][BM][128 B] bf16
  char* sB = smem + 2 * BM * 128;  // [2][BN][128 B] bf16 (widened from fp8)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;

  const uint16_t* pa[CA];
  const uint8_t* pb[CB];
  int la[CA], lb[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int id = tid + i * NT, r = id >> 3, c = id & 7;
    pa[i] = A + (int64_t)min(m0 + r, M - 1) * lda + c * 8;
    la[i] = swz(r, c);
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int id = tid + i * NT, r = id >> 3, c = id & 7;
    pb[i] = W + (int64_t)min(n0 + r, N - 1) * ldw + c * 8;
    lb[i] = swz(r, c);
  }
  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto widen = [](const u32x2_t w) -> u32x4_t { return fp8x8_to_bf16(w[0], w[1]); };
  u32x4_t ra[CA];
  u32x2_t rb[CB];
  const int nk = K / 64;
#pragma unroll
  for (int i = 0; i < CA; ++i) ra[i] = *(const u32x4_t*)(pa[i]);
#pragma unroll
  for (int i = 0; i < CB; ++i) rb[i] = *(const u32x2_t*)(pb[i]);
#pragma unroll
  for (int i = 0; i < CA; ++i) *(u32x4_t*)(sA + la[i]) = ra[i];
#pragma unroll
  for (int i = 0; i < CB; ++i) *(u32x4_t*)(sB + lb[i]) = widen(rb[i]);
  __syncthreads();
  const int frow = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      const int koff = (kt + 1) * 64;
#pragma unroll
      for (int i = 0; i < CA; ++i) ra[i] = *(const u32x4_t*)(pa[i] + koff);
#pragma unroll
      for (int i = 0; i < CB; ++i) rb[i] = *(const u32x2_t*)(pb[i] + koff);
    }
    const char* tA = sA + cur * BM * 128;
    const char* tB = sB + cur * BN * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t fa[MR], fb[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) fa[i] = *(const bf16x8_t*)(tA + swz(wm * TM + i * 16 + frow, s * 4 + fq));
#pragma unroll
      for (int j = 0; j < NR; ++j) fb[j] = *(const bf16x8_t*)(tB + swz(wn * TN + j * 16 + frow, s * 4 + fq));
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      char* nA = sA + (cur ^ 1) * BM * 128;
      char* nB = sB + (cur ^ 1) * BN * 128;
#pragma unroll
      for (int i = 0; i < CA; ++i) *(u32x4_t*)(nA + la[i]) = ra[i];
#pragma unroll
      for (int i = 0; i < CB; ++i) *(u32x4_t*)(nB + lb[i]) = widen(rb[i]);
    }
    __syncthreads();
  }
  // epilogue through LDS, 16-row slabs; the per-channel scale is applied in fp32
  constexpr int LDSTR = TN + 4;
  float* es = (float*)smem + wid * 16 * LDSTR;
  constexpr int LPR = TN / 16;
  constexpr int RPP = 64 / LPR;
  constexpr int NPASS = RPP >= 16 ? 1 : 16 / RPP;
  Unroll<0, MR>::run([&](const int i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) es[(fq * 4 + r) * LDSTR + j * 16 + frow] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int rr = p * RPP + lane / LPR;
      const int cc = (lane % LPR) * 16;
      if (rr < 16) {
        const int n = n0 + wn * TN + cc;
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
          v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] *= n + q < N ? scale[n + q] : 0.f;
        epi_store16(v, m0 + wm * TM + i * 16 + rr, n, M, N, C, ldc, ep);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  });
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_w8(const uint16_t* A, int64_t lda, const uint8_t* W, int64_t ldw, const float* scale, void* C,
                            int64_t ldc, int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  size_t lds = 2 * (size_t)(BM + BN) * 128;
  const size_t epi = (size_t)WM * WN * 16 * (BN / WN + 4) * 4;
  if (epi > lds) lds = epi;
  auto kern = gemm_w8_kernel<BM, BN, WM, WN>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(tiles), dim3(WM * WN * 64), lds, stream, A, lda, W, ldw, scale, C, ldc, M, N, K, ep);
  return hipGetLastError();
}

int skinny_ksplit(int N, int K);

// Decode plan for fp8 weights, 4 < M <= 32 (M <= 4 runs the unsplit row-streaming GEMV):
// M <= 16: column stripes of 64 / 32 / 16 (N divisibility), K split so that stripes x splits
// reach ~512 workgroups (2 per CU), every split >= 4 k blocks (one per wave);
// 16 < M <= 32: 16-column tiles, the skinny split heuristic.
W8DecPlan w8_dec_plan(int M, int N, int K) {
  W8DecPlan p{};
  p.tpw = 1;
  p.ks = 1;
  p.kchunk = K;
  if (M <= 4) return p;
  int ks = 1;
  if (M <= 16) {
    p.tpw = N % 64 == 0 ? 4 : (N % 32 == 0 ? 2 : 1);
    const int stripes = (N + 16 * p.tpw - 1) / (16 * p.tpw);
    ks = (512 + stripes - 1) / stripes;
    const int kmax = K / 256 > 1 ? K / 256 : 1;
    ks = ks < kmax ? ks : kmax;
    int kchunk = (K + ks - 1) / ks;
    kchunk = (kchunk + 63) / 64 * 64;
    p.kchunk = kchunk;
    p.ks = (K + kchunk - 1) / kchunk;
  } else {
    ks = skinny_ksplit(N, K);
    int kchunk = (K + ks - 1) / ks;
    kchunk = (kchunk + 255) / 256 * 256;   // whole 64-wide blocks for every wave
    p.kchunk = kchunk;
    p.ks = (K + kchunk - 1) / kchunk;
  }
  if (p.ks == 1) p.kchunk = K;
  return p;
}

hipError_t gemm_w8(const uint16_t* A, int64_t lda, const uint8_t* W, int64_t ldw, const float* scale, void* C,
                   int64_t ldc, int M, int N, int K, const GemmEpi& ep, float* ws, uint32_t* cnt, int ksplit,
                   hipStream_t stream) {
  if (K % 64 != 0 || M <= 0) return hipErrorInvalidValue;
  if (M <= 4) {   // row-streaming GEMV, non-temporal weight loads
    const dim3 grid((N + 15) / 16);
#define ROWS_LAUNCH(MR_, U_)                                                                                      \
  hipLaunchKernelGGL((gemv_w8_rows_kernel<MR_, U_, true>), grid, dim3(256), 0, stream, A, lda, W, ldw, scale, C, \
                     ldc, M, N, K, ep)
    if (M == 1) ROWS_LAUNCH(1, 2);
    else if (M == 2) ROWS_LAUNCH(2, 2);
    else ROWS_LAUNCH(4, 1);
#undef ROWS_LAUNCH
    return hipGetLastError();
  }
  if (M <= 32) {
    const W8DecPlan pl = w8_dec_plan(M, N, K);
    if (pl.ks > 1 && pl.ks != ksplit) return hipErrorInvalidValue;   // host sized ws / counters for its plan
    const int gy = pl.ks;
    if (gy > 1 && (ws == nullptr || cnt == nullptr)) return hipErrorInvalidValue;
    float* w = gy > 1 ? ws : nullptr;
    if (M <= 16) {
      const dim3 grid((N + 16 * pl.tpw - 1) / (16 * pl.tpw), gy);
#define MFMA_LAUNCH(T_)                                                                                          \
  hipLaunchKernelGGL((gemv_w8_mfma_kernel<T_, 2>), grid, dim3(256), 0, stream, A, lda, W, ldw, scale, C, ldc, w, cnt, \
                     M, N, K, pl.kchunk, ep)
      if (pl.tpw == 4) MFMA_LAUNCH(4);
      else if (pl.tpw == 2) MFMA_LAUNCH(2);
      else MFMA_LAUNCH(1);
#undef MFMA_LAUNCH
    } else {
      hipLaunchKernelGGL((gemm_skinny_w8_kernel<2>), dim3((N + 15) / 16, gy), dim3(256), 0, stream, A, lda, W, ldw,
                         scale, C, ldc, w, cnt, M, N, K, pl.kchunk, ep);
    }
    return hipGetLastError();
  }
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (t128 >= 256) return launch_w8<128, 128, 2, 2>(A, lda, W, ldw, scale, C, ldc, M, N, K, ep, stream);
  return launch_w8<64, 64, 2, 2>(A, lda, W, ldw, scale, C, ldc, M, N, K, ep, stream);
}

}  // namespace lumen
