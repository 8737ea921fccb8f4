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

__device__ __forceinline__ void fp8x16_to_bf16(const u32x4_t w, bf16x8_t& f0, bf16x8_t& f1) {
  f0 = __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(w[0], w[1]));
  f1 = __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(w[2], w[3]));
}

// ============================================================================ decode
// UNR: 64-wide k blocks loaded per wave before any MFMA issues; NT: weights streamed with
// non-temporal loads (read once per token; keep L2 for the activations / KV).  NWV waves
// per workgroup split the workgroup's K range: a decode GEMM is a chain of HBM round trips
// per wave (k blocks / UNR of them), so more waves per 16-column tile = fewer round trips
// (measured r2: 4 waves stay best, profiles/r2_w8_skinny_waves_v1.txt).
template <int MT, int W8_UNROLL, bool NT, int NWV = 4>
__global__ void __launch_bounds__(64 * NWV) gemm_skinny_w8_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                             const uint8_t* __restrict__ W, int64_t ldw,
                                                             const float* __restrict__ scale, void* __restrict__ C,
                                                             int64_t ldc, float* __restrict__ ws, uint32_t* __restrict__ cnt, int M, int N, int K,
                                                             int kchunk, GemmEpi ep) {
  __shared__ float red[NWV][MT * 16][17];
  __shared__ float rstd_s[MT * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int k_begin = blockIdx.y * kchunk;
  const int k_end = min(K, k_begin + kchunk);
  const int nrow = min(n0 + col, N - 1);
  const uint8_t* wr = W + (int64_t)nrow * ldw + g * 16;
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

  // 64-wide k blocks: wave wid takes blocks wid, wid + NWV, ... (W8_UNROLL at a time)
  const int nblk = (k_end - k_begin) / 64;
  int s = wid;
  for (; s + NWV * (W8_UNROLL - 1) < nblk; s += NWV * W8_UNROLL) {
    u32x4_t wf[W8_UNROLL];
    u32x4_t af[W8_UNROLL][MT][2];
#pragma unroll
    for (int u = 0; u < W8_UNROLL; ++u) {
      const int k = k_begin + (s + NWV * u) * 64;
      wf[u] = NT ? __builtin_nontemporal_load((const u32x4_t*)(wr + k)) : *(const u32x4_t*)(wr + k);
      load_a(k, af[u]);
    }
#pragma unroll
    for (int u = 0; u < W8_UNROLL; ++u) mma_block(wf[u], af[u]);
  }
  for (; s < nblk; s += NWV) {
    const int k = k_begin + s * 64;
    const u32x4_t wf = NT ? __builtin_nontemporal_load((const u32x4_t*)(wr + k)) : *(const u32x4_t*)(wr + k);
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
      for (int c = 0; c < 16; ++c) v[c] = red[1][tid][c];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] *= n0 + c < N ? scale[n0 + c] : 0.f;
      epi_store16_dec(v, rstd_s[tid], tid, n0, M, N, C, ldc, ep);
    }
    return;
  }
  if (tid < MT * 16) {
    const int m = tid;
    if (m < M) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) t += red[w][m][c];
        v[c] = t * (n0 + c < N ? scale[n0 + c] : 0.f);
      }
      epi_store16_dec(v, rstd_s[m], m, n0, M, N, C, ldc, ep);
    }
  }
}

// Two 16-column tiles per workgroup (unsplit K, M <= 16): the A fragments of each k block feed
// both tiles' MFMAs and every wave keeps twice the weight bytes in flight.  For the widest decode
// GEMMs (Llama-3-8B gate|up: 1792 tiles, lm_head) this halves the workgroup count, so the grid
// fits in one round of resident workgroups instead of 1.2+ (6 per CU at 70 VGPRs).
template <int W8_UNROLL, int NWV = 4>
__global__ void __launch_bounds__(64 * NWV) gemm_skinny_w8x2_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                               const uint8_t* __restrict__ W, int64_t ldw,
                                                               const float* __restrict__ scale, void* __restrict__ C,
                                                               int64_t ldc, int M, int N, int K, GemmEpi ep) {
  __shared__ float red[NWV][16][33];
  __shared__ float rstd_s[16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 32;
  const uint8_t* wr0 = W + (int64_t)min(n0 + col, N - 1) * ldw + g * 16;
  const uint8_t* wr1 = W + (int64_t)min(n0 + 16 + col, N - 1) * ldw + g * 16;
  const bool av = col < M;
  const uint16_t* ar = A + (int64_t)(av ? col : 0) * lda + g * 16;
  f32x4_t acc0 = (f32x4_t){0.f, 0.f, 0.f, 0.f}, acc1 = acc0;

  auto mma2 = [&](const u32x4_t w8, const u32x4_t a0, const u32x4_t a1, f32x4_t& acc) {
    bf16x8_t f0, f1;
    fp8x16_to_bf16(w8, f0, f1);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0), f0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1), f1, acc, 0, 0, 0);
  };
  const int nblk = K / 64;
  int s = wid;
  for (; s + NWV * (W8_UNROLL - 1) < nblk; s += NWV * W8_UNROLL) {
    u32x4_t w0[W8_UNROLL], w1[W8_UNROLL], a0[W8_UNROLL], a1[W8_UNROLL];
#pragma unroll
    for (int u = 0; u < W8_UNROLL; ++u) {
      const int k = (s + NWV * u) * 64;
      w0[u] = *(const u32x4_t*)(wr0 + k);
      w1[u] = *(const u32x4_t*)(wr1 + k);
      a0[u] = av ? *(const u32x4_t*)(ar + k) : (u32x4_t){0u, 0u, 0u, 0u};
      a1[u] = av ? *(const u32x4_t*)(ar + k + 8) : (u32x4_t){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < W8_UNROLL; ++u) {
      mma2(w0[u], a0[u], a1[u], acc0);
      mma2(w1[u], a0[u], a1[u], acc1);
    }
  }
  for (; s < nblk; s += NWV) {
    const int k = s * 64;
    const u32x4_t w0 = *(const u32x4_t*)(wr0 + k), w1 = *(const u32x4_t*)(wr1 + k);
    const u32x4_t a0 = av ? *(const u32x4_t*)(ar + k) : (u32x4_t){0u, 0u, 0u, 0u};
    const u32x4_t a1 = av ? *(const u32x4_t*)(ar + k + 8) : (u32x4_t){0u, 0u, 0u, 0u};
    mma2(w0, a0, a1, acc0);
    mma2(w1, a0, a1, acc1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wid][4 * g + r][col] = acc0[r];
    red[wid][4 * g + r][16 + col] = acc1[r];
  }
  if (ep.norm) skinny_rstd<NWV>(A, lda, M, K, ep, rstd_s);
  __syncthreads();
  if (tid < 2 * 16) {   // thread: (row m, tile tl)
    const int m = tid & 15, tl = tid >> 4;
    const int n = n0 + tl * 16;
    if (m < M && n < N) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) t += red[w][m][tl * 16 + c];
        v[c] = t * (n + c < N ? scale[n + c] : 0.f);
      }
      epi_store16_dec(v, rstd_s[m], m, n, M, N, C, ldc, ep);
    }
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
template <int MR, int U>
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
      for (int r = 0; r < R; ++r) wb[slot][u][r] = *(const u32x4_t*)(wp[r] + ko);
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
    for (int r = 0; r < R; ++r) wb[0][0][r] = *(const u32x4_t*)(wp[r] + ko);
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
    for (int r = 0; r < R; ++r) wb[0][0][r] = *(const u32x4_t*)(wp[r] + ko);
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

hipError_t gemm_w8(const uint16_t* A, int64_t lda, const uint8_t* W, int64_t ldw, const float* scale, void* C,
                   int64_t ldc, int M, int N, int K, const GemmEpi& ep, float* ws, uint32_t* cnt, int ksplit,
                   hipStream_t stream) {
  if (K % 64 != 0 || M <= 0) return hipErrorInvalidValue;
  static const int dec_v = [] {
    const char* e = getenv("LUMEN_W8_DEC");
    return e ? atoi(e) : 1;
  }();
  if (M <= 4 && dec_v > 0) {
    const dim3 grid((N + 15) / 16);
#define ROWS_LAUNCH(MR_, U_)                                                                                      \
  hipLaunchKernelGGL((gemv_w8_rows_kernel<MR_, U_>), grid, dim3(256), 0, stream, A, lda, W, ldw, scale, C, ldc, M, \
                     N, K, ep)
    if (dec_v == 2) {
      if (M == 1) ROWS_LAUNCH(1, 4); else if (M == 2) ROWS_LAUNCH(2, 4); else ROWS_LAUNCH(4, 2);
    } else {
      if (M == 1) ROWS_LAUNCH(1, 2); else if (M == 2) ROWS_LAUNCH(2, 2); else ROWS_LAUNCH(4, 1);
    }
#undef ROWS_LAUNCH
    return hipGetLastError();
  }
  if (M <= 32) {
    // LUMEN_W8_SKINNY: bit 0 = non-temporal weight loads, bit 1 = 8 k blocks per wave in flight;
    // LUMEN_W8_SKINNY_NW: waves per workgroup (4, 8 or 16) for M <= 16; 4 measured fastest
    // (graph-replayed, Llama-3-8B shapes: 8 waves +5-10 %, 16 waves 3-8x slower; r2_w8_skinny_waves_v1.txt)
    static const int variant = [] {
      const char* e = getenv("LUMEN_W8_SKINNY");
      return e ? atoi(e) & 3 : 0;
    }();
    static const int nw_env = [] {
      const char* e = getenv("LUMEN_W8_SKINNY_NW");
      const int v = e ? atoi(e) : 4;
      return v == 8 || v == 16 ? v : 4;
    }();
    const int nwv = M <= 16 ? nw_env : 4;
    int kchunk = (K + ksplit - 1) / ksplit;
    kchunk = (kchunk + 64 * nwv - 1) / (64 * nwv) * (64 * nwv);   // whole 64-wide blocks for every wave
    const int gy = (K + kchunk - 1) / kchunk;
    if (gy > 1 && (ws == nullptr || cnt == nullptr)) return hipErrorInvalidValue;
    dim3 grid((N + 15) / 16, gy), block(64 * nwv);
    float* w = gy > 1 ? ws : nullptr;
#define W8_LAUNCH(MT_, U_, NT_, NW_)                                                                            \
  hipLaunchKernelGGL((gemm_skinny_w8_kernel<MT_, U_, NT_, NW_>), grid, dim3(64 * NW_), 0, stream, A, lda, W, ldw,  \
                     scale, C, ldc, w, cnt, M, N, K, kchunk, ep)
#define W8_NW(U_, NT_)                          \
  switch (nwv) {                                \
    case 8: W8_LAUNCH(1, U_, NT_, 8); break;    \
    case 16: W8_LAUNCH(1, U_, NT_, 16); break;  \
    default: W8_LAUNCH(1, U_, NT_, 4);          \
  }
    (void)block;
    // two tiles per workgroup for wide unsplit GEMMs (LUMEN_W8_NTL=1|2 forces; auto: > 6 tiles per CU)
    static const int ntl_env = [] {
      const char* e = getenv("LUMEN_W8_NTL");
      return e ? atoi(e) : 0;
    }();
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (cus <= 0) cus = 256;
    }
    const int ntiles = (N + 15) / 16;
    const bool x2 = M <= 16 && gy == 1 && variant == 0 && nwv == 4 &&
                    (ntl_env == 2 || (ntl_env == 0 && ntiles > 6 * cus));
    if (x2) {
      hipLaunchKernelGGL((gemm_skinny_w8x2_kernel<4, 4>), dim3((N + 31) / 32), dim3(256), 0, stream, A, lda, W, ldw,
                         scale, C, ldc, M, N, K, ep);
      return hipGetLastError();
    }
    if (M <= 16) {
      switch (variant) {
        case 1: W8_NW(4, true); break;
        case 2: W8_NW(8, false); break;
        case 3: W8_NW(8, true); break;
        default: W8_NW(4, false);
      }
    } else {
      W8_LAUNCH(2, 4, false, 4);
    }
#undef W8_NW
#undef W8_LAUNCH
    return hipGetLastError();
  }
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (t128 >= 256) return launch_w8<128, 128, 2, 2>(A, lda, W, ldw, scale, C, ldc, M, N, K, ep, stream);
  return launch_w8<64, 64, 2, 2>(A, lda, W, ldw, scale, C, ldc, M, N, K, ep, stream);
}

}  // namespace lumen
