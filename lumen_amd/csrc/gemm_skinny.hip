// Skinny GEMM for decode: C[M, N] = epi(A[M, K] . W[N, K]^T) with M <= 32.
//
// Decode GEMMs are HBM-bound on W (every weight byte is read once per token), so
// the kernel is shaped for bandwidth, not reuse:
//   * a workgroup owns one 16-column N tile and a K range; its 4 waves take
//     interleaved 32-wide k-steps of that range (split-K inside the workgroup,
//     reduced through LDS), and grid.y splits K across workgroups only when the N
//     tiles alone leave CUs idle (skinny_ksplit: N >= 4096 runs unsplit, narrow N such
//     as 896 splits up to ~1024 workgroups; each K-split writes its fp32 partial
//     slab; the last split of a tile to arrive — per-tile atomic counter — sums the
//     slabs in split order — deterministic, so hipGraph replays and eager launches
//     give bitwise-identical logits — and applies the epilogue, with no second
//     kernel launch);
//   * both MFMA operands come straight from global memory in fragment layout:
//     B = W^T (lane: 16 contiguous bytes of weight row n0 + (lane & 15)), A = the
//     activations (L2-resident, shared by every workgroup), 16 rows per MFMA row
//     tile, rows >= M zero;
//   * 4 k-steps are loaded before any MFMA issues (64 B of W in flight per lane).
// The epilogue is the shared GemmEpi (bias / act / residual / SwiGLU / f32 out).
#include <cstdlib>

#include "common.h"
#include "gemm_epi.h"

namespace lumen {

constexpr int SK_UNROLL = 4;

template <int MT>
__global__ void __launch_bounds__(256) gemm_skinny_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                          const uint16_t* __restrict__ W, int64_t ldw,
                                                          void* __restrict__ C, int64_t ldc, float* __restrict__ ws,
                                                          uint32_t* __restrict__ cnt, int M, int N, int K, int kchunk,
                                                          GemmEpi ep) {
  __shared__ float red[4][MT * 16][17];
  __shared__ float rstd_s[MT * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int k_begin = blockIdx.y * kchunk;
  const int k_end = min(K, k_begin + kchunk);
  const int nrow = min(n0 + col, N - 1);
  const uint16_t* wr = W + (int64_t)nrow * ldw + g * 8;
  const uint16_t* ar[MT];
  bool av[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + col;
    av[t] = m < M;
    ar[t] = A + (int64_t)(av[t] ? m : 0) * lda + g * 8;
  }
  f32x4_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // k-steps of 32: wave wid takes steps wid, wid+4, ... (SK_UNROLL at a time)
  const int nsteps = (k_end - k_begin) / 32;
  int s = wid;
  for (; s + 4 * (SK_UNROLL - 1) < nsteps; s += 4 * SK_UNROLL) {
    bf16x8_t wf[SK_UNROLL], af[SK_UNROLL][MT];
#pragma unroll
    for (int u = 0; u < SK_UNROLL; ++u) {
      const int k = k_begin + (s + 4 * u) * 32;
      wf[u] = *(const bf16x8_t*)(wr + k);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        u32x4_t v = *(const u32x4_t*)(ar[t] + k);
        if (!av[t]) v = (u32x4_t){0u, 0u, 0u, 0u};
        af[u][t] = __builtin_bit_cast(bf16x8_t, v);
      }
    }
#pragma unroll
    for (int u = 0; u < SK_UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u][t], wf[u], acc[t], 0, 0, 0);
  }
  for (; s < nsteps; s += 4) {
    const int k = k_begin + s * 32;
    const bf16x8_t wf = *(const bf16x8_t*)(wr + k);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      u32x4_t v = *(const u32x4_t*)(ar[t] + k);
      if (!av[t]) v = (u32x4_t){0u, 0u, 0u, 0u};
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, v), wf, acc[t], 0, 0, 0);
    }
  }
  // C fragment: row (m) = t*16 + 4g + r, column n0 + col
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][t * 16 + 4 * g + r][col] = acc[t][r];
  if (ep.norm) skinny_rstd<4>(A, lda, M, K, ep, rstd_s);
  __syncthreads();
  if (ws != nullptr) {   // K split over grid.y: the last split to arrive reduces + runs the epilogue
    if (!splitk_reduce_last(red, ws, cnt, M, N, n0)) return;
    if (tid < M) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = red[1][tid][c];
      epi_store16_dec(v, rstd_s[tid], tid, n0, M, N, C, ldc, ep);
    }
    return;
  }
  if (tid < MT * 16) {
    const int m = tid;
    if (m < M) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = red[0][m][c] + red[1][m][c] + red[2][m][c] + red[3][m][c];
      epi_store16_dec(v, rstd_s[m], m, n0, M, N, C, ldc, ep);
    }
  }
}

// K split per shape: when the 16-column N tiles already cover every CU (ntiles >= 256,
// all four Llama-3-8B decode GEMMs) the split only adds slab traffic and is skipped;
// narrower N (FastVLM-0.5B: 896 / 1152 wide) splits K until the grid reaches ~target
// workgroups, each keeping >= 512 of K.
int skinny_ksplit(int N, int K) {
  const int ntiles = (N + 15) / 16;
  constexpr int target = 1024;
  constexpr int full = 256;   // tile count that already fills the chip without a split
  if (ntiles >= full) return 1;
  int ks = (target + ntiles - 1) / ntiles;
  const int kmax = K / 512 > 1 ? K / 512 : 1;
  ks = ks < kmax ? ks : kmax;
  ks = ks > 1 ? ks : 1;
  return ks;
}

hipError_t gemm_skinny(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                       int N, int K, const GemmEpi& ep, float* ws, uint32_t* cnt, int ksplit, hipStream_t stream) {
  if (M <= 0 || M > 32 || K % 32 != 0) return hipErrorInvalidValue;
  // K chunk per workgroup: a multiple of 32 * 4 waves
  int kchunk = (K + ksplit - 1) / ksplit;
  kchunk = (kchunk + 127) / 128 * 128;
  const int gy = (K + kchunk - 1) / kchunk;
  dim3 grid((N + 15) / 16, gy), block(256);
  float* w = gy > 1 ? ws : nullptr;
  if (gy > 1 && ws == nullptr) return hipErrorInvalidValue;
  if (gy > 1 && cnt == nullptr) return hipErrorInvalidValue;
  if (M <= 16)
    hipLaunchKernelGGL(gemm_skinny_kernel<1>, grid, block, 0, stream, A, lda, W, ldw, C, ldc, w, cnt, M, N, K, kchunk,
                       ep);
  else
    hipLaunchKernelGGL(gemm_skinny_kernel<2>, grid, block, 0, stream, A, lda, W, ldw, C, ldc, w, cnt, M, N, K, kchunk,
                       ep);
  return hipGetLastError();
}

}  // namespace lumen
