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
