// bf16 MFMA GEMM with fused epilogues for gfx950.
//
//   C[M, N] = epi( alpha * A[M, K] . W[N, K]^T )
//
// A is row-major activations, W is an nn.Linear-style [out, in] weight, so both
// operand tiles are K-contiguous and every MFMA fragment is one 16-byte
// ds_read_b128 from an XOR-swizzled LDS image.  The hot loop is the 2-stage
// register-staged pipeline (issue global loads for tile k+1, MFMA tile k from
// LDS, write tile k+1 to the other LDS buffer, one barrier per K-tile).
//
// Epilogue (all in fp32 before the single bf16 rounding):
//   v = alpha*acc (+ bias[n]) -> act(v) (+ table[(m % P) + off][n]) (+ residual[m][n])
// and an optional output row remap  orow = (m / G) * GS + RO + (m % G)  used to
// scatter patch-embedding rows straight into the [B, 1+P, D] token buffer.
// The accumulator tile goes through LDS so every global store / residual load
// is a coalesced 16-byte access.
//
// Replaces the ONNX-Runtime MatMul/Gemm nodes the reference executes for every
// linear layer (e.g. CLIP vision/text towers, reference
// packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:166,192).
#include "common.h"

namespace lumen {

struct GemmEpi {
  const void* bias;          // [N] (f32 if bias_f32 else bf16) or null
  const uint16_t* residual;  // [M, ldr] bf16 or null (indexed by *output* row)
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
};

constexpr int BK = 64;  // K elements per tile = 128-byte LDS rows

__device__ __forceinline__ int swz(int row, int chunk) {
  // 16-byte chunk index XOR row bits 1..3: a 16-lane ds_read_b128 group that
  // reads the same logical chunk of 16 consecutive rows hits 16 distinct
  // 16-byte bank slots (two rows share a 256-B bank row).
  return (row << 7) + (((chunk ^ ((row >> 1) & 7))) << 4);
}

template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_bf16_kernel(const uint16_t* __restrict__ A, int64_t lda,
                 const uint16_t* __restrict__ W, int64_t ldw,
                 void* __restrict__ C, int64_t ldc, int M, int N, int K,
                 GemmEpi ep) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int CA = BM * 8 / NT;  // 16-byte chunks per thread, A tile
  constexpr int CB = BN * 8 / NT;
  static_assert(CA >= 1 && CB >= 1, "tile too small for block");
  static_assert(BM * 8 % NT == 0 && BN * 8 % NT == 0, "bad tiling");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;                       // [2][BM][128B]
  char* sB = smem + 2 * BM * 128;        // [2][BN][128B]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // tile coordinates with XCD-aware remap; n fastest so the blocks that share
  // an A panel run back to back on one XCD.
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // global source pointers for the staging chunks
  const uint16_t* pa[CA];
  const uint16_t* pb[CB];
  int la[CA], lb[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    int id = tid + i * NT, r = id >> 3, c = id & 7;
    int gr = min(m0 + r, M - 1);
    pa[i] = A + (int64_t)gr * lda + c * 8;
    la[i] = swz(r, c);
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    int id = tid + i * NT, r = id >> 3, c = id & 7;
    int gr = min(n0 + r, N - 1);
    pb[i] = W + (int64_t)gr * ldw + c * 8;
    lb[i] = swz(r, c);
  }

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  u32x4_t ra[CA], rb[CB];
  const int nk = K / BK;

  // prologue: tile 0 -> buffer 0
#pragma unroll
  for (int i = 0; i < CA; ++i) ra[i] = *(const u32x4_t*)(pa[i]);
#pragma unroll
  for (int i = 0; i < CB; ++i) rb[i] = *(const u32x4_t*)(pb[i]);
#pragma unroll
  for (int i = 0; i < CA; ++i) *(u32x4_t*)(sA + la[i]) = ra[i];
#pragma unroll
  for (int i = 0; i < CB; ++i) *(u32x4_t*)(sB + lb[i]) = rb[i];
  __syncthreads();

  // per-lane fragment read offsets (row low bits = lane & 15)
  const int frow = lane & 15, fq = lane >> 4;

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      const int koff = (kt + 1) * BK;
#pragma unroll
      for (int i = 0; i < CA; ++i) ra[i] = *(const u32x4_t*)(pa[i] + koff);
#pragma unroll
      for (int i = 0; i < CB; ++i) rb[i] = *(const u32x4_t*)(pb[i] + koff);
    }
    const char* tA = sA + cur * BM * 128;
    const char* tB = sB + cur * BN * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t fa[MR], fb[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        int row = wm * TM + i * 16 + frow;
        fa[i] = *(const bf16x8_t*)(tA + swz(row, s * 4 + fq));
      }
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        int row = wn * TN + j * 16 + frow;
        fb[j] = *(const bf16x8_t*)(tB + swz(row, s * 4 + fq));
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      char* nA = sA + (cur ^ 1) * BM * 128;
      char* nB = sB + (cur ^ 1) * BN * 128;
#pragma unroll
      for (int i = 0; i < CA; ++i) *(u32x4_t*)(nA + la[i]) = ra[i];
#pragma unroll
      for (int i = 0; i < CB; ++i) *(u32x4_t*)(nB + lb[i]) = rb[i];
    }
    __syncthreads();
  }

  // ---------------- epilogue through LDS ----------------
  constexpr int LDSTR = TN + 4;  // floats; +4 breaks the row-to-bank alias
  float* es = (float*)smem + wid * 16 * LDSTR;
  constexpr int LPR = TN / 16;           // lanes per row when each lane owns 16 cols
  constexpr int RPP = 64 / LPR;          // rows per pass (may exceed 16: idle lanes)
  constexpr int NPASS = RPP >= 16 ? 1 : 16 / RPP;
  static_assert(TN % 16 == 0 && 64 % LPR == 0, "epilogue tiling");

  // static unroll over accumulator slabs: acc is only ever indexed by constants
  Unroll<0, MR>::run([&](const int i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) es[(fq * 4 + r) * LDSTR + j * 16 + frow] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int rr = p * RPP + lane / LPR;
      if (rr >= 16) continue;
      const int cc = (lane % LPR) * 16;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
        v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
      }
      const int m = m0 + wm * TM + i * 16 + rr;
      const int n = n0 + wn * TN + cc;
      if (m < M && n < N) {
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
              float f[8];
              unpack8(*(const u32x4_t*)b, f);
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] += f[q];
              unpack8(*(const u32x4_t*)(b + 8), f);
#pragma unroll
              for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
            } else {
#pragma unroll
              for (int q = 0; q < 16; ++q) if (n + q < N) v[q] += bf2f(b[q]);
            }
          }
        }
        if (ep.act) {
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = apply_act(v[q], ep.act);
        }
        int64_t orow = m;
        if (ep.out_group > 0)
          orow = (int64_t)(m / ep.out_group) * ep.out_group_stride + ep.out_row_offset + (m % ep.out_group);
        if (ep.table) {
          const uint16_t* t = ep.table + (int64_t)((m % ep.table_period) + ep.table_offset) * ep.ldt + n;
          if (full) {
            float f[8];
            unpack8(*(const u32x4_t*)t, f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += f[q];
            unpack8(*(const u32x4_t*)(t + 8), f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) if (n + q < N) v[q] += bf2f(t[q]);
          }
        }
        if (ep.residual) {
          const uint16_t* t = ep.residual + orow * ep.ldr + n;
          if (full) {
            float f[8];
            unpack8(*(const u32x4_t*)t, f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += f[q];
            unpack8(*(const u32x4_t*)(t + 8), f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) if (n + q < N) v[q] += bf2f(t[q]);
          }
        }
        if (ep.out_f32) {
          float* o = (float*)C + orow * ldc + n;
          if (full) {
#pragma unroll
            for (int q = 0; q < 4; ++q) *(f32x4_t*)(o + 4 * q) = (f32x4_t){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
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
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  });
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_cfg(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                             void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep,
                             hipStream_t stream) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  size_t lds = 2 * (size_t)(BM + BN) * 128;
  size_t epi = (size_t)WM * WN * 16 * (BN / WN + 4) * 4;
  if (epi > lds) lds = epi;
  auto kern = gemm_bf16_kernel<BM, BN, WM, WN>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(tiles), dim3(WM * WN * 64), lds, stream, A, lda, W, ldw, C, ldc,
                     M, N, K, ep);
  return hipGetLastError();
}

// Host entry: tile choice by problem size.  tile = -1 auto, else forced config id.
hipError_t gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                     int64_t ldc, int M, int N, int K, const GemmEpi& ep, int tile,
                     hipStream_t stream) {
  if (tile < 0) {
    const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
    const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
    if (t256 >= 512) tile = 0;
    else if (t128 >= 256) tile = 1;
    else if (M <= 64) tile = 3;
    else tile = 2;
  }
  switch (tile) {
    case 0: return launch_cfg<256, 256, 2, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 1: return launch_cfg<128, 128, 2, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 2: return launch_cfg<64, 64, 2, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    default: return launch_cfg<32, 64, 1, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
  }
}

}  // namespace lumen
