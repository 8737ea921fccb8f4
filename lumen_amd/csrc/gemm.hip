// bf16 MFMA GEMM with fused epilogues for gfx950.
//
//   C[M, N] = epi( alpha * A[M, K] . W[N, K]^T )
//
// A is row-major activations, W is an nn.Linear-style [out, in] weight, so both
// operand tiles are K-contiguous and every MFMA fragment is one 16-byte
// ds_read_b128 from an XOR-swizzled LDS image (v_mfma_f32_16x16x32_bf16).
//
// Two main loops:
//  * gemm_glds_kernel (256x256x64, 8 waves): LDS-DMA (global_load_lds_dwordx4)
//    staging straight into a lane-linear LDS image whose XOR swizzle is applied
//    on the per-lane *source* address; the K-tile is cut into 4 phases (one
//    64x32 accumulator quadrant per wave each) and the next tile streams in
//    half-tile by half-tile, one half per phase, with counted
//    `s_waitcnt vmcnt(4)` + raw s_barrier so up to 3 half-tiles stay in flight
//    across barriers (never draining to 0 inside the loop).
//  * gemm_bf16_kernel (generic BMxBN, register-staged, 2-stage) for small or
//    odd shapes.
//
// Epilogue (all in fp32 before the single bf16 rounding):
//   v = alpha*acc (+ bias[n]) -> act(v) (+ table[(m % P) + off][n]) (+ residual[orow][n])
// with an optional output row remap  orow = (m / G) * GS + RO + (m % G)  used to
// scatter patch-embedding rows straight into the [B, 1+P, D] token buffer.
// The accumulator goes through LDS so every global store / residual load is a
// coalesced 16-byte access.
//
// Replaces the ONNX-Runtime MatMul/Gemm nodes the reference executes for every
// linear layer (e.g. CLIP vision/text towers, reference
// packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:166,192).
#include "gemm_epi.h"

namespace lumen {

constexpr int BK = 64;  // K elements per tile = 128-byte LDS rows

// ============================================================================
// Generic register-staged kernel
// ============================================================================
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

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

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
#pragma unroll
  for (int i = 0; i < CA; ++i) ra[i] = *(const u32x4_t*)(pa[i]);
#pragma unroll
  for (int i = 0; i < CB; ++i) rb[i] = *(const u32x4_t*)(pb[i]);
#pragma unroll
  for (int i = 0; i < CA; ++i) *(u32x4_t*)(sA + la[i]) = ra[i];
#pragma unroll
  for (int i = 0; i < CB; ++i) *(u32x4_t*)(sB + lb[i]) = rb[i];
  __syncthreads();

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
      for (int i = 0; i < MR; ++i) fa[i] = *(const bf16x8_t*)(tA + swz(wm * TM + i * 16 + frow, s * 4 + fq));
#pragma unroll
      for (int j = 0; j < NR; ++j) fb[j] = *(const bf16x8_t*)(tB + swz(wn * TN + j * 16 + frow, s * 4 + fq));
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

  // epilogue through LDS: one 16-row slab at a time
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
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
          v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
        }
        epi_store16(v, m0 + wm * TM + i * 16 + rr, n0 + wn * TN + cc, M, N, C, ldc, ep);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  });
}

// ============================================================================
// 256x256x64 LDS-DMA phased kernel (8 waves = 2(M) x 4(N))
// ============================================================================
// Wave (wm, wn) owns rows {qm*128 + wm*64 + [0,64)} and cols {qn*128 + wn*32 + [0,32)}
// for quadrants qm, qn in {0,1}: quadrant (qm, qn) reads only A-half qm and
// B-half qn, so half-tiles can be streamed and retired independently.
// LDS: [buf 2][op 2 (A,B)][half 2][128 rows][128 B] = 128 KiB.
constexpr int G_HALF = 128 * 128;       // bytes per half-tile image
constexpr int G_OP = 2 * G_HALF;
constexpr int G_BUF = 2 * G_OP;

__device__ __forceinline__ void vm_wait4() { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
__device__ __forceinline__ void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// MODE 0: 4 phases/K-tile, one half-tile prefetch per phase, counted vmcnt(4) +
//         raw barrier after phases 0, 1, 3.
// MODE 1: MODE 0 + s_setprio(1) around each MFMA cluster.
// MODE 2: whole next tile prefetched at phase 0, one vmcnt(0) + barrier per
//         K-tile (phases free to interleave LDS reads with MFMAs), setprio.
template <int MODE>
__global__ void __launch_bounds__(512)
gemm_glds_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                 void* __restrict__ C, int64_t ldc, int M, int N, int K, GemmEpi ep, int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  const int tiles_n = (N + 255) / 256;
  const int tiles_m = (M + 255) / 256;
  const int bid = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  int tm, tn;
  if (group_m > 1) {
    // each XCD's run of consecutive tiles walks GM row panels x many columns, so
    // the ~32 tiles co-resident on one XCD share both A panels and W panels in L2
    const int span = group_m * tiles_n;
    const int grp = bid / span, first = grp * group_m;
    const int gsz = min(tiles_m - first, group_m);
    const int r = bid % span;
    tm = first + r % gsz;
    tn = r / gsz;
  } else {
    tm = bid / tiles_n;
    tn = bid % tiles_n;
  }
  const int m0 = tm * 256, n0 = tn * 256;

  // ---- staging geometry: half-tile = 16 wave-instructions of 8 rows x 128 B;
  // wave wid issues groups g = 2*wid + i (i = 0, 1).  Lane l writes LDS row
  // g*8 + l/8, physical chunk l%8, so it must fetch logical chunk
  // (l%8) ^ ((row >> 1) & 7): the swizzle lives on the source address.
  const uint16_t* src[2][2][2];  // [op][half][i]
  int dst_off[2];                // LDS byte offset of group (i) inside a half image
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    dst_off[i] = g * 1024;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ra = min(m0 + h * 128 + r, M - 1);
      const int rb = min(n0 + h * 128 + r, N - 1);
      src[0][h][i] = A + (int64_t)ra * lda + c * 8;
      src[1][h][i] = W + (int64_t)rb * ldw + c * 8;
    }
  }
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  auto stage = [&](int op, int h, int buf, int koff) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_global_load_lds((g_ptr_t)(src[op][h][i] + koff),
                                       (lds_ptr_t)(smem + buf * G_BUF + op * G_OP + h * G_HALF + dst_off[i]),
                                       16, 0, 0);
    }
  };

  const int frow = lane & 15, fq = lane >> 4;
  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  // prologue: whole tile 0 in phase order A0, B0, B1, A1
  stage(0, 0, 0, 0);
  stage(1, 0, 0, 0);
  stage(1, 1, 0, 0);
  stage(0, 1, 0, 0);
  if (MODE != 2 && nk > 1) vm_wait4(); else vm_wait0();
  __builtin_amdgcn_s_barrier();

  bf16x8_t fa[4][2], fb[2][2];
  auto load_a = [&](const char* base, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[i][s] = *(const bf16x8_t*)(base + qm * G_HALF + swz(wm * 64 + i * 16 + frow, s * 4 + fq));
  };
  auto load_b = [&](const char* base, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fb[j][s] = *(const bf16x8_t*)(base + G_OP + qn * G_HALF + swz(wn * 32 + j * 16 + frow, s * 4 + fq));
  };

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    const int buf = kt & 1, nbuf = buf ^ 1;
    const int koff = (kt + 1) * BK;
    const char* base = smem + buf * G_BUF;
#define LUMEN_QUAD(QM, QN)                                                                                     \
    if constexpr (MODE >= 1) __builtin_amdgcn_s_setprio(1);                                                    \
    Unroll<0, 4>::run([&](const int i) {                                                                      \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                            \
      _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                            \
        acc[QM][QN][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[QM][QN][i][j], 0, 0, 0); \
    });                                                                                                        \
    if constexpr (MODE >= 1) __builtin_amdgcn_s_setprio(0);
    // ---- phase 0: quadrant (0,0)
    if constexpr (MODE == 2) {
      if (more) { stage(0, 0, nbuf, koff); stage(1, 0, nbuf, koff); stage(1, 1, nbuf, koff); stage(0, 1, nbuf, koff); }
    } else {
      if (more) stage(0, 0, nbuf, koff);
    }
    load_a(base, 0);
    load_b(base, 0);
    LUMEN_QUAD(0, 0)
    if constexpr (MODE != 2) {
      if (more) vm_wait4(); else vm_wait0();   // B1(t) landed
      __builtin_amdgcn_s_barrier();
      if (more) stage(1, 0, nbuf, koff);
    }
    // ---- phase 1: quadrant (0,1)
    load_b(base, 1);
    LUMEN_QUAD(0, 1)
    if constexpr (MODE != 2) {
      if (more) vm_wait4(); else vm_wait0();   // A1(t) landed
      __builtin_amdgcn_s_barrier();
      if (more) stage(1, 1, nbuf, koff);
    }
    // ---- phase 2: quadrant (1,1)
    load_a(base, 1);
    LUMEN_QUAD(1, 1)
    // ---- phase 3: quadrant (1,0)   (B0(t) already resident)
    if constexpr (MODE != 2) {
      if (more) stage(0, 1, nbuf, koff);
    }
    load_b(base, 0);
    LUMEN_QUAD(1, 0)
#undef LUMEN_QUAD
    if constexpr (MODE != 2) {
      if (more) vm_wait4(); else vm_wait0();   // A0(t+1), B0(t+1) landed
    } else {
      vm_wait0();
    }
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: per (qm, i) slab of 16 rows x 64 cols (2 x 32 col groups)
  __syncthreads();
  constexpr int LDSTR = 68;
  float* es = (float*)smem + wid * 16 * LDSTR;
  const int rr = lane >> 2, cq = lane & 3;   // 16 rows x 4 col-chunks of 16
  const int ncol = n0 + (cq >> 1) * 128 + wn * 32 + (cq & 1) * 16;
  Unroll<0, 2>::run([&](const int qm) {
    Unroll<0, 4>::run([&](const int i) {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            es[(fq * 4 + r) * LDSTR + qn * 32 + j * 16 + frow] = acc[qm][qn][i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cq * 16 + q * 4);
        v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      epi_store16(v, m0 + qm * 128 + wm * 64 + i * 16 + rr, ncol, M, N, C, ldc, ep);
    });
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

template <int MODE>
static hipError_t launch_glds(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                              int64_t ldc, int M, int N, int K, const GemmEpi& ep, int group_m, hipStream_t stream) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const size_t lds = 2 * G_BUF;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_glds_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(gemm_glds_kernel<MODE>, dim3(tiles), dim3(512), lds, stream, A, lda, W, ldw, C, ldc, M, N, K, ep,
                     group_m);
  return hipGetLastError();
}

// Host entry: tile choice by problem size.  tile = -1 auto, else forced config id:
//   0 = 256x256 register-staged, 1 = 128x128, 2 = 64x64, 3 = 32x64, 4 = 256x256 LDS-DMA phased
hipError_t gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                     int64_t ldc, int M, int N, int K, const GemmEpi& ep, int tile,
                     hipStream_t stream) {
  bool allow_split = true;          // tile codes >= 1000: same config without the tail-round split
  if (tile >= 1000) { allow_split = false; tile -= 1000; }
  if (tile < 0) {
    const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
    const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
    if (t256 >= 512) tile = 5;
    else if (t128 >= 256) tile = 1;
    else if (M <= 64) tile = 3;
    else tile = 2;
  }
  // tile = config + 10 * group_m (group_m 0 -> default 4 for the 256x256 LDS-DMA kernel)
  int group_m = tile / 10;
  tile = tile % 10;
  if (group_m == 0) group_m = 4;
  if (group_m == 1) group_m = 0;
  // Tail-round split: with one 256x256 workgroup per CU, a tile count just above a
  // multiple of the 256 CUs (ViT batch 512: M = 512*257 -> 514 row tiles -> 2056
  // tiles for N = 1024) leaves a nearly empty last round that still costs a full
  // tile time.  Run the largest row range whose tile count is a multiple of 256 on
  // the 256x256 kernel and the few remaining rows on 128x128 tiles (4x more, 4x
  // shorter workgroups) so the tail costs ~1/4 of a round.  Only for plain row maps.
  if (allow_split && tile >= 4 && tile <= 6 && ep.out_group == 0 && ep.table == nullptr) {
    const int tiles_n = (N + 255) / 256;
    const int tiles_m = (M + 255) / 256;
    int q = 256;
    for (int g = tiles_n; g % 2 == 0 && q > 1; g /= 2) q /= 2;      // q = 256 / gcd(256, tiles_n) (power-of-2 part)
    const int main_m_tiles = tiles_m / q * q;
    const int tail = tiles_m * tiles_n - main_m_tiles * tiles_n;
    if (main_m_tiles > 0 && main_m_tiles < tiles_m && tail < 128) {
      const int M0 = main_m_tiles * 256;
      hipError_t e = gemm_bf16(A, lda, W, ldw, C, ldc, M0, N, K, ep, tile + 10 * (group_m == 0 ? 1 : group_m), stream);
      if (e != hipSuccess) return e;
      GemmEpi e2 = ep;
      if (e2.residual) e2.residual += (int64_t)M0 * e2.ldr;
      char* C2 = (char*)C + (int64_t)M0 * ldc * (ep.out_f32 ? 4 : 2);
      return launch_cfg<128, 128, 2, 2>(A + (int64_t)M0 * lda, lda, W, ldw, C2, ldc, M - M0, N, K, e2, stream);
    }
  }
  switch (tile) {
    case 0: return launch_cfg<256, 256, 2, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 1: return launch_cfg<128, 128, 2, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 2: return launch_cfg<64, 64, 2, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 4: return launch_glds<0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    case 5: return launch_glds<1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    case 6: return launch_glds<2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    default: return launch_cfg<32, 64, 1, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
  }
}

}  // namespace lumen
