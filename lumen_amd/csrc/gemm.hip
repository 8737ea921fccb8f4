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


// Row-coalesced epilogue of the 256x256 kernels (8 waves, wave (wm, wn) holding
// acc[qm][qn][i][j] = rows qm*128 + wm*64 + i*16 + [0,16), cols qn*128 + wn*32 + j*16 +
// [0,16)).  Per 16-row slab the four waves of one wm group scatter their 16 x 64
// pieces into a shared [16][256] fp32 LDS image, then each wave reads back 4 whole
// rows, so 16 consecutive lanes cover one 256-column half-row: every store
// instruction writes 4 rows x 256 contiguous bytes (full 128-B lines).  Writing the
// per-wave 16 x 64 pieces directly (32-B fragments of 32 different lines per store
// instruction) capped the C write stream at ~1.7 TB/s and cost ~15 us per tile.
// Needs 2 x 2 x 16 x 260 x 4 B = 66.5 KiB of free LDS; slabs alternate between two
// images, one barrier per slab.  (Written inline in each kernel: as a helper taking
// the accumulator by reference hipcc keeps `acc` in scratch.)
constexpr int EPI_RS = 260;   // row stride (floats): 4 extra dwords -> conflict-free scatter


// MODE 0: 4 phases/K-tile, one half-tile prefetch per phase, counted vmcnt(4) +
//         raw barrier after phases 0, 1, 3.
// MODE 1: MODE 0 + s_setprio(1) around each MFMA cluster.
// MODE 2: whole next tile prefetched at phase 0, one vmcnt(0) + barrier per
//         K-tile (phases free to interleave LDS reads with MFMAs), setprio.
template <int MODE, int GLU, int EPI>
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
  const int64_t t_start = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

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
  const int64_t t_pro = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

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
#define LM_QUAD(QM, QN)                                                                                     \
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
    LM_QUAD(0, 0)
    if constexpr (MODE != 2) {
      if (more) vm_wait4(); else vm_wait0();   // B1(t) landed
      __builtin_amdgcn_s_barrier();
      if (more) stage(1, 0, nbuf, koff);
    }
    // ---- phase 1: quadrant (0,1)
    load_b(base, 1);
    LM_QUAD(0, 1)
    if constexpr (MODE != 2) {
      if (more) vm_wait4(); else vm_wait0();   // A1(t) landed
      __builtin_amdgcn_s_barrier();
      if (more) stage(1, 1, nbuf, koff);
    }
    // ---- phase 2: quadrant (1,1)
    load_a(base, 1);
    LM_QUAD(1, 1)
    // ---- phase 3: quadrant (1,0)   (B0(t) already resident)
    if constexpr (MODE != 2) {
      if (more) stage(0, 1, nbuf, koff);
    }
    load_b(base, 0);
    LM_QUAD(1, 0)
#undef LM_QUAD
    if constexpr (MODE != 2) {
      if (more) vm_wait4(); else vm_wait0();   // A0(t+1), B0(t+1) landed
    } else {
      vm_wait0();
    }
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue (row-coalesced through LDS)
  __syncthreads();
  const int64_t t_loop = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);   // write-through C stores (host guarantees < 4 GiB of C)
  if constexpr (EPI == 0 || EPI == 3) {
    // per-wave 16-row slabs (each wave stores its own 16 x 64 pieces)
    constexpr int LDSTR = 68;
    float* es = (float*)smem + wid * 16 * LDSTR;
    const int rr = lane >> 2, cq = lane & 3;
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
        epi_store16_t<EPI == 3>(v, m0 + qm * 128 + wm * 64 + i * 16 + rr, ncol, M, N, C, ldc, ep, crs);
      });
    });
  } else {
    const int rrow = wn * 4 + (lane >> 4), rl = lane & 15;
    Unroll<0, 2>::run([&](const int qm) {
      Unroll<0, 4>::run([&](const int i) {
        float* R = (float*)smem + (((qm * 4 + i) & 1) * 2 + wm) * 16 * EPI_RS;
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              R[(fq * 4 + r) * EPI_RS + qn * 128 + wn * 32 + j * 16 + frow] = acc[qm][qn][i][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int m = m0 + qm * 128 + wm * 64 + i * 16 + rrow;
        const float* row = R + rrow * EPI_RS;
        if constexpr (GLU) {   // SwiGLU needs 16 consecutive (interleaved gate|up) columns per lane
          float v[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4_t t = *(const f32x4_t*)(row + rl * 16 + q * 4);
            v[q * 4] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
          }
          epi_store16_t<EPI == 2>(v, m, n0 + rl * 16, M, N, C, ldc, ep, crs);
        } else {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v[8];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const f32x4_t t = *(const f32x4_t*)(row + h * 128 + rl * 8 + q * 4);
              v[q * 4] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
            }
            epi_store8_t<EPI == 2>(v, m, n0 + h * 128 + rl * 8, M, N, C, ldc, ep, crs);
          }
        }
      });
    });
  }
  if (ep.dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int64_t* d = ep.dbg + (int64_t)blockIdx.x * 4;
      d[0] = t_start; d[1] = t_pro; d[2] = t_loop; d[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
  }
}

// ============================================================================
// Persistent 256x256x64 LDS-DMA kernel: one workgroup per CU walks its tiles
// (lin = slot, slot + G, ...) and the staging pipeline never drains between
// tiles — the last K-step of tile t prefetches K-tile 0 of tile t+1, so the
// epilogue (LDS-staged, coalesced stores) of t runs while t+1's first operands
// are already in flight, and its stores drain under t+1's first MFMAs.  With one
// tile per launch-slot instead (gemm_glds_kernel) every CU issues its whole C tile
// in the same instant, then waits a full HBM latency for the next tile's first
// operands: ~15 us per tile at K = 1024, a third of the tile's MFMA time.
// Same phase schedule / counted vmcnt / raw barriers as gemm_glds_kernel<1>.
// ============================================================================

// FK > 0 (FAST): every tile interior (M, N multiples of 256), bf16 output, optional bf16
// bias (FK-1 bit 0) / activation / residual (FK-1 bit 1) -> bias + residual prefetched, no
// bounds checks, and every VMEM count static so hipcc's own waits are exact (chosen on the
// host).  FK = 0: the generic bounds-checked epilogue.
template <bool WT, int FK>
__global__ void __launch_bounds__(512)
gemm_persist_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                    void* __restrict__ C, int64_t ldc, int M, int N, int K, GemmEpi ep, int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = (N + 255) / 256;
  const int tiles_m = (M + 255) / 256;
  const int ntiles = tiles_n * tiles_m;
  const int G = gridDim.x;
  int lin = xcd_remap(blockIdx.x, G);   // concurrent tiles of one XCD are consecutive -> share panels in L2
  if (lin >= ntiles) return;

  // staging geometry (see gemm_glds_kernel): lane writes LDS row g*8 + l/8, physical
  // chunk l%8, fetching logical chunk (l%8) ^ ((row >> 1) & 7)
  int srow[2], scol[2], dst_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    srow[i] = r;
    scol[i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    dst_off[i] = g * 1024;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  auto stageA = [&](int h, int buf, int m0_, int koff) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = min(m0_ + h * 128 + srow[i], M - 1);
      __builtin_amdgcn_global_load_lds((g_ptr_t)(A + (int64_t)row * lda + scol[i] + koff),
                                       (lds_ptr_t)(smem + buf * G_BUF + h * G_HALF + dst_off[i]), 16, 0, 0);
    }
  };
  auto stageB = [&](int h, int buf, int n0_, int koff) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = min(n0_ + h * 128 + srow[i], N - 1);
      __builtin_amdgcn_global_load_lds((g_ptr_t)(W + (int64_t)row * ldw + scol[i] + koff),
                                       (lds_ptr_t)(smem + buf * G_BUF + G_OP + h * G_HALF + dst_off[i]), 16, 0, 0);
    }
  };

  const int frow = lane & 15, fq = lane >> 4;
  const int nk = K / BK;
  int tm, tn;
  tile_coords(lin, tiles_m, tiles_n, group_m, tm, tn);
  int m0 = tm * 256, n0 = tn * 256;
  // prologue: K-tile 0 of the first tile in phase order A0, B0, B1, A1
  stageA(0, 0, m0, 0);
  stageB(0, 0, n0, 0);
  stageB(1, 0, n0, 0);
  stageA(1, 0, m0, 0);
  if (nk > 1 || lin + G < ntiles) vm_wait4(); else vm_wait0();
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

  int buf = 0;
  bool after_epi = false;
  while (true) {
    const int nlin = lin + G;
    const bool has_next = nlin < ntiles;
    int nm0 = 0, nn0 = 0;
    if (has_next) {
      int ntm, ntn;
      tile_coords(nlin, tiles_m, tiles_n, group_m, ntm, ntn);
      nm0 = ntm * 256;
      nn0 = ntn * 256;
    }
    f32x4_t acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      const bool last = kt + 1 == nk;
      const bool more = !last || has_next;
      const int pm0 = last ? nm0 : m0, pn0 = last ? nn0 : n0;
      const int koff = last ? 0 : (kt + 1) * BK;
      const int nbuf = buf ^ 1;
      // First K-step after an epilogue: the epilogue's C stores (>= 16 VMEM ops per wave on
      // the FAST path) are younger than the B1 / A1 loads waited for below, so vmcnt(4)
      // would also wait for most of those stores to be acknowledged; vmcnt(20) waits for
      // exactly the loads (stores and loads share the in-order vmcnt counter).
      const bool relax = FK > 0 && after_epi && kt == 0 && more;
      const char* base = smem + buf * G_BUF;
#define LM_PQUAD(QM, QN)                                                                                    \
      __builtin_amdgcn_s_setprio(1);                                                                           \
      Unroll<0, 4>::run([&](const int i) {                                                                    \
        _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                          \
        _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                          \
          acc[QM][QN][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[QM][QN][i][j], 0, 0, 0); \
      });                                                                                                      \
      __builtin_amdgcn_s_setprio(0);
      // phase 0: quadrant (0,0)
      if (more) stageA(0, nbuf, pm0, koff);
      load_a(base, 0);
      load_b(base, 0);
      LM_PQUAD(0, 0)
      if (relax) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      else if (more) vm_wait4(); else vm_wait0();   // B1 landed
      __builtin_amdgcn_s_barrier();
      if (more) stageB(0, nbuf, pn0, koff);
      // phase 1: quadrant (0,1)
      load_b(base, 1);
      LM_PQUAD(0, 1)
      if (relax) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      else if (more) vm_wait4(); else vm_wait0();   // A1 landed
      __builtin_amdgcn_s_barrier();
      if (more) stageB(1, nbuf, pn0, koff);
      // phase 2: quadrant (1,1)
      load_a(base, 1);
      LM_PQUAD(1, 1)
      // phase 3: quadrant (1,0)
      if (more) stageA(1, nbuf, pm0, koff);
      load_b(base, 0);
      LM_PQUAD(1, 0)
#undef LM_PQUAD
      if (more) vm_wait4(); else vm_wait0();   // next A0, B0 landed
      __builtin_amdgcn_s_barrier();
      buf = nbuf;
    }

    // epilogue through the LDS buffer the last K-step consumed (buf ^ 1); the next
    // tile's first K-tile is landing in `buf` meanwhile.  Every wave finished reading
    // that buffer before the loop's final barrier.
    constexpr int LDSTR = 68;
    float* es = (float*)(smem + (buf ^ 1) * G_BUF) + wid * 16 * LDSTR;
    const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
    const int rr = lane >> 2, cq = lane & 3;
    const int ncol = n0 + (cq >> 1) * 128 + wn * 32 + (cq & 1) * 16;
    // interior tiles with plain epilogues: the bias and the residual rows are prefetched
    // (residual RD slabs ahead) instead of being loaded inside each slab's store
    constexpr bool fast = FK > 0;
    constexpr bool FB = fast && ((FK - 1) & 1), FR = fast && ((FK - 1) & 2);
    constexpr int RD = LM_GEMM_RES_PREFETCH;
    u32x4_t bz0 = {0u, 0u, 0u, 0u}, bz1 = {0u, 0u, 0u, 0u};
    u32x4_t rz[RD][2];
    auto res_ptr = [&](int s) {
      return ep.residual + (int64_t)(m0 + (s >> 2) * 128 + wm * 64 + (s & 3) * 16 + rr) * ep.ldr + ncol;
    };
    if constexpr (fast) {
      if constexpr (FB) {
        bz0 = *(const u32x4_t*)((const uint16_t*)ep.bias + ncol);
        bz1 = *(const u32x4_t*)((const uint16_t*)ep.bias + ncol + 8);
      }
      if constexpr (FR) {
#pragma unroll
        for (int s = 0; s < RD; ++s) {
          rz[s][0] = *(const u32x4_t*)res_ptr(s);
          rz[s][1] = *(const u32x4_t*)(res_ptr(s) + 8);
        }
      }
    }
    Unroll<0, 8>::run([&](const int s) __attribute__((always_inline)) {
      const int qm = s >> 2, i = s & 3;
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
      const int m = m0 + qm * 128 + wm * 64 + i * 16 + rr;
      if constexpr (fast) {
        const u32x4_t r0 = rz[s % RD][0], r1 = rz[s % RD][1];
        if constexpr (FR) {
          if (s + RD < 8) {
            rz[s % RD][0] = *(const u32x4_t*)res_ptr(s + RD);
            rz[s % RD][1] = *(const u32x4_t*)(res_ptr(s + RD) + 8);
          }
        }
        epi_store16_fast<WT, FR>(v, m, ncol, C, ldc, ep, bz0, bz1, r0, r1, crs);
      } else {
        epi_store16_t<WT>(v, m, ncol, M, N, C, ldc, ep, crs);
      }
    });
    if (!has_next) break;
    after_epi = true;
    // the next tile's phase 0 restages this epilogue buffer: all waves' LDS reads first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    lin = nlin;
    m0 = nm0;
    n0 = nn0;
  }
}

// ============================================================================
// 256x256x64 LDS-DMA kernel on a 10-slot half-tile ring (all 160 KiB of LDS)
// ============================================================================
// The K loop is a stream of half-tiles g = 4 kt + h (h: A0, B0, B1, A1), each a
// 128-row x 128-B image in ring slot g % 10.  Half-tile g is issued at phase g - 5,
// i.e. 4-5 phases (one phase = one 64x32 accumulator quadrant per wave, 16 MFMAs)
// before its first read, where the two-buffer kernels above get 2-3: at K = 1024
// with M in the 10^5 range most A rows come from HBM, and that latency, not MFMA
// issue, bounds the two-buffer loop.  Phase P: counted vmcnt for the half-tile it
// reads -> raw barrier -> issue half-tile P + 5 into the slot of P - 5 (last read at
// phase <= P - 3, behind a barrier) -> ds_read fragments -> 16 MFMAs.  Phase 3 of a
// K-step re-reads B0 (landed long ago) and needs neither wait nor barrier.
constexpr int R_SLOTS = 10;
constexpr int R_DIST = 5;
constexpr int R_SLOT = 128 * 128;

__device__ __forceinline__ void vm_wait_halves(int rem) {
  // rem = half-tiles (2 glds each) allowed to remain in flight
  if (rem >= 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (rem == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (rem == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void __launch_bounds__(512)
gemm_ring_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                 void* __restrict__ C, int64_t ldc, int M, int N, int K, GemmEpi ep, int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = (N + 255) / 256;
  const int tiles_m = (M + 255) / 256;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, tiles_n * tiles_m), tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;

  int srow[2], scol[2], dst_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    srow[i] = r;
    scol[i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    dst_off[i] = g * 1024;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  // half-tile g: h = g & 3 -> A0, B0, B1, A1
  auto issue = [&](int g, int slot) {
    const int h = g & 3;
    const int koff = (g >> 2) * BK;
    char* dst = smem + slot * R_SLOT;
    if (h == 0 || h == 3) {
      const int base = m0 + (h == 3 ? 128 : 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = min(base + srow[i], M - 1);
        __builtin_amdgcn_global_load_lds((g_ptr_t)(A + (int64_t)row * lda + scol[i] + koff),
                                         (lds_ptr_t)(dst + dst_off[i]), 16, 0, 0);
      }
    } else {
      const int base = n0 + (h == 2 ? 128 : 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = min(base + srow[i], N - 1);
        __builtin_amdgcn_global_load_lds((g_ptr_t)(W + (int64_t)row * ldw + scol[i] + koff),
                                         (lds_ptr_t)(dst + dst_off[i]), 16, 0, 0);
      }
    }
  };

  const int frow = lane & 15, fq = lane >> 4;
  const int nk = K / BK;
  const int nh = 4 * nk;
  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[4][2], fb[2][2];
  auto load_a = [&](int slot) {
    const char* base = smem + slot * R_SLOT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[i][s] = *(const bf16x8_t*)(base + swz(wm * 64 + i * 16 + frow, s * 4 + fq));
  };
  auto load_b = [&](int slot) {
    const char* base = smem + slot * R_SLOT;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb[j][s] = *(const bf16x8_t*)(base + swz(wn * 32 + j * 16 + frow, s * 4 + fq));
  };

  // prologue: half-tiles 0 .. R_DIST-1
  const int npro = nh < R_DIST ? nh : R_DIST;
#pragma unroll
  for (int g = 0; g < R_DIST; ++g)
    if (g < npro) issue(g, g);
  int last = npro - 1;     // newest half-tile issued
  int islot = npro % R_SLOTS;   // slot of the next half-tile to issue
  int s0 = 0;              // slot of A0 of the current K-step

  for (int kt = 0; kt < nk; ++kt) {
    const int P = 4 * kt;
    const int sA0 = s0, sB0 = s0 + 1 >= R_SLOTS ? s0 + 1 - R_SLOTS : s0 + 1;
    const int sB1 = sB0 + 1 >= R_SLOTS ? sB0 + 1 - R_SLOTS : sB0 + 1;
    const int sA1 = sB1 + 1 >= R_SLOTS ? sB1 + 1 - R_SLOTS : sB1 + 1;
#define LM_RQUAD(QM, QN)                                                                                    \
    __builtin_amdgcn_s_setprio(1);                                                                             \
    Unroll<0, 4>::run([&](const int i) {                                                                      \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                            \
      _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                            \
        acc[QM][QN][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[QM][QN][i][j], 0, 0, 0); \
    });                                                                                                        \
    __builtin_amdgcn_s_setprio(0);
#define LM_RISSUE(PP)                                                                                       \
    if ((PP) + R_DIST < nh) {                                                                                  \
      issue((PP) + R_DIST, islot);                                                                             \
      last = (PP) + R_DIST;                                                                                    \
      islot = islot + 1 == R_SLOTS ? 0 : islot + 1;                                                            \
    }
    // phase 0: quadrant (0,0) needs A0 (P) and B0 (P + 1)
    vm_wait_halves(last - (P + 1));
    __builtin_amdgcn_s_barrier();
    LM_RISSUE(P)
    load_a(sA0);
    load_b(sB0);
    LM_RQUAD(0, 0)
    // phase 1: quadrant (0,1) needs B1 (P + 2)
    vm_wait_halves(last - (P + 2));
    __builtin_amdgcn_s_barrier();
    LM_RISSUE(P + 1)
    load_b(sB1);
    LM_RQUAD(0, 1)
    // phase 2: quadrant (1,1) needs A1 (P + 3)
    vm_wait_halves(last - (P + 3));
    __builtin_amdgcn_s_barrier();
    LM_RISSUE(P + 2)
    load_a(sA1);
    LM_RQUAD(1, 1)
    // phase 3: quadrant (1,0): B0 again (resident), no wait / barrier
    LM_RISSUE(P + 3)
    load_b(sB0);
    LM_RQUAD(1, 0)
#undef LM_RQUAD
#undef LM_RISSUE
    s0 = s0 + 4 >= R_SLOTS ? s0 + 4 - R_SLOTS : s0 + 4;
  }

  // epilogue through LDS (nothing in flight any more: every issued half-tile was read)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  constexpr int LDSTR = 68;
  float* es = (float*)smem + wid * 16 * LDSTR;
  const int rr = lane >> 2, cq = lane & 3;
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

static hipError_t launch_ring(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                              int64_t ldc, int M, int N, int K, const GemmEpi& ep, int group_m, hipStream_t stream) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const size_t lds = (size_t)R_SLOTS * R_SLOT;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_ring_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(gemm_ring_kernel, dim3(tiles), dim3(512), lds, stream, A, lda, W, ldw, C, ldc, M, N, K, ep,
                     group_m);
  return hipGetLastError();
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

template <int MODE, int EPI>
static hipError_t launch_glds_e(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                                int64_t ldc, int M, int N, int K, const GemmEpi& ep, int group_m, hipStream_t stream) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const size_t lds = 2 * G_BUF;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_glds_kernel<MODE, 0, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)gemm_glds_kernel<MODE, 1, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  if (ep.glu)
    hipLaunchKernelGGL((gemm_glds_kernel<MODE, 1, EPI>), dim3(tiles), dim3(512), lds, stream, A, lda, W, ldw, C, ldc, M,
                       N, K, ep, group_m);
  else
    hipLaunchKernelGGL((gemm_glds_kernel<MODE, 0, EPI>), dim3(tiles), dim3(512), lds, stream, A, lda, W, ldw, C, ldc, M,
                       N, K, ep, group_m);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_glds(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                              int64_t ldc, int M, int N, int K, const GemmEpi& ep, int group_m, int epi,
                              hipStream_t stream) {
  switch (epi) {
    case 1: return launch_glds_e<MODE, 1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    case 2: return launch_glds_e<MODE, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    case 3: return launch_glds_e<MODE, 3>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    default: return launch_glds_e<MODE, 0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
  }
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

// wt: write-through (sc1) C stores via a buffer descriptor (C extent < 2 GiB: 32-bit offsets)
template <bool WT, int FK>
static void launch_persist_t(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc,
                             int M, int N, int K, const GemmEpi& ep, int group_m, int grid, size_t lds,
                             hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_persist_kernel<WT, FK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_persist_kernel<WT, FK>), dim3(grid), dim3(512), lds, stream, A, lda, W, ldw, C, ldc, M, N,
                     K, ep, group_m);
}

template <bool WT>
static void launch_persist_fk(int fk, const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                              int64_t ldc, int M, int N, int K, const GemmEpi& ep, int group_m, int grid, size_t lds,
                              hipStream_t stream) {
  switch (fk) {
    case 1: return launch_persist_t<WT, 1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
    case 2: return launch_persist_t<WT, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
    case 3: return launch_persist_t<WT, 3>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
    case 4: return launch_persist_t<WT, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
    default: return launch_persist_t<WT, 0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
  }
}

static hipError_t launch_persist(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                                 int64_t ldc, int M, int N, int K, const GemmEpi& ep, int group_m, bool wt,
                                 hipStream_t stream) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int grid = tiles < num_cus() ? tiles : num_cus();
  const size_t lds = 2 * G_BUF;
  const int64_t extent = (int64_t)M * ldc * (ep.out_f32 ? 4 : 2);
  wt = wt && ep.out_group == 0 && extent < ((int64_t)1 << 31);
  const bool fast = M % 256 == 0 && N % 256 == 0 && ep.out_group == 0 && !ep.glu && !ep.table && !ep.prelu &&
                    !ep.post_act && !ep.out_f32 && !(ep.bias && ep.bias_f32) && extent < ((int64_t)1 << 31);
  const int fk = fast && !ep.row_aff ? 1 + (ep.bias ? 1 : 0) + (ep.residual ? 2 : 0) : 0;
  if (wt) launch_persist_fk<true>(fk, A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
  else launch_persist_fk<false>(fk, A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, grid, lds, stream);
  return hipGetLastError();
}

// Host entry: tile choice by problem size.  tile = -1 auto, else forced config id
// (+ 10 * group_m + 100 * epilogue variant + 1000 to disable the tail split):
//   0 = 256x256 register-staged, 1 = 128x128, 2 = 64x64, 3 = 32x64, 4 = 256x256 LDS-DMA phased,
//   5 = 4 + setprio, 6 = one wait per K-tile, 7 = persistent 256x256 (cross-tile prefetch),
//   8 = 256x256 on the 10-slot half-tile ring (deeper prefetch), 9 = 256x256 ping-pong (gemm_pp.hip;
//   hundreds digit = variant: bit 0 persistent, bit 1 static priority for the lagging group, bit 2 two
//   phases per K-tile)
hipError_t gemm_lds128_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc,
                            int M, int N, int K, const GemmEpi& ep, int variant, hipStream_t stream);

// tile codes 20000 + v: the 128x128 LDS-DMA pipeline of gemm_f8.hip on bf16 operands
// (v = 0 auto, 1..5 stage / wave variants)
hipError_t gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                     int64_t ldc, int M, int N, int K, const GemmEpi& ep, int tile,
                     hipStream_t stream) {
  if (tile >= 20000) return gemm_lds128_bf16(A, lda, W, ldw, C, ldc, M, N, K, ep, tile - 20000, stream);
  bool allow_split = true;          // tile codes >= 1000: same config without the tail-round split
  if (tile >= 1000) { allow_split = false; tile -= 1000; }
  if (tile < 0) {
    const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
    const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
    // measured on MI355X (tools/gemm_bench.py, random bf16, profiles/r1_gemm_epilogue_ab_v1.jsonl):
    // K <= 512: row-coalesced write-through epilogue (+25-30 %); K 1024-2048: persistent
    // kernel (+4-8 %); K >= 4096: per-wave epilogue LDS-DMA kernel
    // r2: the ping-pong kernel (gemm_pp.hip, two phases per K-tile, static priority for the
    // lagging wave group) beats all of these at K >= 1024 (profiles/r2_gemm_pp_v2.jsonl)
    // residual epilogues at K <= 2048 run the persistent form (next tile's operands stream in
    // during the residual-reading epilogue: +2-7 %, profiles/r2_gemm_pps_phase_v1.txt)
    // r2 mid-size shapes (a few hundred to a few thousand rows, profiles/r2_gemm_mid_lds128_v1.jsonl): the
    // 128x128 LDS-DMA pipeline (gemm_f8.hip, bf16 form) beats the register-staged 128x128 / 64x64 tiles
    // once there are ~150+ 128x128 tiles; fewer tiles (e.g. 577 x 1024 x 4096) stay on 64x64
    const bool lds_ok = K % 64 == 0 && N % 16 == 0 && lda % 8 == 0 && ldw % 8 == 0 &&
                        ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0;
    if (t256 >= 512) tile = K <= 512 ? 245 : (ep.residual && K <= 2048 && M % 256 == 0 && N % 256 == 0 ? 709 : 609);
    else if (t128 >= 256) tile = lds_ok ? 20000 : 1;
    // few rows over a deep K (the IResNet embedding FC at 64 faces: 64 x 512 x 25088 took 268 us as
    // 16 register-staged 32x64 tiles): the LDS-DMA pipeline with K split over gridDim.y streams W once
    else if (M <= 64 && !(lds_ok && K >= 4096)) tile = 3;
    else if (M <= 64) tile = 20000;
    // (r4, cold weights: 577 x 4096 x 1024 + quick_gelu 17.5 us as <4 stages, 8 waves> vs 21.9 us as
    // <2, 8>, profiles/r4_cold_vit_gemm_variants_v1.txt)
    else if (t128 >= 144 && lds_ok) tile = 20003;
    // fewer 128x128 tiles (VLM vision tower at 577 tokens: 40-120): the same pipeline with K split
    // over gridDim.y + one reduce/epilogue pass (gemm_f8.hip f8_pick_splits) instead of 64x64 tiles
    else if (lds_ok && M >= 128 && K >= 4096) tile = 20000;
    else tile = 2;
    if (tile >= 20000) return gemm_lds128_bf16(A, lda, W, ldw, C, ldc, M, N, K, ep, tile - 20000, stream);
  }
  // tile = config + 10 * group_m + 100 * epilogue (group_m 0 -> default 4 for the 256x256 LDS-DMA kernel;
  // epilogue 0 = per-wave slabs, 1 = row-coalesced, 2 = row-coalesced write-through, 3 = per-wave write-through)
  const int epi = (tile / 100) % 10;
  int group_m = (tile / 10) % 10;
  tile = tile % 10;
  if (group_m == 0) group_m = 4;
  if (group_m == 1) group_m = 0;
  // Tail-round split: with one 256x256 workgroup per CU, a tile count just above a
  // multiple of the 256 CUs (ViT batch 512: M = 512*257 -> 514 row tiles -> 2056
  // tiles for N = 1024) leaves a nearly empty last round that still costs a full
  // tile time.  Run the largest row range whose tile count is a multiple of 256 on
  // the 256x256 kernel and the few remaining rows on 128x128 tiles (4x more, 4x
  // shorter workgroups) so the tail costs ~1/4 of a round.  Only for plain row maps.
  if (allow_split && tile >= 4 && tile <= 9 && ep.out_group == 0 && ep.table == nullptr) {
    const int tiles_n = (N + 255) / 256;
    const int tiles_m = (M + 255) / 256;
    int q = 256;
    for (int g = tiles_n; g % 2 == 0 && q > 1; g /= 2) q /= 2;      // q = 256 / gcd(256, tiles_n) (power-of-2 part)
    const int main_m_tiles = tiles_m / q * q;
    const int tail = tiles_m * tiles_n - main_m_tiles * tiles_n;
    if (main_m_tiles > 0 && main_m_tiles < tiles_m && tail < 128) {
      const int M0 = main_m_tiles * 256;
      hipError_t e = gemm_bf16(A, lda, W, ldw, C, ldc, M0, N, K, ep, tile + 10 * (group_m == 0 ? 1 : group_m) + 100 * epi,
                               stream);
      if (e != hipSuccess) return e;
      GemmEpi e2 = ep;
      if (e2.residual) e2.residual += (int64_t)M0 * e2.ldr;
      // every per-A-row epilogue operand follows the row shift (LN-folded row stats, RMS sums)
      if (e2.row_aff) e2.row_aff += 2 * (int64_t)M0;
      if (e2.ssq_in) e2.ssq_in += (int64_t)M0 * e2.ssq_tiles;
      if (e2.ssq_out) e2.ssq_out += (int64_t)M0 * e2.ssq_tiles;
      char* C2 = (char*)C + (int64_t)M0 * ldc * (ep.out_f32 ? 4 : 2);
      // tail rows: split-K ping-pong + reduce/epilogue pass (r2: the 128x128 register-staged
      // tail took 9.5 % of the ViT-L/14 step for 0.4 % of its FLOPs)
      if (gemm_tail_splitk(A + (int64_t)M0 * lda, lda, W, ldw, C2, ldc, M - M0, N, K, e2, stream) == hipSuccess)
        return hipSuccess;
      (void)hipGetLastError();
      return launch_cfg<128, 128, 2, 2>(A + (int64_t)M0 * lda, lda, W, ldw, C2, ldc, M - M0, N, K, e2, stream);
    }
  }
  if ((tile >= 4 && tile <= 6) || tile == 9) {
    // the 256x256 LDS-DMA kernels store C through a 32-bit-offset buffer descriptor
    const int64_t last_row = ep.out_group > 0 ? (int64_t)((M - 1) / ep.out_group) * ep.out_group_stride +
                                                    ep.out_row_offset + (M - 1) % ep.out_group
                                              : (int64_t)M - 1;
    const int64_t extent = ((last_row + 1) * ldc) * (ep.out_f32 ? 4 : 2);
    if (extent >= ((int64_t)1 << 32)) tile = 1;
  }
  switch (tile) {
    case 0: return launch_cfg<256, 256, 2, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 1: return launch_cfg<128, 128, 2, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 2: return launch_cfg<64, 64, 2, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
    case 4: return launch_glds<0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, epi, stream);
    case 5: return launch_glds<1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, epi, stream);
    case 6: return launch_glds<2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, epi, stream);
    case 7: return launch_persist(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, epi == 3, stream);
    case 8: return launch_ring(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    case 9: return gemm_pp(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, epi, stream);
    default: return launch_cfg<32, 64, 1, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, stream);
  }
}

}  // namespace lumen
