// 256x256x64 bf16 "ping-pong" MFMA GEMM for gfx950 (tile code 9 of gemm_bf16).
//
//   C[M, N] = epi( alpha * A[M, K] . W[N, K]^T )      (same epilogues as gemm.hip)
//
// 8 waves = 2 (M) x 4 (N); wave (wm, wn) owns rows qm*128 + wm*64 + [0, 64) and columns
// qn*128 + wn*32 + [0, 32) for quadrants qm, qn in {0, 1}, so quadrant (qm, qn) reads only
// A-half qm and B-half qn and the four half-tiles (A0, B0, B1, A1: 128 rows x 128 B each)
// are staged and retired independently by LDS-DMA (global_load_lds_dwordx4, XOR swizzle on
// the per-lane source address, lane-linear LDS image).
//
// Wave group wm = 1 (waves 4-7, one per SIMD) runs ONE BARRIER BEHIND group wm = 0: every
// phase is [ds_read fragments | issue LDS-DMA | counted vmcnt | lgkmcnt(0)] -> s_barrier ->
// MFMA cluster -> s_barrier, so on each SIMD one wave's MFMAs run while its partner reads
// fragments and issues the next staging loads (cdna_hip_programming.md §5, "256² 8-phase
// template": stagger + two barriers per phase, counted vmcnt, raw s_barrier).
//
//  * 4-phase form: one 64x32 quadrant (16 MFMAs) per phase, one half-tile issued per phase.
//  * 2-phase form: one 64x64 half (32 MFMAs) per phase: half the barriers per MFMA.
//
// Hazards (barrier instances counted with group 1 lagging by one): with lgkmcnt(0) ahead of
// each phase's first barrier a buffer region may be restaged one phase after its last read,
// and a region waited for (vmcnt) in phase r may be read from phase r + 1 on, for both groups.
//
// Replaces the ONNX-Runtime MatMul/Gemm nodes of every linear layer (reference
// packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:466-495 runs the CLIP tower
// through them).
#include "gemm_epi.h"

namespace lumen {

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void vm_wait_n() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

// NPH: phases per K-tile (4 or 2).  PRIO 0: s_setprio(1) around every MFMA cluster;
// PRIO 1: static priority 1 for the lagging group (MI355X_MICROARCH "Two waves per SIMD" 4).
template <bool WT, int FK, int PRIO, int NPH>
__global__ void __launch_bounds__(512)
gemm_pp_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
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

  // half-tile h: 0 = A0, 1 = B0, 2 = B1, 3 = A1.  Lane writes LDS row g*8 + l/8, physical
  // chunk l%8, fetching logical chunk (l%8) ^ ((row >> 1) & 7).
  const uint16_t* src[4][2];
  int dst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    const int c = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    dst[i] = g * 1024;
    src[0][i] = A + (int64_t)min(m0 + r, M - 1) * lda + c;
    src[3][i] = A + (int64_t)min(m0 + 128 + r, M - 1) * lda + c;
    src[1][i] = W + (int64_t)min(n0 + r, N - 1) * ldw + c;
    src[2][i] = W + (int64_t)min(n0 + 128 + r, N - 1) * ldw + c;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  auto issue = [&](const int h, int buf, int kt) {
    const int hoff = (h == 1 || h == 2 ? G_OP : 0) + (h >= 2 ? G_HALF : 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((g_ptr_t)(src[h][i] + kt * BK),
                                       (lds_ptr_t)(smem + buf * G_BUF + hoff + dst[i]), 16, 0, 0);
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
  bf16x8_t fa[4][2], fb[2][2][2];   // fb[qn][j][s]
  auto load_a = [&](const char* base, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[i][s] = *(const bf16x8_t*)(base + qm * G_HALF + swz(wm * 64 + i * 16 + frow, s * 4 + fq));
  };
  auto load_b = [&](const char* base, int qn, int slot) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fb[slot][j][s] = *(const bf16x8_t*)(base + G_OP + qn * G_HALF + swz(wn * 32 + j * 16 + frow, s * 4 + fq));
  };

#define LUMEN_PP_CLUSTER(QM, QN, SLOT)                                                                          \
  Unroll<0, 4>::run([&](const int i) {                                                                        \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                              \
    _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                              \
      acc[QM][QN][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[SLOT][j][s], acc[QM][QN][i][j], 0, 0, 0); \
  });
#define LUMEN_PP_SYNC_IN()                                                                                      \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                           \
  pp_barrier();                                                                                                \
  if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#define LUMEN_PP_SYNC_OUT()                                                                                     \
  if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);                                                      \
  pp_barrier();

  const int nk = K / BK;
  if constexpr (NPH == 4) {
    // prologue: tile 0 whole, then A0, B1, A1 of tile 1 (B0(1) goes out at phase 0 of tile 0)
    issue(0, 0, 0);
    issue(1, 0, 0);
    issue(2, 0, 0);
    issue(3, 0, 0);
    if (nk > 1) {
      issue(0, 1, 1);
      issue(2, 1, 1);
      issue(3, 1, 1);
      vm_wait_n<6>();
    } else {
      vm_wait_n<0>();
    }
  } else {
    // prologue: tile 0 whole (A0, B0, B1, A1), then A0, B0, B1 of tile 1 (A1(1) at phase 0)
    issue(0, 0, 0);
    issue(1, 0, 0);
    issue(2, 0, 0);
    issue(3, 0, 0);
    if (nk > 1) {
      issue(0, 1, 1);
      issue(1, 1, 1);
      issue(2, 1, 1);
      vm_wait_n<8>();
    } else {
      vm_wait_n<2>();
    }
  }
  pp_barrier();
  if (wm == 1) pp_barrier();   // the stagger
  if constexpr (PRIO == 1) { if (wm == 1) __builtin_amdgcn_s_setprio(1); }

  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    const char* base = smem + b * G_BUF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    if constexpr (NPH == 4) {
      // phase 0: quadrant (0,0) <- A0, B0; stage B0(t+1)
      load_a(base, 0);
      load_b(base, 0, 0);
      if (n1) issue(1, b ^ 1, kt + 1);
      LUMEN_PP_SYNC_IN()
      LUMEN_PP_CLUSTER(0, 0, 0)
      LUMEN_PP_SYNC_OUT()
      // phase 1: quadrant (0,1) <- B1; stage A0(t+2) (A0(t) last read at phase 0)
      load_b(base, 1, 1);
      if (n2) issue(0, b, kt + 2);
      LUMEN_PP_SYNC_IN()
      LUMEN_PP_CLUSTER(0, 1, 1)
      LUMEN_PP_SYNC_OUT()
      // phase 2: quadrant (1,1) <- A1; stage B1(t+2)
      load_a(base, 1);
      if (n2) issue(2, b, kt + 2);
      LUMEN_PP_SYNC_IN()
      LUMEN_PP_CLUSTER(1, 1, 1)
      LUMEN_PP_SYNC_OUT()
      // phase 3: quadrant (1,0) <- B0 (still in fb slot 0); stage A1(t+2); retire tile t+1
      if (n2) {
        issue(3, b, kt + 2);
        vm_wait_n<6>();
      } else {
        vm_wait_n<0>();
      }
      LUMEN_PP_SYNC_IN()
      LUMEN_PP_CLUSTER(1, 0, 0)
      LUMEN_PP_SYNC_OUT()
    } else {
      // phase 0: rows qm = 0 x all columns <- A0, B0, B1; stage A1(t+1) (A1(t-1) read last
      // phase); retire A1(t)
      load_a(base, 0);
      load_b(base, 0, 0);
      load_b(base, 1, 1);
      if (n1) {
        issue(3, b ^ 1, kt + 1);
        vm_wait_n<8>();
      } else {
        vm_wait_n<0>();
      }
      LUMEN_PP_SYNC_IN()
      LUMEN_PP_CLUSTER(0, 0, 0)
      LUMEN_PP_CLUSTER(0, 1, 1)
      LUMEN_PP_SYNC_OUT()
      // phase 1: rows qm = 1 <- A1 (B fragments kept); stage A0, B0, B1 of t+2 (read last
      // at phase 0); retire A0, B0, B1 of t+1
      load_a(base, 1);
      if (n2) {
        issue(0, b, kt + 2);
        issue(1, b, kt + 2);
        issue(2, b, kt + 2);
        vm_wait_n<8>();
      } else if (n1) {
        vm_wait_n<2>();
      } else {
        vm_wait_n<0>();
      }
      LUMEN_PP_SYNC_IN()
      LUMEN_PP_CLUSTER(1, 0, 0)
      LUMEN_PP_CLUSTER(1, 1, 1)
      LUMEN_PP_SYNC_OUT()
    }
  }
#undef LUMEN_PP_CLUSTER
#undef LUMEN_PP_SYNC_IN
#undef LUMEN_PP_SYNC_OUT
  if constexpr (PRIO == 1) { if (wm == 1) __builtin_amdgcn_s_setprio(0); }
  if (wm == 0) pp_barrier();   // re-align the groups: every LDS read of the K loop is done

  // ---- epilogue: per-wave 16-row slabs through LDS (bias / residual prefetched on the FAST path)
  constexpr int LDSTR = 68;
  float* es = (float*)smem + wid * 16 * LDSTR;
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
  const int rr = lane >> 2, cq = lane & 3;
  const int ncol = n0 + (cq >> 1) * 128 + wn * 32 + (cq & 1) * 16;
  constexpr bool fast = FK > 0;
  constexpr bool FB = fast && ((FK - 1) & 1), FR = fast && ((FK - 1) & 2);
  constexpr int RD = LUMEN_GEMM_RES_PREFETCH;
  u32x4_t bz0 = {0u, 0u, 0u, 0u}, bz1 = {0u, 0u, 0u, 0u};
  u32x4_t rz[RD][2];
  auto res_ptr = [&](int s) {
    return ep.residual + (int64_t)(m0 + (s >> 2) * 128 + wm * 64 + (s & 3) * 16 + rr) * ep.ldr + ncol;
  };
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
  Unroll<0, 8>::run([&](const int s) __attribute__((always_inline)) {
    const int qm = s >> 2, i = s & 3;
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) es[(fq * 4 + r) * LDSTR + qn * 32 + j * 16 + frow] = acc[qm][qn][i][j][r];
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
}

template <bool WT, int FK, int PRIO, int NPH>
static void launch_pp_t(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                        int N, int K, const GemmEpi& ep, int group_m, hipStream_t stream) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const size_t lds = 2 * G_BUF;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_pp_kernel<WT, FK, PRIO, NPH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_pp_kernel<WT, FK, PRIO, NPH>), dim3(tiles), dim3(512), lds, stream, A, lda, W, ldw, C, ldc,
                     M, N, K, ep, group_m);
}

template <int FK>
static void launch_pp_fk(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                         int N, int K, const GemmEpi& ep, int group_m, bool wt, bool prio1, bool two,
                         hipStream_t stream) {
  // write-through stores measured slower on every shape (profiles/r2_gemm_pp_v1.jsonl): not instantiated
  (void)wt;
  if (two) {
    if (prio1) launch_pp_t<false, FK, 1, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    else launch_pp_t<false, FK, 0, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
  } else {
    if (prio1) launch_pp_t<false, FK, 1, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    else launch_pp_t<false, FK, 0, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
  }
}

hipError_t gemm_pp(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                   int N, int K, const GemmEpi& ep, int group_m, int variant, hipStream_t stream) {
  const int64_t extent = (int64_t)M * ldc * (ep.out_f32 ? 4 : 2);
  const bool wt = (variant & 1) && ep.out_group == 0 && extent < ((int64_t)1 << 31);
  const bool fast = M % 256 == 0 && N % 256 == 0 && ep.out_group == 0 && !ep.glu && !ep.table && !ep.prelu &&
                    !ep.post_act && !ep.out_f32 && !(ep.bias && ep.bias_f32) && extent < ((int64_t)1 << 31);
  const int fk = fast ? 1 + (ep.bias ? 1 : 0) + (ep.residual ? 2 : 0) : 0;
  const bool prio1 = (variant & 2) != 0, two = (variant & 4) != 0;
  switch (fk) {
    case 1: launch_pp_fk<1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, stream); break;
    case 2: launch_pp_fk<2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, stream); break;
    case 3: launch_pp_fk<3>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, stream); break;
    case 4: launch_pp_fk<4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, stream); break;
    default: launch_pp_fk<0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, stream); break;
  }
  return hipGetLastError();
}

}  // namespace lumen
