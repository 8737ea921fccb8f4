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
#include "workspace.h"

#include <cstdlib>

namespace lumen {

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Direct-store epilogue (DS kernels): the lane holds row m0 + qm*128 + wm*64 + i*16 + (lane & 15),
// columns n0 + qn*128 + wn*32 + 8*(lane >> 4) + [0, 8) in acc[qm][qn][i][0..1][0..3]; 16 passes of one
// 16-byte store each.  Bias / residual / LN-fold operands are loaded up front (residual RD passes ahead).
template <bool WT, int FK>
__device__ __forceinline__ void pp_epilogue_direct(const f32x4_t (&acc)[2][2][4][2], int m0, int n0, int M, int N,
                                                   void* __restrict__ C, int64_t ldc, const GemmEpi& ep, int wm,
                                                   int wn, int lane, const float* aff_lds = nullptr) {
  constexpr bool FL = FK == 5;
  constexpr bool fast = FK > 0 && !FL;
  constexpr bool FB = fast && ((FK - 1) & 1), FR = fast && ((FK - 1) & 2);
  constexpr int RD = LM_GEMM_RES_PREFETCH;   // residual passes in flight
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
  const int fr = lane & 15, fc = lane >> 4;
  auto col_of = [&](int qn) { return n0 + qn * 128 + wn * 32 + fc * 8; };
  auto row_of = [&](int p) { return m0 + (p >> 3) * 128 + wm * 64 + ((p >> 1) & 3) * 16 + fr; };
  u32x4_t bq[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  u32x4_t rz[RD];
  if constexpr (FB) {
    bq[0] = *(const u32x4_t*)((const uint16_t*)ep.bias + col_of(0));
    bq[1] = *(const u32x4_t*)((const uint16_t*)ep.bias + col_of(1));
  }
  if constexpr (FR) {
#pragma unroll
    for (int p = 0; p < RD; ++p) rz[p] = *(const u32x4_t*)(ep.residual + (int64_t)row_of(p) * ep.ldr + col_of(p & 1));
  }
  float lcs[FL ? 16 : 1], lcb[FL ? 16 : 1], lrs[FL ? 8 : 1], lro[FL ? 8 : 1];
  if constexpr (FL) {
    if (aff_lds) {   // staged by the kernel ahead of its K loop: [col scale 256 | col shift 256 | rstd 256 | -mean*rstd 256]
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = col_of(qn) - n0 + 4 * h;
          const f32x4_t a = *(const f32x4_t*)(aff_lds + c);
          const f32x4_t b = *(const f32x4_t*)(aff_lds + 256 + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            lcs[qn * 8 + 4 * h + e] = a[e];
            lcb[qn * 8 + 4 * h + e] = b[e];
          }
        }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int lr = row_of(2 * r) - m0;
        lrs[r] = aff_lds[512 + lr];
        lro[r] = aff_lds[768 + lr];
      }
    } else {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4_t a = *(const f32x4_t*)(ep.col_aff + col_of(qn) + 4 * h);
          const f32x4_t b = *(const f32x4_t*)(ep.col_aff + N + col_of(qn) + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            lcs[qn * 8 + 4 * h + e] = a[e];
            lcb[qn * 8 + 4 * h + e] = b[e];
          }
        }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int64_t m = row_of(2 * r);
        lrs[r] = ep.row_aff[2 * m];
        lro[r] = ep.row_aff[2 * m + 1];
      }
    }
  }
  Unroll<0, 16>::run([&](const int p) __attribute__((always_inline)) {
    const int qm = p >> 3, i = (p >> 1) & 3, qn = p & 1;
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = acc[qm][qn][i][0][r];
      v[4 + r] = acc[qm][qn][i][1][r];
    }
    const int m = row_of(p), n = col_of(qn);
    if constexpr (FL) {
      epi_store_lnf<WT, 8>(v, m, n, C, ldc, ep, lrs[p >> 1], lro[p >> 1], lcs + qn * 8, lcb + qn * 8, crs);
    } else if constexpr (fast) {
      float f[8];
      unpack8(bq[qn], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] * ep.alpha + f[q];
      if (ep.act) apply_act_n<8>(v, ep.act);
      if constexpr (FR) {
        unpack8(rz[p % RD], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += f[q];
        if (p + RD < 16) rz[p % RD] = *(const u32x4_t*)(ep.residual + (int64_t)row_of(p + RD) * ep.ldr + col_of((p + RD) & 1));
      }
      st16<WT>(C, crs, ((int64_t)m * ldc + n) * 2, pack8(v));
    } else {
      epi_store8_t<WT>(v, m, n, M, N, C, ldc, ep, crs);
    }
  });
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
// DS: direct-store epilogue (gemm_epi.h swzb): transposed accumulators, 16-byte stores straight
// from registers, no LDS staging (no SwiGLU).
template <bool WT, int FK, int PRIO, int NPH, bool DS = false>
__global__ void __launch_bounds__(512)
gemm_pp_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
               void* __restrict__ C, int64_t ldc, int M, int N, int K, GemmEpi ep, int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t_start = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = (N + 255) / 256;
  const int tiles_m = (M + 255) / 256;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, tiles_n * tiles_m), tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  if (ep.split_koff) {   // split-K: this workgroup's K slice and fp32 slab
    A += blockIdx.y * ep.split_koff;
    W += blockIdx.y * ep.split_koff;
    C = (float*)C + blockIdx.y * ep.split_cstride;
  }

  // half-tile h: 0 = A0, 1 = B0, 2 = B1, 3 = A1.  Lane writes LDS row g*8 + l/8, physical
  // chunk l%8, fetching logical chunk (l%8) ^ ((row >> 1) & 7).
  const uint16_t* src[4][2];
  int dst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    const int c = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    const int cb = DS ? ((lane & 7) ^ ds_bxor(r)) * 8 : c;
    dst[i] = g * 1024;
    src[0][i] = A + (int64_t)min(m0 + r, M - 1) * lda + c;
    src[3][i] = A + (int64_t)min(m0 + 128 + r, M - 1) * lda + c;
    src[1][i] = W + (int64_t)min(n0 + r, N - 1) * ldw + cb;
    src[2][i] = W + (int64_t)min(n0 + 128 + r, N - 1) * ldw + cb;
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
        fb[slot][j][s] = *(const bf16x8_t*)(base + G_OP + qn * G_HALF +
                                             (DS ? swzb(wn * 32 + 8 * (frow >> 2) + 4 * j + (frow & 3), s * 4 + fq)
                                                 : swz(wn * 32 + j * 16 + frow, s * 4 + fq)));
  };

#define LM_PP_CLUSTER(QM, QN, SLOT)                                                                          \
  Unroll<0, 4>::run([&](const int i) {                                                                        \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                              \
    _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                              \
      acc[QM][QN][i][j] = DS ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[SLOT][j][s], fa[i][s], acc[QM][QN][i][j], 0, 0, 0) \
                             : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[SLOT][j][s], acc[QM][QN][i][j], 0, 0, 0); \
  });
#define LM_PP_SYNC_IN()                                                                                      \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                           \
  pp_barrier();                                                                                                \
  if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#define LM_PP_SYNC_OUT()                                                                                     \
  if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);                                                      \
  pp_barrier();

  // direct store + LN fold: the epilogue's column / row affine operands staged in LDS past the pipeline
  // buffers, loaded ahead of the K loop -- loaded after it, their round trip sat between the last MFMA
  // and the first store of every tile
  constexpr bool PRE = DS && FK == 5;
  float* aff_lds = (float*)(smem + 2 * G_BUF);
  float pre0 = 0.f, pre1 = 0.f;
  if constexpr (PRE) {
    if (tid < 256) {
      pre0 = ep.col_aff[n0 + tid];
      pre1 = ep.col_aff[N + n0 + tid];
    } else {
      const int64_t r = m0 + tid - 256;
      pre0 = ep.row_aff[2 * r];
      pre1 = ep.row_aff[2 * r + 1];
    }
    asm volatile("" ::: "memory");   // issued before the prologue's staging loads
  }
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
  if constexpr (PRE) {   // older than every staging load: landed by the wait above
    aff_lds[(tid & 255) + (tid < 256 ? 0 : 512)] = pre0;
    aff_lds[(tid & 255) + (tid < 256 ? 256 : 768)] = pre1;
  }
  pp_barrier();
  const int64_t t_pro = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
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
      LM_PP_SYNC_IN()
      LM_PP_CLUSTER(0, 0, 0)
      LM_PP_SYNC_OUT()
      // phase 1: quadrant (0,1) <- B1; stage A0(t+2) (A0(t) last read at phase 0)
      load_b(base, 1, 1);
      if (n2) issue(0, b, kt + 2);
      LM_PP_SYNC_IN()
      LM_PP_CLUSTER(0, 1, 1)
      LM_PP_SYNC_OUT()
      // phase 2: quadrant (1,1) <- A1; stage B1(t+2)
      load_a(base, 1);
      if (n2) issue(2, b, kt + 2);
      LM_PP_SYNC_IN()
      LM_PP_CLUSTER(1, 1, 1)
      LM_PP_SYNC_OUT()
      // phase 3: quadrant (1,0) <- B0 (still in fb slot 0); stage A1(t+2); retire tile t+1
      if (n2) {
        issue(3, b, kt + 2);
        vm_wait_n<6>();
      } else {
        vm_wait_n<0>();
      }
      LM_PP_SYNC_IN()
      LM_PP_CLUSTER(1, 0, 0)
      LM_PP_SYNC_OUT()
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
      LM_PP_SYNC_IN()
      LM_PP_CLUSTER(0, 0, 0)
      LM_PP_CLUSTER(0, 1, 1)
      LM_PP_SYNC_OUT()
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
      LM_PP_SYNC_IN()
      LM_PP_CLUSTER(1, 0, 0)
      LM_PP_CLUSTER(1, 1, 1)
      LM_PP_SYNC_OUT()
    }
  }
#undef LM_PP_CLUSTER
#undef LM_PP_SYNC_IN
#undef LM_PP_SYNC_OUT
  if constexpr (PRIO == 1) { if (wm == 1) __builtin_amdgcn_s_setprio(0); }
  if (wm == 0) pp_barrier();   // re-align the groups: every LDS read of the K loop is done
  const int64_t t_loop = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

  if constexpr (DS) {
    pp_epilogue_direct<WT, FK>(acc, m0, n0, M, N, C, ldc, ep, wm, wn, lane, PRE ? aff_lds : nullptr);
  } else {
  // ---- epilogue: per-wave 16-row slabs through LDS (bias / residual prefetched on the FAST path)
  constexpr int LDSTR = 68;
  float* es = (float*)smem + wid * 16 * LDSTR;
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
  const int rr = lane >> 2, cq = lane & 3;
  const int ncol = n0 + (cq >> 1) * 128 + wn * 32 + (cq & 1) * 16;
  constexpr bool FL = FK == 5;   // LN-folded row / column affine (GemmEpi::row_aff), no residual
  constexpr bool fast = FK > 0 && !FL;
  constexpr bool FB = fast && ((FK - 1) & 1), FR = fast && ((FK - 1) & 2);
  constexpr int RD = LM_GEMM_RES_PREFETCH;
  u32x4_t bz0 = {0u, 0u, 0u, 0u}, bz1 = {0u, 0u, 0u, 0u};
  u32x4_t rz[RD][2];
  float lcs[FL ? 16 : 1], lcb[FL ? 16 : 1], lrs[FL ? 8 : 1], lro[FL ? 8 : 1];
  if constexpr (FL) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4_t a = *(const f32x4_t*)(ep.col_aff + ncol + 4 * q);
      const f32x4_t b = *(const f32x4_t*)(ep.col_aff + N + ncol + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lcs[4 * q + e] = a[e];
        lcb[4 * q + e] = b[e];
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int64_t m = m0 + (s >> 2) * 128 + wm * 64 + (s & 3) * 16 + rr;
      lrs[s] = ep.row_aff[2 * m];
      lro[s] = ep.row_aff[2 * m + 1];
    }
  }
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
    if constexpr (FL) {
      epi_store_lnf<WT, 16>(v, m, ncol, C, ldc, ep, lrs[s], lro[s], lcs, lcb, crs);
    } else if constexpr (fast) {
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
  if (ep.dbg && tid == 0) {   // profiling (tools/gemm_timeline.py): wave 0's view of the tile
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int64_t* d = ep.dbg + 4 * (int64_t)blockIdx.x;
    d[0] = t_start; d[1] = t_pro; d[2] = t_loop; d[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
}

template <bool WT, int FK, int PRIO, int NPH, bool DS = false>
static void launch_pp_t(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                        int N, int K, const GemmEpi& ep, int group_m, hipStream_t stream, int splits = 1) {
  const dim3 tiles(((M + 255) / 256) * ((N + 255) / 256), splits);
  const size_t lds = 2 * G_BUF + (DS && FK == 5 ? 4096 : 0);   // + the LN-fold affine stage
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_pp_kernel<WT, FK, PRIO, NPH, DS>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_pp_kernel<WT, FK, PRIO, NPH, DS>), dim3(tiles), dim3(512), lds, stream, A, lda, W, ldw,
                     C, ldc, M, N, K, ep, group_m);
}

template <int FK>
static void launch_pp_fk(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                         int N, int K, const GemmEpi& ep, int group_m, bool wt, bool prio1, bool two, bool ds,
                         hipStream_t stream) {
  // write-through stores measured slower on every shape (profiles/r2_gemm_pp_v1.jsonl): not instantiated
  (void)wt;
  if (ds) {   // direct-store epilogue: the production two-phase, static-priority form only
    // (r5 A/Bs, profiles/r5_gemm_pp_ds_v1.txt: write-through C stores and 8 / 16 residual rows in flight
    // both lost to plain stores with 4 rows in flight; those variants were removed in r6)
    launch_pp_t<false, FK, 1, 2, true>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    return;
  }
  if (two) {
    if (prio1) launch_pp_t<false, FK, 1, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    else launch_pp_t<false, FK, 0, 2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
  } else {
    if (prio1) launch_pp_t<false, FK, 1, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
    else launch_pp_t<false, FK, 0, 4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);
  }
}

// ============================================================================
// Persistent form of the 2-phase ping-pong kernel (interior tiles: M, N multiples of 256,
// K / 64 >= 2).  One workgroup per CU walks tiles lin, lin + G, ... as ONE continuous
// stream of K-tiles ("units"): the LDS-DMA staging of units u + 1 / u + 2 runs across tile
// boundaries, so the next tile's first operands land while an epilogue runs.
//
// (A phase-shifted variant -- each workgroup starting part-way into its first tile so the
// 256 C-write bursts spread over the tile period -- measured slower on the ViT-L/14 shapes:
// workgroups sharing a row panel drifted apart and lost the shared L2 panel reads,
// profiles/r2_gemm_pps_phase_v1.txt.  It was removed.)
//
// The epilogue stages 16 x 32 fp32 pieces in its own 18 KiB LDS region beside the 128 KiB
// pipeline.  Its VMEM ops (E per wave, static on the FAST path) sit between staging loads in
// the in-order vmcnt queue, so the two waits after an epilogue count them in (a count may
// only under-state the ops issued after the awaited one).
// ============================================================================
template <int N>
__device__ __forceinline__ void vm_wait_i() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int PPS_STR = 36;                       // epilogue staging row stride (floats)
constexpr int PPS_WAVE = 16 * PPS_STR * 4;        // bytes per wave
constexpr int PPS_LDS = 2 * G_BUF + 8 * PPS_WAVE;

template <int FK, int PRIO, bool DS = false>
__global__ void __launch_bounds__(512)
gemm_pps_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                void* __restrict__ C, int64_t ldc, int M, int N, int K, GemmEpi ep, int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = N / 256;
  const int tiles_m = M / 256;
  const int ntiles = tiles_n * tiles_m;
  const int G = gridDim.x;
  const int lin0 = xcd_remap(blockIdx.x, G);
  if (lin0 >= ntiles) return;
  const int nk = K / BK;
  const int R = (ntiles - lin0 + G - 1) / G;          // tiles of this workgroup

  int off[4][2];   // per-lane element offsets inside a tile: h 0 = A0, 1 = B0, 2 = B1, 3 = A1
  int dst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    const int c = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    const int cb = DS ? ((lane & 7) ^ ds_bxor(r)) * 8 : c;
    dst[i] = g * 1024;
    off[0][i] = r * (int)lda + c;
    off[3][i] = (128 + r) * (int)lda + c;
    off[1][i] = r * (int)ldw + cb;
    off[2][i] = (128 + r) * (int)ldw + cb;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  // Segment s = tile s of this workgroup, K-tiles [kb, ke) = [0, nk).  Every segment has >= 2
  // K-tiles, so K-tile u + 2 is at most one segment ahead.
  const int S = R;
  auto seg_info = [&](int s_, int& m0, int& n0, int& kb, int& ke) {
    int tm, tn;
    tile_coords(lin0 + s_ * G, tiles_m, tiles_n, group_m, tm, tn);
    m0 = tm * 256;
    n0 = tn * 256;
    kb = 0;
    ke = nk;
  };
  auto issue = [&](const int h, int buf, int m0, int n0, int kt) {
    const int hoff = (h == 1 || h == 2 ? G_OP : 0) + (h >= 2 ? G_HALF : 0);
    const uint16_t* base = (h == 0 || h == 3) ? A + (int64_t)m0 * lda : W + (int64_t)n0 * ldw;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((g_ptr_t)(base + off[h][i] + kt * BK),
                                       (lds_ptr_t)(smem + buf * G_BUF + hoff + dst[i]), 16, 0, 0);
  };

  const int frow = lane & 15, fq = lane >> 4;
  bf16x8_t fa[4][2], fb[2][2][2];
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
        fb[qn][j][s] = *(const bf16x8_t*)(base + G_OP + qn * G_HALF +
                                           (DS ? swzb(wn * 32 + 8 * (frow >> 2) + 4 * j + (frow & 3), s * 4 + fq)
                                               : swz(wn * 32 + j * 16 + frow, s * 4 + fq)));
  };

  constexpr bool FL = FK == 5;   // LN-folded row / column affine, no residual
  constexpr bool fast = FK > 0 && !FL;
  constexpr bool FB = fast && ((FK - 1) & 1), FR = fast && ((FK - 1) & 2);
  // VMEM ops of one epilogue (0: unknown): 16 stores (+ bias / residual loads; LN-folded: 8 column
  // vectors + 16 row scalars).  DS: only its 16 stores can still be in flight at the next wait (every
  // load of the epilogue feeds a store), and an under-stated count only waits longer.
  constexpr int E = DS ? ((FL || fast) ? 16 : 0) : FL ? 16 + 8 + 16 : fast ? 16 + (FB ? 2 : 0) + (FR ? 16 : 0) : 0;

  int m0, n0, kb, ke;
  seg_info(0, m0, n0, kb, ke);
  // prologue: K-tile kb whole, then A0, B0, B1 of K-tile kb + 1 (every segment has >= 2)
  issue(0, 0, m0, n0, kb);
  issue(1, 0, m0, n0, kb);
  issue(2, 0, m0, n0, kb);
  issue(3, 0, m0, n0, kb);
  issue(0, 1, m0, n0, kb + 1);
  issue(1, 1, m0, n0, kb + 1);
  issue(2, 1, m0, n0, kb + 1);
  vm_wait_i<8>();
  pp_barrier();
  if (wm == 1) pp_barrier();   // the stagger
  if constexpr (PRIO == 1) { if (wm == 1) __builtin_amdgcn_s_setprio(1); }

  float* es = (float*)(smem + 2 * G_BUF + wid * PPS_WAVE);
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
  int T = 0;       // global K-tile counter (LDS buffer parity)
  int after = 0;   // 0: none, 1: a C epilogue since the previous staging
  for (int sg = 0; sg < S; ++sg) {
    const int64_t t_seg = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
    const bool has_next = sg + 1 < S;
    int nm0 = m0, nn0 = n0, nkb = 0, nke = 0;
    if (has_next) seg_info(sg + 1, nm0, nn0, nkb, nke);
    f32x4_t acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bq = 0; bq < 2; ++bq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][bq][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

#define LM_PPS_CLUSTER(QM, QN)                                                                               \
    Unroll<0, 4>::run([&](const int i) {                                                                      \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                            \
      _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                            \
        acc[QM][QN][i][j] = DS ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[QN][j][s], fa[i][s], acc[QM][QN][i][j], 0, 0, 0) \
                               : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[QN][j][s], acc[QM][QN][i][j], 0, 0, 0); \
    });
    for (int kt = kb; kt < ke; ++kt) {
      const int b = T & 1;
      const char* base = smem + b * G_BUF;
      // K-tile T + 1 / T + 2 (possibly in the next segment)
      const bool c1 = kt + 1 < ke, c2 = kt + 2 < ke;
      const bool e1 = c1 || has_next, e2 = c2 || has_next;
      const int k1 = c1 ? kt + 1 : nkb;
      const int k2 = c2 ? kt + 2 : nkb + (kt + 2 - ke);
      const int af = kt == kb ? after : 0;
      // phase 0: rows qm = 0 <- A0, B0, B1; stage A1(T+1); retire A1(T)
      load_a(base, 0);
      load_b(base, 0);
      load_b(base, 1);
      if (e1) {
        issue(3, b ^ 1, c1 ? m0 : nm0, c1 ? n0 : nn0, k1);
        if (af == 0) vm_wait_i<8>(); else vm_wait_i<8 + E>();
      } else {
        vm_wait_i<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
      LM_PPS_CLUSTER(0, 0)
      LM_PPS_CLUSTER(0, 1)
      if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
      pp_barrier();
      // phase 1: rows qm = 1 <- A1; stage A0, B0, B1 of T+2; retire A0, B0, B1 of T+1
      load_a(base, 1);
      if (e2) {
        const int am = c2 ? m0 : nm0, an = c2 ? n0 : nn0;
        issue(0, b, am, an, k2);
        issue(1, b, am, an, k2);
        issue(2, b, am, an, k2);
        if (af == 0) vm_wait_i<8>(); else vm_wait_i<8 + E>();
      } else if (e1) {
        if (af == 0) vm_wait_i<2>(); else vm_wait_i<2 + E>();
      } else {
        vm_wait_i<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
      LM_PPS_CLUSTER(1, 0)
      LM_PPS_CLUSTER(1, 1)
      if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
      pp_barrier();
      ++T;
    }
#undef LM_PPS_CLUSTER
    const int64_t t_loop = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

    if constexpr (DS) {
      pp_epilogue_direct<false, FK>(acc, m0, n0, M, N, C, ldc, ep, wm, wn, lane);
      after = 1;
    } else {
      // ---- C epilogue: 16 passes (qm, i, qn) of 16 rows x 32 columns through this wave's
      // staging region; lane (rr, cq) stores 8 columns (16 B) of one row.
      const int rr = lane >> 2, cq = lane & 3;
      constexpr int RD = LM_GEMM_RES_PREFETCH;
      u32x4_t bq[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
      u32x4_t rz[RD];
      auto col_of = [&](int qn) { return n0 + qn * 128 + wn * 32 + cq * 8; };
      auto row_of = [&](int p) { return m0 + (p >> 3) * 128 + wm * 64 + ((p >> 1) & 3) * 16 + rr; };
      if constexpr (FB) {
        bq[0] = *(const u32x4_t*)((const uint16_t*)ep.bias + col_of(0));
        bq[1] = *(const u32x4_t*)((const uint16_t*)ep.bias + col_of(1));
      }
      if constexpr (FR) {
#pragma unroll
        for (int p = 0; p < RD; ++p) rz[p] = *(const u32x4_t*)(ep.residual + (int64_t)row_of(p) * ep.ldr + col_of(p & 1));
      }
      float lcs[FL ? 16 : 1], lcb[FL ? 16 : 1], lrs[FL ? 8 : 1], lro[FL ? 8 : 1];
      if constexpr (FL) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x4_t a = *(const f32x4_t*)(ep.col_aff + col_of(qn) + 4 * h);
            const f32x4_t b = *(const f32x4_t*)(ep.col_aff + N + col_of(qn) + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              lcs[qn * 8 + 4 * h + e] = a[e];
              lcb[qn * 8 + 4 * h + e] = b[e];
            }
          }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int64_t m = row_of(2 * r);
          lrs[r] = ep.row_aff[2 * m];
          lro[r] = ep.row_aff[2 * m + 1];
        }
      }
      Unroll<0, 16>::run([&](const int p) __attribute__((always_inline)) {
        const int qm = p >> 3, i = (p >> 1) & 3, qn = p & 1;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int rq = 0; rq < 4; ++rq) es[(fq * 4 + rq) * PPS_STR + j * 16 + frow] = acc[qm][qn][i][j][rq];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        float v[8];
        {
          const f32x4_t t0 = *(const f32x4_t*)(es + rr * PPS_STR + cq * 8);
          const f32x4_t t1 = *(const f32x4_t*)(es + rr * PPS_STR + cq * 8 + 4);
          v[0] = t0[0]; v[1] = t0[1]; v[2] = t0[2]; v[3] = t0[3];
          v[4] = t1[0]; v[5] = t1[1]; v[6] = t1[2]; v[7] = t1[3];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int m = row_of(p), n = col_of(qn);
        if constexpr (FL) {
          epi_store_lnf<false, 8>(v, m, n, C, ldc, ep, lrs[p >> 1], lro[p >> 1], lcs + qn * 8, lcb + qn * 8, crs);
        } else if constexpr (fast) {
          float f[8];
          unpack8(bq[qn], f);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = v[q] * ep.alpha + f[q];
          if (ep.act) apply_act_n<8>(v, ep.act);
          if constexpr (FR) {
            unpack8(rz[p % RD], f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += f[q];
            if (p + RD < 16) rz[p % RD] = *(const u32x4_t*)(ep.residual + (int64_t)row_of(p + RD) * ep.ldr + col_of((p + RD) & 1));
          }
          st16<false>(C, crs, ((int64_t)m * ldc + n) * 2, pack8(v));
        } else {
          epi_store8_t<false>(v, m, n, M, N, C, ldc, ep, crs);
        }
      });
      after = 1;
    }
    if (ep.dbg && tid == 0) {   // profiling (tools/gemm_pp_timeline.py): stamps of this tile
      int64_t* d = ep.dbg + 4 * (int64_t)(lin0 + sg * G);
      d[0] = t_seg; d[1] = t_seg; d[2] = t_loop; d[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
    m0 = nm0;
    n0 = nn0;
    kb = nkb;
    ke = nke;
  }
  if constexpr (PRIO == 1) { if (wm == 1) __builtin_amdgcn_s_setprio(0); }
  if (wm == 0) pp_barrier();
}

static int pp_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

template <int FK, int PRIO, bool DS = false>
static void launch_pps_t(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                         int N, int K, const GemmEpi& ep, int group_m, hipStream_t stream) {
  const int tiles = (M / 256) * (N / 256);
  // one workgroup per CU (r5: fewer tiles per workgroup, dispatched as CUs free up, lost in the 2-stream
  // tower -- a workgroup's next tile shares no L2 panels with its neighbours', profiles/r5_gemm_pp_ds_v1.txt)
  const int grid = tiles < pp_num_cus() ? tiles : pp_num_cus();
  const int lds = DS ? 2 * G_BUF : PPS_LDS;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_pps_kernel<FK, PRIO, DS>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_pps_kernel<FK, PRIO, DS>), dim3(grid), dim3(512), lds, stream, A, lda, W, ldw, C, ldc, M,
                     N, K, ep, group_m);
}

hipError_t gemm_pp(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                   int N, int K, const GemmEpi& ep, int group_m, int variant, hipStream_t stream) {
  // variants 8 / 9: 6 / 7 with the direct-store epilogue (pp_epilogue_direct; not for SwiGLU)
  bool ds = false;
  if (variant >= 8) {
    variant -= 2;
    ds = !ep.glu;
  }
  if (variant & 1) {
    // persistent form: interior tiles only, 32-bit in-tile offsets, >= 2 K-tiles
    const bool ok = M % 256 == 0 && N % 256 == 0 && K / BK >= 2 && 255 * lda + K < (1LL << 31) &&
                    255 * ldw + K < (1LL << 31) && ep.out_group == 0 && !ep.glu && !ep.out_f32;
    if (ok) {
      const int64_t extent = (int64_t)M * ldc * 2;
      const bool fast = !ep.table && !ep.prelu && !ep.post_act && !(ep.bias && ep.bias_f32) &&
                        extent < ((int64_t)1 << 31);
      const bool lnf = ep.row_aff && !ep.bias && !ep.residual && ep.alpha == 1.f && fast;
      const int fk = lnf ? 5 : fast && !ep.row_aff ? 1 + (ep.bias ? 1 : 0) + (ep.residual ? 2 : 0) : 0;
      const bool prio1 = (variant & 2) != 0;
#define LM_PPS_CASE(FKV)                                                                                     \
      case FKV:                                                                                                 \
        if (ds) launch_pps_t<FKV, 1, true>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);               \
        else if (prio1) launch_pps_t<FKV, 1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);             \
        else launch_pps_t<FKV, 0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, stream);                        \
        break;
      switch (fk) {
        LM_PPS_CASE(1)
        LM_PPS_CASE(2)
        LM_PPS_CASE(3)
        LM_PPS_CASE(4)
        LM_PPS_CASE(5)
        default:
        LM_PPS_CASE(0)
      }
#undef LM_PPS_CASE
      return hipGetLastError();
    }
    variant |= 4;   // two-phase non-persistent form otherwise
  }
  const int64_t extent = (int64_t)M * ldc * (ep.out_f32 ? 4 : 2);
  const bool wt = false;
  const bool fast = M % 256 == 0 && N % 256 == 0 && ep.out_group == 0 && !ep.glu && !ep.table && !ep.prelu &&
                    !ep.post_act && !ep.out_f32 && !(ep.bias && ep.bias_f32) && extent < ((int64_t)1 << 31);
  const bool lnf = ep.row_aff && !ep.bias && !ep.residual && ep.alpha == 1.f && fast;
  const int fk = lnf ? 5 : fast && !ep.row_aff ? 1 + (ep.bias ? 1 : 0) + (ep.residual ? 2 : 0) : 0;
  const bool prio1 = (variant & 2) != 0, two = (variant & 4) != 0;
  switch (fk) {
    case 1: launch_pp_fk<1>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, ds, stream); break;
    case 2: launch_pp_fk<2>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, ds, stream); break;
    case 3: launch_pp_fk<3>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, ds, stream); break;
    case 4: launch_pp_fk<4>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, ds, stream); break;
    case 5: launch_pp_fk<5>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, ds, stream); break;
    default: launch_pp_fk<0>(A, lda, W, ldw, C, ldc, M, N, K, ep, group_m, wt, prio1, two, ds, stream); break;
  }
  return hipGetLastError();
}


// ============================================================================
// Split-K tail: out = epi( sum_s slab[s] ), 8 columns per thread, fp32 throughout
// ============================================================================
__global__ void __launch_bounds__(256)
splitk_reduce_epi_kernel(const float* __restrict__ slabs, int S, int M, int N, void* __restrict__ C, int64_t ldc,
                         GemmEpi ep) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nc = N / 8;
  if (idx >= (int64_t)M * nc) return;
  const int m = (int)(idx / nc), n = (int)(idx % nc) * 8;
  const int64_t slab = (int64_t)M * N;
  float v[8];
  {
    const f32x4_t a = *(const f32x4_t*)(slabs + (int64_t)m * N + n);
    const f32x4_t b = *(const f32x4_t*)(slabs + (int64_t)m * N + n + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
  for (int s = 1; s < S; ++s) {   // split order: deterministic
    const f32x4_t a = *(const f32x4_t*)(slabs + s * slab + (int64_t)m * N + n);
    const f32x4_t b = *(const f32x4_t*)(slabs + s * slab + (int64_t)m * N + n + 4);
    v[0] += a[0]; v[1] += a[1]; v[2] += a[2]; v[3] += a[3]; v[4] += b[0]; v[5] += b[1]; v[6] += b[2]; v[7] += b[3];
  }
  GemmEpi e = ep;
  e.alpha = 1.f;   // applied by the slab GEMM
  epi_store8_t<false>(v, m, n, M, N, C, ldc, e, c_rsrc(C));
}

static float* tail_workspace(size_t bytes, hipStream_t stream) {
  return (float*)stream_workspace(bytes, stream, WS_PP_TAIL, (size_t)64 << 20);
}

hipError_t gemm_tail_splitk(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc,
                            int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
  if (ep.glu || ep.out_group || ep.table || ep.split_koff || N % 8 != 0 || K % BK != 0 || M <= 0)
    return hipErrorNotSupported;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int nk = K / BK;
  // splits: power of two, >= 2 K-tiles each, <= 128 workgroups in all (slab traffic vs parallelism)
  int S = 1;
  while (S * 2 * tiles <= pp_num_cus() / 2 && nk % (S * 2) == 0 && nk / (S * 2) >= 2) S *= 2;
  if (S == 1) return hipErrorNotSupported;
  float* slabs = tail_workspace((size_t)S * M * N * sizeof(float), stream);
  if (slabs == nullptr) return hipErrorNotSupported;
  GemmEpi e{};
  e.alpha = ep.alpha;
  e.out_f32 = 1;
  e.split_koff = (int64_t)(nk / S) * BK;
  e.split_cstride = (int64_t)M * N;
  launch_pp_t<false, 0, 1, 2>(A, lda, W, ldw, slabs, N, M, N, K / S, e, 4, stream, S);
  const int64_t work = (int64_t)M * (N / 8);
  hipLaunchKernelGGL(splitk_reduce_epi_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, slabs, S, M,
                     N, C, ldc, ep);
  return hipGetLastError();
}

}  // namespace lumen
