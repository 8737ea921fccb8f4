// 256 x 256 W8A8 "ping-pong" GEMM on the gfx950 block-scaled matrix cores (launch_variant code 17 of
// csrc/gemm_f8.hip).
//
//   C[M, N] = epi( (A8[M, K] . W8[N, K]^T) * sa[m] * sw[n] )      (OCP e4m3fn operands)
//
// The fp8 twin of the bf16 ping-pong kernel (csrc/gemm_pp.hip, 2-phase form, static priority for the
// lagging wave group): same 256 x 256 tile, same 128-byte LDS rows staged as four 128 x 128 B
// half-tiles by LDS-DMA, same barrier schedule -- but a 128-byte K-tile is 128 fp8 k-values, and each
// fragment pair (chunks g, g + 4 of a row: 32 bytes per lane) feeds ONE
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales) instead of two bf16 MFMAs: the same LDS
// bytes and the same MFMA cycles per K-tile for twice the K, i.e. twice the bf16 kernel's rate.
//
// Why 256 x 256 for the W8A8 prefill (M = 624): the 128 x 128 pipelines (gemm_f8.hip, gemm_f8ks.hip)
// pull 32 KiB per 4.2 MFLOP into a CU, and tools/gemm_floor_probe.py measured them at the same
// ~0.5 us per K-step with operands cache-resident as from HBM (r5): the per-CU LDS-DMA intake sets
// their pace.  This tile pulls 64 KiB per 16.8 MFLOP (2x the FLOP per byte).  The Llama-3-8B
// gate|up projection (N = 28672: 336 tiles) is the shape it is for; split-K over gridDim.y (fp32
// slabs + an ordered reduce with the real epilogue) covers the narrow ones.
//
// Epilogue: each lane's 16 output columns' weight scales / bias and its 8 rows' token scales are
// loaded together when the K loop ends; residual rows stream in 4 slabs ahead (gemm_pp's fast path).
#include <type_traits>

#include "common.h"
#include "gemm_epi.h"
#include "workspace.h"

namespace lumen {

typedef int i32x8_t __attribute__((ext_vector_type(8)));

constexpr int WS_F8PP_SPLIT = 4;   // stream_workspace tag (workspace.h tags 0-3 are taken)

__device__ __forceinline__ void f8pp_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void f8pp_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ i32x8_t cat8(const u32x4_t a, const u32x4_t b) {
  return (i32x8_t){(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

__global__ void __launch_bounds__(512)
gemm_f8pp_kernel(const uint8_t* __restrict__ A, int64_t lda, const float* __restrict__ sa, const uint8_t* __restrict__ W,
                 int64_t ldw, const float* __restrict__ sw, void* __restrict__ C, int64_t ldc, int M, int N, int K,
                 GemmEpi ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int tiles_n = (N + 255) / 256;
  const int tiles_m = (M + 255) / 256;
  // XCD-aware: consecutive logical tiles (row tiles fastest) share a W column panel on one XCD
  const int lin = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int tm = lin % tiles_m, tn = lin / tiles_m;
  const int m0 = tm * 256, n0 = tn * 256;
  if (ep.split_koff) {   // split-K: this workgroup's K slice and fp32 slab
    A += blockIdx.y * ep.split_koff;
    W += blockIdx.y * ep.split_koff;
    C = (float*)C + blockIdx.y * ep.split_cstride;
  }

  // half-tile h: 0 = A0, 1 = B0, 2 = B1, 3 = A1 (128 rows x 128 B each); lane writes LDS row
  // g * 8 + l / 8, physical chunk l % 8, fetching logical chunk (l % 8) ^ ((row >> 1) & 7)
  const uint8_t* src[4][2];
  int dst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int r = g * 8 + (lane >> 3);
    const int c = ((lane & 7) ^ ((r >> 1) & 7)) * 16;
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
      __builtin_amdgcn_global_load_lds((g_ptr_t)(src[h][i] + (int64_t)kt * 128),
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
  u32x4_t fa[4][2], fb[2][2][2];   // fb[qn][j][chunk]
  auto load_a = [&](const char* base, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[i][s] = *(const u32x4_t*)(base + qm * G_HALF + swz(wm * 64 + i * 16 + frow, s * 4 + fq));
  };
  auto load_b = [&](const char* base, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fb[qn][j][s] = *(const u32x4_t*)(base + G_OP + qn * G_HALF + swz(wn * 32 + j * 16 + frow, s * 4 + fq));
  };
#define LM_F8PP_CLUSTER(QM, QN)                                                                                \
  Unroll<0, 4>::run([&](const int i) {                                                                          \
    const i32x8_t a8 = cat8(fa[i][0], fa[i][1]);                                                                \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                                \
      acc[QM][QN][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, cat8(fb[QN][j][0], fb[QN][j][1]), \
                                                                          acc[QM][QN][i][j], 0, 0, 0, 127, 0, 127); \
  });

  const int nk = K / 128;
  // prologue: tile 0 whole (A0, B0, B1, A1), then A0, B0, B1 of tile 1 (A1(1) at phase 0)
  issue(0, 0, 0);
  issue(1, 0, 0);
  issue(2, 0, 0);
  issue(3, 0, 0);
  if (nk > 1) {
    issue(0, 1, 1);
    issue(1, 1, 1);
    issue(2, 1, 1);
    f8pp_vm_wait<6>();
  } else {
    f8pp_vm_wait<0>();
  }
  f8pp_bar();
  if (wm == 1) f8pp_bar();   // the stagger: group 1 runs one barrier behind
  if (wm == 1) __builtin_amdgcn_s_setprio(1);

  // One K-tile = two phases.  The steady-state loop body has no branches (every K-tile has two more
  // after it), the last two K-tiles are peeled: with the staging conditions inside the loop the
  // compiler sank phase 0's MFMAs past both of its barriers into phase 1 (r5 ISA), which undid the
  // ping-pong.
  auto ktile = [&](const int kt, auto N1, auto N2) __attribute__((always_inline)) {
    constexpr bool n1 = decltype(N1)::value, n2 = decltype(N2)::value;
    const int b = kt & 1;
    const char* base = smem + b * G_BUF;
    // phase 0: rows qm = 0 x all columns <- A0, B0, B1; stage A1(t+1); retire A1(t)
    load_a(base, 0);
    load_b(base, 0);
    load_b(base, 1);
    if constexpr (n1) {
      issue(3, b ^ 1, kt + 1);
      f8pp_vm_wait<8>();
    } else {
      f8pp_vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f8pp_bar();
    LM_F8PP_CLUSTER(0, 0)
    LM_F8PP_CLUSTER(0, 1)
    f8pp_bar();
    // phase 1: rows qm = 1 <- A1 (B fragments kept); stage A0, B0, B1 of t+2; retire those of t+1
    load_a(base, 1);
    if constexpr (n2) {
      issue(0, b, kt + 2);
      issue(1, b, kt + 2);
      issue(2, b, kt + 2);
      f8pp_vm_wait<8>();
    } else if constexpr (n1) {
      f8pp_vm_wait<2>();
    } else {
      f8pp_vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f8pp_bar();
    LM_F8PP_CLUSTER(1, 0)
    LM_F8PP_CLUSTER(1, 1)
    f8pp_bar();
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int kt = 0;
  for (; kt + 2 < nk; ++kt) ktile(kt, T_{}, T_{});
  if (kt + 1 < nk) {
    ktile(kt, T_{}, F_{});
    ++kt;
  }
  ktile(kt, F_{}, F_{});
#undef LM_F8PP_CLUSTER
  if (wm == 1) __builtin_amdgcn_s_setprio(0);
  if (wm == 0) f8pp_bar();   // re-align the groups: every LDS read of the K loop is done

  // ---- epilogue operands (loaded here, not before the K loop: the 128 accumulators + fragments
  // leave no room to hold them through it -- 54 VGPRs spilled)
  const int rr = lane >> 2, cq = lane & 3;
  const int ncol = n0 + (cq >> 1) * 128 + wn * 32 + (cq & 1) * 16;
  const bool fast = !ep.row_aff && !ep.table && ep.out_group == 0 && !ep.prelu && !ep.post_act && !ep.out_f32 &&
                    !(ep.bias && ep.bias_f32) && !ep.act && ncol + 16 <= N;
  float cs[16], ra[8];
  if (sw && ncol + 16 <= N) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4_t t = *(const f32x4_t*)(sw + ncol + 4 * q);
      cs[4 * q] = t[0]; cs[4 * q + 1] = t[1]; cs[4 * q + 2] = t[2]; cs[4 * q + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) cs[q] = ncol + q < N ? (sw ? sw[ncol + q] : 1.f) : 0.f;
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int m = m0 + (s >> 2) * 128 + wm * 64 + (s & 3) * 16 + rr;
    ra[s] = m < M ? (sa ? sa[m] : 1.f) : 0.f;
  }
  u32x4_t bz0 = {0u, 0u, 0u, 0u}, bz1 = {0u, 0u, 0u, 0u};
  if (fast && ep.bias) {
    bz0 = *(const u32x4_t*)((const uint16_t*)ep.bias + ncol);
    bz1 = *(const u32x4_t*)((const uint16_t*)ep.bias + ncol + 8);
  }

  // ---- epilogue: per-wave 16-row slabs through LDS; lane (rr, cq) -> 16 columns of one row
  constexpr int LDSTR = 68;
  float* es = (float*)smem + wid * 16 * LDSTR;
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
  constexpr int RD = 2;          // residual slabs in flight (4, gemm_pp's depth, spills here)
  const bool res = fast && ep.residual && !ep.glu;
  u32x4_t rz[RD][2];
  auto res_ptr = [&](int s) {
    const int m = min(m0 + (s >> 2) * 128 + wm * 64 + (s & 3) * 16 + rr, M - 1);
    return ep.residual + (int64_t)m * ep.ldr + ncol;
  };
  if (res) {
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
      const f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cq * 16 + q * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[q * 4 + e] = t[e] * ra[s] * cs[q * 4 + e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int m = m0 + qm * 128 + wm * 64 + i * 16 + rr;
    if (fast) {
      u32x4_t r0 = {0u, 0u, 0u, 0u}, r1 = {0u, 0u, 0u, 0u};
      if (res) {
        r0 = rz[s % RD][0];
        r1 = rz[s % RD][1];
        if (s + RD < 8) {
          rz[s % RD][0] = *(const u32x4_t*)res_ptr(s + RD);
          rz[s % RD][1] = *(const u32x4_t*)(res_ptr(s + RD) + 8);
        }
      }
      if (m < M) {
        float f[8];
        unpack8(bz0, f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = v[q] * ep.alpha + f[q];
        unpack8(bz1, f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[8 + q] = v[8 + q] * ep.alpha + f[q];
        if (ep.glu) {
          float o[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = v[q] * fast_rcp(1.f + __expf(-v[q])) * v[8 + q];
          st16<false>(C, crs, ((int64_t)m * ldc + (ncol >> 1)) * 2, pack8(o));
        } else {
          if (res) {
            unpack8(r0, f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += f[q];
            unpack8(r1, f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
          }
          st16<false>(C, crs, ((int64_t)m * ldc + ncol) * 2, pack8(v));
          st16<false>(C, crs, ((int64_t)m * ldc + ncol + 8) * 2, pack8(v + 8));
        }
      }
    } else {
      epi_store16_t<false>(v, m, ncol, M, N, C, ldc, ep, crs);
    }
  });
}

// split-K tail: out = epi( sum_s slab[s] ) over 16 columns per thread (scales already applied)
__global__ void __launch_bounds__(256)
f8pp_reduce16_kernel(const float* __restrict__ slabs, int S, int M, int N, void* __restrict__ C, int64_t ldc,
                     GemmEpi ep) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nc = N / 16;
  if (idx >= (int64_t)M * nc) return;
  const int m = (int)(idx / nc), n = (int)(idx % nc) * 16;
  const int64_t slab = (int64_t)M * N;
  float v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = 0.f;
  for (int s = 0; s < S; ++s) {   // split order: deterministic
    const float* p = slabs + s * slab + (int64_t)m * N + n;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4_t a = *(const f32x4_t*)(p + 4 * q);
      v[4 * q] += a[0]; v[4 * q + 1] += a[1]; v[4 * q + 2] += a[2]; v[4 * q + 3] += a[3];
    }
  }
  GemmEpi e = ep;
  e.alpha = 1.f;   // applied by the slab GEMM
  epi_store16_t<false>(v, m, n, M, N, C, ldc, e, c_rsrc(C));
}

static int f8pp_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

static void f8pp_launch(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw,
                        const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, int S,
                        hipStream_t stream) {
  constexpr size_t lds = 2 * G_BUF;   // 128 KiB: two K-tiles of A0 | B0 | B1 | A1
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_f8pp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  hipLaunchKernelGGL(gemm_f8pp_kernel, dim3(tiles, S), dim3(512), lds, stream, A, lda, sa, W, ldw, sw, C, ldc, M, N,
                     K, ep);
}

// splits <= 0: automatic (only grids of at most a third of the CUs split, to ~1-2 workgroups per CU,
// keeping >= 8 K-tiles per split)
hipError_t gemm_f8pp(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw, const float* sw,
                     void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, int splits, hipStream_t stream) {
  if (K % 128 != 0 || N % 16 != 0 || M <= 0 || lda % 16 != 0 || ldw % 16 != 0) return hipErrorInvalidValue;
  if (ep.split_koff || (ep.glu && ep.out_f32)) return hipErrorInvalidValue;
  const int nk = K / 128;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  int S = splits;
  if (S <= 0) {
    S = 1;
    if (3 * tiles <= f8pp_num_cus() && !ep.out_group && !ep.table && !ep.prelu && !ep.post_act)
      for (int c : {2, 3, 4, 5, 6, 8})
        if (tiles * c <= 2 * f8pp_num_cus() && nk % c == 0 && nk / c >= 8) S = c;
  }
  while (S > 1 && (nk % S != 0 || nk / S < 2)) --S;
  if (S > 1) {
    float* slabs = (float*)stream_workspace((size_t)S * M * N * sizeof(float), stream, WS_F8PP_SPLIT, (size_t)64 << 20);
    if (slabs != nullptr) {
      GemmEpi e{};
      e.alpha = 1.f;
      e.out_f32 = 1;
      e.split_koff = (int64_t)(K / S);
      e.split_cstride = (int64_t)M * N;
      f8pp_launch(A, lda, sa, W, ldw, sw, slabs, N, M, N, K / S, e, S, stream);
      const int64_t work = (int64_t)M * (N / 16);
      hipLaunchKernelGGL(f8pp_reduce16_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, slabs, S, M,
                         N, C, ldc, ep);
      return hipGetLastError();
    }
  }
  f8pp_launch(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, 1, stream);
  return hipGetLastError();
}

}  // namespace lumen
