// W8A8 prefill GEMM, intra-workgroup split-K form (launch_variant code 16 of csrc/gemm_f8.hip).
//
//   C[M, N] = epi( (A8[M, K] . W8[N, K]^T) * sa[m] * sw[n] )      (OCP e4m3fn operands)
//
// Replaces the decoder prefill projections of the reference's ORT decoder
// (packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:420-492) on the single-wave grids.
#include "common.h"
#include "gemm_epi.h"
#include "workspace.h"

namespace lumen {

constexpr int WS_F8KS_SK = 5, WS_F8KS_CNT = 6;   // stream_workspace tags (0-3 workspace.h, 4 gemm_f8pp)

typedef int i32x8_t __attribute__((ext_vector_type(8)));

template <int N>
__device__ __forceinline__ void ks_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void ks_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ---------------------------------------------------------------------------- intra-workgroup split-K
// The single-wave prefill grids (M = 624: qkv / o / down, 160-240 tiles of 128 x 128) run every
// 128 x 128 tile at ONE workgroup per CU.  Measured (tools/gemm_floor_probe.py, r5): the 8-wave
// 64 x 32-per-wave pipeline costs ~0.45 us per 128-deep K-step with operands from HBM AND with a
// cache-resident footprint -- the kernel is bound by its own instruction stream, not memory:
// each wave reads 12 KiB of fragments per 8 MFMAs, the 8 waves read them at the same moment
// after every barrier, then all MFMA at once.
//
// Here the two 4-wave groups of the workgroup split K instead of M: group g computes the whole
// 128 x 128 tile (64 x 64 per wave, 16 MFMAs per K-step: 1 KiB of fragment reads per MFMA, half
// the 8-wave form's) over the K-steps s = g (mod 2), and the groups run one barrier apart
// (ping-pong), so on every SIMD one group's 16 MFMAs cover the other group's fragment reads and
// staging issue.  Barriers B_s are numbered by K-step: the group whose read segment precedes
// B_s (the group that MFMAs step s) stages K-step s + NS - 1 (whole stage, 8 x 1 KiB pieces per wave) into
// the buffer step s - 1 freed at B_{s - 1}; step s' is waited for (vmcnt, issuing waves) before
// B_{s' - 1}, so its readers (after B_{s' - 1}) see it.  At the end the groups swap halves of
// their partial tiles through LDS (each finalises 64 of the 128 rows) and store.
// Per-token / per-channel scales, bias and residual of the stored rows are loaded before the
// K loop (no epilogue round trip).  Plain epilogues only (no MX outputs, no split-K slabs).
// Stream-K (SK): the grid is one workgroup per CU and workgroup w runs the K-steps
// [w * L, (w + 1) * L) of the (tile, K-step) sequence -- the tail of one tile and the head of the
// next (L <= nk): a 160-tile grid (M = 624: o / down) then keeps all 256 CUs busy instead of 160.
// A segment that does not end its tile leaves its fp32 partial tile in the workspace and bumps the
// tile's counter; the segment that ends the tile (always the highest workgroup of the tile, so it
// only waits on workgroups dispatched before it) adds the partials and runs the epilogue.
struct F8SkArgs {
  int L;          // K-steps per workgroup (<= nk)
  float* ws;      // [grid][2 segments][16384] fp32 partial tiles
  int* cnt;       // [tiles] arrival counters, zero between launches
};

template <int NS, bool SK>
__global__ void __launch_bounds__(512)
gemm_f8ks_kernel(const uint8_t* __restrict__ A, int64_t lda, const float* __restrict__ sa,
                 const uint8_t* __restrict__ W, int64_t ldw, const float* __restrict__ sw, void* __restrict__ C,
                 int64_t ldc, int M, int N, int K, GemmEpi ep, F8SkArgs sk) {
  static_assert(NS == 4, "stage parity: the issuing group of step s' is (s' + 1) % 2 for an even ring");
  constexpr int STAGE = 2 * 128 * 128;       // A image | W image (128 rows x 128 B each)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, w4 = wid & 3, wm = w4 >> 1, wn = w4 & 1;
  const int tiles_m = (M + 127) / 128, tiles_n = (N + 127) / 128;
  const int nk = K / 128;
  const int frow = lane & 15, g = lane >> 4;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  // Stream-K segments of this workgroup's range: seg 0 = (the tail of) the first tile, seg 1 = the
  // head of the next.  They run seg 1 FIRST: the head is partial work another (higher) workgroup
  // finishes, so it is published early, and a tile's finisher -- which does its tail last --
  // finds the partials of the lower workgroups (who did that tile's head first) ready.
  const int total = tiles_m * tiles_n * nk;
  const int wbeg = SK ? blockIdx.x * sk.L : 0;
  const int wend = SK ? min(total, wbeg + sk.L) : 0;
  const int t0 = SK ? wbeg / nk : 0;
  const int kb0 = wbeg - t0 * nk, ke0 = SK ? min(nk, wend - t0 * nk) : 0;
  const int nseg = SK ? ((t0 + 1) * nk < wend ? 2 : 1) : 1;

  for (int q = 0; q < nseg; ++q) {
    int tile, kb, ke;
    const int seg = nseg - 1 - q;
    if (SK) {
      tile = t0 + seg;
      kb = seg ? 0 : kb0;
      ke = seg ? wend - tile * nk : ke0;
      if (q) __syncthreads();                 // the previous segment's LDS (swap / epilogue) is free
    } else {
      tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
      kb = 0;
      ke = nk;
    }
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int m0 = tm * 128, n0 = tn * 128;
    const int nkl = ke - kb;

    // ---- epilogue operands of the rows / columns this lane stores: loaded before any staging (so
    // every counted vmcnt below only ever waits for them in addition); under Stream-K after the
    // K loop instead (their registers would spill the segment loop)
    const int rr = lane >> 2, cc = (lane & 3) * 16;
    const int ncol = n0 + wn * 64 + cc;
    const bool fast = !ep.row_aff && !ep.table && ep.out_group == 0 && !ep.prelu && !ep.post_act && !ep.out_f32 &&
                      !(ep.bias && ep.bias_f32) && !ep.act && ncol + 16 <= N;
    float cs[16], ra[2];
    u32x4_t bz[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}}, rz[2][2];
    auto load_epi = [&]() {
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
      for (int ii = 0; ii < 2; ++ii) {
        const int m = m0 + wm * 64 + (grp * 2 + ii) * 16 + rr;
        ra[ii] = m < M ? (sa ? sa[m] : 1.f) : 0.f;
        if (fast && ep.residual && !ep.glu) {
          const uint16_t* rp = ep.residual + (int64_t)min(m, M - 1) * ep.ldr + ncol;
          rz[ii][0] = *(const u32x4_t*)rp;
          rz[ii][1] = *(const u32x4_t*)(rp + 8);
        }
      }
      if (fast && ep.bias) {
        bz[0] = *(const u32x4_t*)((const uint16_t*)ep.bias + ncol);
        bz[1] = *(const u32x4_t*)((const uint16_t*)ep.bias + ncol + 8);
      }
    };
    if (!SK) load_epi();

    // ---- staging: a group copies a whole stage; wave w4 the A and W pieces 4 * w4 + i (8 rows x 128 B)
    const uint8_t* src_a[4];
    const uint8_t* src_w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (4 * w4 + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      src_a[i] = A + (int64_t)min(m0 + r, M - 1) * lda + (int64_t)kb * 128 + c * 16;
      src_w[i] = W + (int64_t)min(n0 + r, N - 1) * ldw + (int64_t)kb * 128 + c * 16;
    }
    auto stage = [&](const int s) {
      char* base = smem + (s % NS) * STAGE;
      const int64_t koff = (int64_t)s * 128;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((g_ptr_t)(src_a[i] + koff), (lds_ptr_t)(base + (4 * w4 + i) * 1024), 16, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((g_ptr_t)(src_w[i] + koff),
                                         (lds_ptr_t)(base + 16384 + (4 * w4 + i) * 1024), 16, 0, 0);
    };

    f32x4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    u32x4_t fa[4][2], fb[4][2];
    auto frags = [&](const int s) {
      const char* sA = smem + (s % NS) * STAGE;
      const char* sW = sA + 16384;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + frow;
        fb[j][0] = *(const u32x4_t*)(sW + swz(r, g));
        fb[j][1] = *(const u32x4_t*)(sW + swz(r, g + 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + frow;
        fa[i][0] = *(const u32x4_t*)(sA + swz(r, g));
        fa[i][1] = *(const u32x4_t*)(sA + swz(r, g + 4));
      }
    };
    auto mfmas = [&]() {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const i32x8_t a8 = (i32x8_t){(int)fa[i][0][0], (int)fa[i][0][1], (int)fa[i][0][2], (int)fa[i][0][3],
                                       (int)fa[i][1][0], (int)fa[i][1][1], (int)fa[i][1][2], (int)fa[i][1][3]};
          const i32x8_t b8 = (i32x8_t){(int)fb[j][0][0], (int)fb[j][0][1], (int)fb[j][0][2], (int)fb[j][0][3],
                                       (int)fb[j][1][0], (int)fb[j][1][1], (int)fb[j][1][2], (int)fb[j][1][3]};
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[i][j], 0, 0, 0, 127, 0, 127);
        }
    };

    // ---- prologue: stage s' < NS is issued by group (s' + 1) % 2 (the in-loop rule)
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (((s + 1) & 1) == grp && s < nkl) stage(s);
    if (grp == 1) {      // step 0 (group 1's stage) lands before B_{-1}; stage 2 may stay in flight
      if (2 < nkl) ks_vm_wait<8>();
      else ks_vm_wait<0>();
    }
    int bars = 1;
    ks_bar();                                   // B_{-1}
    if (grp == 1) { ks_bar(); ++bars; }         // the stagger: group 1 runs one barrier behind
    for (int s = grp; s < nkl; s += 2) {
      // read segment before B_s: fragments of step s (landed and published at B_{s-1}), the stage
      // s + NS - 1 into the buffer step s - 1 left at B_{s-1}, then step s + 1 (this group's
      // stage) landed before B_s
      frags(s);
      const bool issue = s >= 1 && s + NS - 1 < nkl;
      if (issue) stage(s + NS - 1);
      if (s + NS - 1 < nkl) ks_vm_wait<8>();
      else ks_vm_wait<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ks_bar();                                 // B_s
      __builtin_amdgcn_s_setprio(1);
      mfmas();
      __builtin_amdgcn_s_setprio(0);
      ks_bar();                                 // B_{s+1}
      bars += 2;
    }
    // equalise the barrier count of the two groups (group g ran 1 + [g] + 2 * #steps(g))
    const int n0s = (nkl + 1) / 2, n1s = nkl / 2;
    const int nbar = max(1 + 2 * n0s, 2 + 2 * n1s);
    for (int b = bars; b < nbar; ++b) ks_bar();
    __syncthreads();   // every DMA waited (vmcnt(0) on each group's last steps), every fragment read done

    // ---- swap halves: group 0 keeps row fragments 0-1 of its wave tile, group 1 rows 2-3
    f32x4_t* xb = (f32x4_t*)smem;               // [grp][w4][8][64] f32x4 = 64 KiB
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // the row fragment the other group finalises (constant indices: a runtime index into acc
        // would put the accumulators in scratch)
        xb[((grp * 4 + w4) * 8 + ii * 4 + j) * 64 + lane] = grp ? acc[ii][j] : acc[2 + ii][j];
      }
    __syncthreads();
    f32x4_t fin[2][4];
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fin[ii][j] = (grp ? acc[2 + ii][j] : acc[ii][j]) + xb[(((1 - grp) * 4 + w4) * 8 + ii * 4 + j) * 64 + lane];

    if (SK && (kb > 0 || ke < nk)) {
      // hand-off per cdna_hip_programming.md (in-launch split-K): write-through (sc1) partial
      // stores, every wave drains, ONE relaxed agent-scope add; the finisher polls relaxed, ONE
      // agent-scope acquire, then plain loads
      const int fidx = (grp * 4 + w4) * 8;     // this thread's 8 f32x4 of a partial tile
      if (ke < nk) {
        // not the tile's last segment: leave the partial, count in
        const __amdgpu_buffer_rsrc_t wrs = c_rsrc(sk.ws + ((int64_t)blockIdx.x * 2 + seg) * 16384);
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4_t*)&fin[ii][j], wrs, ((fidx + ii * 4 + j) * 64 + lane) * 16,
                                                   0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(sk.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      // the tile's last segment: wait for the workgroups before it, add their partials
      const int wfirst = (tile * nk) / sk.L;
      const int expect = (int)blockIdx.x - wfirst;
      if (tid == 0) {
        while (__hip_atomic_load(sk.cnt + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < expect)
          __builtin_amdgcn_s_sleep(1);
        __hip_atomic_store(sk.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // for the next launch
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      for (int wq = wfirst; wq < (int)blockIdx.x; ++wq) {
        const int sq = ((wq * sk.L) / nk == tile) ? 0 : 1;   // which of its segments covered this tile
        const f32x4_t* src = (const f32x4_t*)(sk.ws + ((int64_t)wq * 2 + sq) * 16384);
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j) fin[ii][j] += src[(fidx + ii * 4 + j) * 64 + lane];
      }
    }

    if (SK) load_epi();
    // ---- epilogue: two 16 x 64 slabs per wave through a private LDS region past the swap buffer
    constexpr int LDSTR = 68;
    float* es = (float*)(smem + 65536) + wid * 16 * LDSTR;
    const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) es[(g * 4 + r) * LDSTR + j * 16 + frow] = fin[ii][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[q * 4 + e] = t[e] * ra[ii] * cs[q * 4 + e];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // es is rewritten by the next slab
      const int m = m0 + wm * 64 + (grp * 2 + ii) * 16 + rr;
      if (fast && m < M) {
        float f[8];
        unpack8(bz[0], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = v[q] * ep.alpha + f[q];
        unpack8(bz[1], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[8 + q] = v[8 + q] * ep.alpha + f[q];
        if (ep.glu) {
          float o[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = v[q] * fast_rcp(1.f + __expf(-v[q])) * v[8 + q];
          st16<false>(C, crs, ((int64_t)m * ldc + (ncol >> 1)) * 2, pack8(o));
          continue;
        }
        if (ep.residual) {
          unpack8(rz[ii][0], f);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] += f[q];
          unpack8(rz[ii][1], f);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
        }
        st16<false>(C, crs, ((int64_t)m * ldc + ncol) * 2, pack8(v));
        st16<false>(C, crs, ((int64_t)m * ldc + ncol + 8) * 2, pack8(v + 8));
      } else if (!fast) {
        epi_store16_t<false>(v, m, ncol, M, N, C, ldc, ep, crs);
      }
    }
  }
}

template <int NS, bool SK>
static hipError_t launch_f8ks(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw,
                              const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep,
                              int grid, F8SkArgs sk, hipStream_t stream) {
  constexpr size_t lds = (size_t)NS * 2 * 128 * 128;   // >= 64 KiB swap + 8 x 4.25 KiB epilogue slabs
  static_assert(lds >= 65536 + 8 * 16 * 68 * 4, "epilogue LDS");
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm_f8ks_kernel<NS, SK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_f8ks_kernel<NS, SK>), dim3(grid), dim3(512), lds, stream, A, lda, sa, W, ldw, sw, C, ldc, M,
                     N, K, ep, sk);
  return hipGetLastError();
}

// stream_k: 1 = Stream-K (launch code 18), else the tile grid.  Not chosen automatically: at
// M = 624 it measured o 34.2 vs 23.5 us and down 66.4 vs 66.2 us (profiles/r5_f8_streamk_v1.txt) --
// these GEMMs are bound by the chip-wide L2 / MALL -> CU operand traffic (~8.8 TB/s for down's
// 578 MB of tile re-reads), which spreading the same tiles over 256 CUs does not reduce, and the
// partial-tile hand-off costs o its gain.
hipError_t gemm_f8ks(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw, const float* sw,
                     void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, hipStream_t stream, int stream_k) {
  if (K % 128 != 0 || N % 16 != 0 || M <= 0 || lda % 16 != 0 || ldw % 16 != 0) return hipErrorInvalidValue;
  if (ep.split_koff || ep.glu && ep.out_f32) return hipErrorInvalidValue;
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  const int nk = K / 128;
  int cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return hipErrorInvalidValue;
  const bool sk_ok = tiles < cus && !ep.glu;
  const bool use_sk = sk_ok && stream_k > 0;
  if (use_sk) {
    const int total = tiles * nk;
    const int L = (total + cus - 1) / cus;              // <= nk because tiles < cus
    const int grid = (total + L - 1) / L;
    float* ws = (float*)stream_workspace((size_t)grid * 2 * 16384 * sizeof(float), stream, WS_F8KS_SK, (size_t)32 << 20);
    int* cnt = (int*)stream_workspace((size_t)tiles * sizeof(int), stream, WS_F8KS_CNT, 4096, true);
    if (ws != nullptr && cnt != nullptr)
      return launch_f8ks<4, true>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, grid, F8SkArgs{L, ws, cnt}, stream);
  }
  return launch_f8ks<4, false>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, tiles, F8SkArgs{0, nullptr, nullptr},
                               stream);
}

}  // namespace lumen
