// FP8 x FP8 GEMM on the gfx950 block-scaled matrix cores (W8A8, per-token x per-channel).
//
//   C[M, N] = epi( (A8[M, K] . W8[N, K]^T) * sa[m] * sw[n] )
//
// A8 / W8 are OCP e4m3fn (gfx950's fp8 encoding, not the MI300 fnuz one); sa is the
// per-token activation scale written by the quantising producer (rms_norm_quant_fp8 /
// quant_rows_fp8 below), sw the per-output-channel weight scale of quantize_fp8_rows.
// The MFMA is v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 block scales (127): 128
// k-values per instruction at twice the bf16 per-clock rate (MI355X_MICROARCH.md, "FP8
// ~5 PF dense: block-scaled ... 2x BF16 per clock").  The fp32 scales are applied once
// in the epilogue, then the shared GEMM epilogue (fp32 bias, SwiGLU, residual) runs.
//
// This replaces the decoder's prefill projections (reference FastVLM decoder.onnx
// MatMuls, packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:420-492) and
// makes the former bf16 image of the dequantised weights + hipBLASLt path unnecessary.
//
// Tile: 128 x 128 x 128 B per K-step, 4 waves (2 x 2), each wave 64 x 64 = 4 x 4 MFMAs.
// Prefill M is a few hundred tokens, so 128-row tiles keep ~5 x N/128 workgroups in
// flight (240 for Llama-3-8B qkv at 624 tokens) where 256 x 256 tiles would leave most
// of the 256 CUs idle.  Operands stream with LDS-DMA (global_load_lds, 16 B per lane)
// into NSTAGE 32 KiB stages; one counted `s_waitcnt vmcnt` + raw s_barrier per K-step
// keeps NSTAGE-2 stages in flight across the barrier.  LDS rows are 128 B with the
// 16-byte chunk XOR swizzle of gemm_epi.h::swz applied on the per-lane *source*
// address.  Each MFMA lane reads two 16-byte chunks of its row: lane group g = lane/16
// takes chunks g and g+4 (k = 16g..16g+15 and 64+16g..64+16g+15), which is the
// instruction's own k order -- it runs as two k = 64 halves, VGPRs 0-3 then 4-7, lane
// group g holding 16 k of each -- and every ds_read_b128 lane group hits 64 distinct banks.
// In that order the 32-value block b (k = 32b..32b+31) spans lane groups 2(b&1), 2(b&1)+1
// of half b/2, and its E8M0 scale is the byte lane group b supplies (measured: a
// contiguous-32-per-lane assumption scaled the wrong k, tests/test_mx_gpu.py), so MX
// activations (gemm_mx) need no layout change: lane (row, g) passes row's scale of block g.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

#include "common.h"
#include "gemm_epi.h"
#include "workspace.h"

namespace lumen {

typedef int i32x8_t __attribute__((ext_vector_type(8)));

constexpr float FP8_MAX = 448.f;

template <int N>
__device__ __forceinline__ void f8_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// F8 = false: the same pipeline for bf16 operands (a 128-byte LDS row is 64 k-values; two
// v_mfma_f32_16x16x32_bf16 per fragment pair, lane group g reading k 8g..8g+7 and 32+8g..) --
// the mid-size bf16 GEMMs (a few hundred to a few thousand rows: VLM vision tower at 577
// tokens, bf16 decoder prefill) whose 256x256 tile counts cannot fill the chip.
// lda / ldw are in ELEMENTS of the operand type, K in elements; sa / sw may be null (1.0).
// BN: tile width (128, or 64 for grids whose 128x128 tiles leave CUs idle -- twice the tiles,
// 72 KiB of LDS at 3 stages so two workgroups share a CU).
// Stream-K form (SK): the grid is one workgroup per CU and the (tile, K-step) iteration space
// is cut into equal contiguous ranges, one per workgroup, so a mid-size GEMM whose 128x128 tiles
// cannot fill 256 CUs (LLaVA vision tower at 577 tokens: 40-160 tiles; 8B W8A8 prefill at 624
// tokens: 160-240 tiles) still keeps every CU streaming.  A tile whose K range spans several
// workgroups is combined in the launch: each contributor stores its fp32 accumulators
// write-through (sc1) to a slab, drains, and draws a ticket; the last arriver acquires, adds the
// other slabs to its registers and runs the normal epilogue (cdna_hip_programming.md Guideline 16,
// split-K seam).  Nobody waits on another workgroup, so residency is never assumed.
struct SkArgs {
  int ipw;          // (tile, K-step) iterations per workgroup
  int maxc;         // slab slots per tile (max contributors)
  float* ws;        // [tiles][maxc][128 * BN] fp32 slabs
  uint32_t* cnt;    // [tiles] arrival tickets (zero between launches: the last arriver resets)
};

// MX (block-scaled) operand and outputs of the W8A8 prefill chain (ops.linear_mx):
//  * BS launches read A's E8M0 exponents (one per row per 32 k) and feed them to the MFMA's A
//    scale operand, so any producer can quantise with block-local scales (no per-row pass);
//  * ssq_in: the producing GEMM's per-(row, column-tile) sums of squares -> rstd row scale (the
//    RMSNorm folded into this projection, gamma already folded into W: LLM.fold_norms);
//  * q8 / qs: an MX fp8 copy of this GEMM's output for the next projection (32-column blocks;
//    SwiGLU outputs need 64-column wave tiles so one 4-lane group owns a block);
//  * ssq_out: per-(row, BN tile) sums of squares of the stored bf16 output (residual stream).
// (MxArgs: gemm_epi.h)

constexpr int MX_SCRATCH = 40960;    // epilogue LDS bytes past the per-wave slabs: rstd[128], ssq[128][WN]

__device__ __forceinline__ void pp_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int NSTAGE, int WN, bool F8, int BN = 128, bool SK = false, bool BS = false, bool PP = false>
__global__ void __launch_bounds__(128 * WN)
gemm_f8_kernel(const uint8_t* __restrict__ A, int64_t lda, const float* __restrict__ sa, const uint8_t* __restrict__ W,
               int64_t ldw, const float* __restrict__ sw, void* __restrict__ C, int64_t ldc, int M, int N, int K,
               GemmEpi ep, SkArgs sk, MxArgs mx) {
  static_assert(!BS || F8, "block scales: fp8 operands only");
  constexpr int ES = F8 ? 1 : 2;         // bytes per element
  lda *= ES;
  ldw *= ES;
  constexpr int NW = 2 * WN;             // waves: 2 (M) x WN (N)
  constexpr int TN = BN / WN;            // wave tile 64 x TN
  constexpr int NR = TN / 16;
  constexpr int PER = 16 / NW;           // glds instructions per wave for the A image per stage
  constexpr int PERW = (BN / 8) / NW;    // ... and for the W image
  static_assert(NR >= 1 && PERW >= 1, "tile / wave split");
  constexpr int SCB = BS ? NW * 256 : 0;          // A scale bytes per stage (each wave: 64 rows x 4)
  constexpr int STAGE = 128 * 128 + BN * 128 + SCB;   // bytes: A image, W image, A scales
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = (M + 127) / 128, tiles_n = (N + BN - 1) / BN;
  if (!SK && ep.split_koff) {   // split-K (gridDim.y = splits): this workgroup's K slice -> its fp32 slab
    A += blockIdx.y * ep.split_koff * ES;
    W += blockIdx.y * ep.split_koff * ES;
    C = (float*)C + blockIdx.y * ep.split_cstride;
  }
  const int nk = K * ES / 128;
  const int frow = lane & 15, g = lane >> 4;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  f32x4_t acc[4][NR];

  // ---- K-steps [k0, k1) of tile (tm, tn) into acc (zeroed first)
  auto mainloop = [&](const int m0, const int n0, const int k0, const int k1) {
    // staging: wave wid, instruction i covers rows (PER*wid + i)*8 + lane/8 of the A image and
    // rows (PERW*wid + i)*8 + lane/8 of the W image
    const uint8_t* src_a[PER];
    const uint8_t* src_w[PERW];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int r = (PER * wid + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      src_a[i] = A + (int64_t)min(m0 + r, M - 1) * lda + c * 16;
    }
#pragma unroll
    for (int i = 0; i < PERW; ++i) {
      const int r = (PERW * wid + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      src_w[i] = W + (int64_t)min(n0 + r, N - 1) * ldw + c * 16;
    }
    // BS: every wave stages the 4 scale bytes of one 64-row half per K-step (waves 0 / 1 are the
    // copies the fragments read; the others keep the per-wave glds count uniform for vmcnt)
    // (scale planes [K/128][M][4]: a wave's 64 rows x 4 bytes are 256 contiguous bytes, 2 lines)
    const uint8_t* src_s = BS ? mx.a_bs + (int64_t)min(m0 + (wid & 1) * 64 + lane, M - 1) * 4 : nullptr;
    auto stage = [&](int s, int64_t koff) {
      char* base = smem + s * STAGE;
#pragma unroll
      for (int i = 0; i < PER; ++i)
        __builtin_amdgcn_global_load_lds((g_ptr_t)(src_a[i] + koff), (lds_ptr_t)(base + (wid * PER + i) * 1024), 16,
                                         0, 0);
#pragma unroll
      for (int i = 0; i < PERW; ++i)
        __builtin_amdgcn_global_load_lds((g_ptr_t)(src_w[i] + koff),
                                         (lds_ptr_t)(base + 128 * 128 + (wid * PERW + i) * 1024), 16, 0, 0);
      if constexpr (BS)
        __builtin_amdgcn_global_load_lds((g_ptr_t)(src_s + (koff >> 7) * mx.ld_bs),
                                         (lds_ptr_t)(base + 128 * 128 + BN * 128 + wid * 256), 4, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int n = k1 - k0;
#pragma unroll
    for (int s = 0; s < NSTAGE - 1; ++s)
      if (s < n) stage(s, (int64_t)(k0 + s) * 128);

    u32x4_t fa[4][2], fb[NR][2];
    int as[4];
    auto frags = [&](const int kt) {
      const char* sA = smem + (kt % NSTAGE) * STAGE;
      const char* sW = sA + 128 * 128;
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int r = wn * TN + j * 16 + frow;
        fb[j][0] = *(const u32x4_t*)(sW + swz(r, g));
        fb[j][1] = *(const u32x4_t*)(sW + swz(r, g + 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + frow;
        fa[i][0] = *(const u32x4_t*)(sA + swz(r, g));
        fa[i][1] = *(const u32x4_t*)(sA + swz(r, g + 4));
        if constexpr (BS) as[i] = *(const uint8_t*)(sA + 128 * 128 + BN * 128 + wm * 256 + (i * 16 + frow) * 4 + g);
        else as[i] = 127;
      }
    };
    auto mfmas = [&]() {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          if constexpr (F8) {
            const i32x8_t a8 = (i32x8_t){(int)fa[i][0][0], (int)fa[i][0][1], (int)fa[i][0][2], (int)fa[i][0][3],
                                         (int)fa[i][1][0], (int)fa[i][1][1], (int)fa[i][1][2], (int)fa[i][1][3]};
            const i32x8_t b8 = (i32x8_t){(int)fb[j][0][0], (int)fb[j][0][1], (int)fb[j][0][2], (int)fb[j][0][3],
                                         (int)fb[j][1][0], (int)fb[j][1][1], (int)fb[j][1][2], (int)fb[j][1][3]};
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[i][j], 0, 0, 0, as[i], 0, 127);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i][0]),
                                                                __builtin_bit_cast(bf16x8_t, fb[j][0]), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i][1]),
                                                                __builtin_bit_cast(bf16x8_t, fb[j][1]), acc[i][j], 0, 0, 0);
          }
        }
    };
    constexpr int P = PER + PERW + (BS ? 1 : 0);   // glds instructions per wave per stage
    if constexpr (PP) {
      // Ping-pong: wave group wm = 1 runs one barrier behind group 0, so on every SIMD one wave's
      // MFMAs overlap its partner's fragment reads and staging issue (the gemm_pp.hip schedule on
      // this 128 x 128 tile).  Phase kt of a group: read stage kt | issue stage kt + NSTAGE - 1 |
      // own DMAs of stage kt + 1 landed | barrier | MFMAs | barrier.  With the lag, stage kt + 1's
      // DMAs of BOTH groups were waited for before a barrier each group passes before reading it,
      // and the buffer a phase restages (stage kt - 1) was last read by the lagging group before
      // the barrier the leading group passed just before issuing.  Needs NSTAGE >= 3.
      static_assert(!PP || NSTAGE >= 3, "ping-pong needs a stage in flight across each phase");
      if (n > NSTAGE - 2) f8_vm_wait<P * (NSTAGE - 2)>();
      else f8_vm_wait<0>();
      pp_bar();
      if (wm == 1) pp_bar();
      for (int kt = 0; kt < n; ++kt) {
        frags(kt);
        if (kt + NSTAGE - 1 < n) {
          stage((kt + NSTAGE - 1) % NSTAGE, (int64_t)(k0 + kt + NSTAGE - 1) * 128);
          f8_vm_wait<P * (NSTAGE - 2)>();
        } else {
          f8_vm_wait<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_bar();
        __builtin_amdgcn_s_setprio(1);
        mfmas();
        __builtin_amdgcn_s_setprio(0);
        pp_bar();
      }
      if (wm == 0) pp_bar();
    } else {
      for (int kt = 0; kt < n; ++kt) {
        // stage kt landed for this wave (NSTAGE-2 younger stages may stay in flight) ...
        if (kt + NSTAGE - 2 < n) f8_vm_wait<P * (NSTAGE - 2)>();
        else f8_vm_wait<0>();
        // ... and for every wave; every wave is also done reading stage kt-1's buffer
        __builtin_amdgcn_s_barrier();
        if (kt + NSTAGE - 1 < n) stage((kt + NSTAGE - 1) % NSTAGE, (int64_t)(k0 + kt + NSTAGE - 1) * 128);
        frags(kt);
        mfmas();
      }
    }
    __syncthreads();   // every wave done with the stage buffers (the epilogue reuses them)
  };

  // ---- epilogue: per-wave 16-row slabs through LDS; lane -> (row, 16 columns)
  auto epilogue = [&](const int m0, const int n0) {
    constexpr int LDSTR = TN + 4;
    constexpr int LPR = TN / 16;           // lanes per row
    constexpr int RPP = 64 / LPR;          // rows per pass
    constexpr int NPASS = RPP >= 16 ? 1 : 16 / RPP;
    float* es = (float*)smem + wid * 16 * LDSTR;
    float* rstd_s = (float*)(smem + MX_SCRATCH);     // [128]
    float* ssq_s = rstd_s + 128;                      // [128][WN]
    const bool mx_out = mx.q8 != nullptr || mx.ssq_out != nullptr;
    if (mx.ssq_in) {
      // rstd of the tile's rows from the producer's partial sums of squares: WN threads per row
      // (128 * WN threads), their loads unrolled so they are all in flight at once, partial sums
      // in a fixed order through LDS
      constexpr int PARTS = WN;
      float* red = ssq_s;                             // [PARTS][128], free until the slab loop
      const int row = tid & 127, part = tid >> 7;
      const float* p = mx.ssq_in + (int64_t)min(m0 + row, M - 1) * mx.ssq_in_tiles;
      float ss = 0.f;
#pragma unroll 8
      for (int j = part; j < mx.ssq_in_tiles; j += PARTS) ss += p[j];
      red[part * 128 + row] = ss;
      __syncthreads();
      if (tid < 128) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < PARTS; ++q) t += red[q * 128 + tid];
        rstd_s[tid] = rsqrtf(t / (float)K + mx.norm_eps);
      }
      __syncthreads();
    }
    const int cc = (lane % LPR) * 16;
    const int n = n0 + wn * TN + cc;
    float cs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) cs[q] = n + q < N ? (sw ? sw[n + q] : 1.f) : 0.f;
    const __amdgpu_buffer_rsrc_t crs = c_rsrc(C);
    // Prefetched epilogue (plain bf16 stores: bias / activation / residual / LN-fold affine): every
    // per-row and per-column operand of the tile's 4 slabs is loaded once before the slab loop, so
    // no slab waits on a global round trip (the generic path loads residual rows, row_aff and
    // col_aff inside each slab).  NPASS == 1 here (TN >= 32).
    const bool fastep = NPASS == 1 && !mx_out && !ep.glu && !ep.out_group && !ep.table && !ep.prelu && !ep.post_act &&
                        !ep.out_f32 && !ep.split_koff && n + 16 <= N;
    const bool lnf = ep.row_aff != nullptr;
    float pa[16], pb[16], rsr[4], ror[4];
    u32x4_t res[4][2];
    if (fastep) {
      const int rr0 = lane / LPR;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        pa[q] = lnf ? ep.col_aff[n + q] : 0.f;
        pb[q] = lnf ? ep.col_aff[N + n + q]
                    : (ep.bias ? (ep.bias_f32 ? ((const float*)ep.bias)[n + q] : bf2f(((const uint16_t*)ep.bias)[n + q]))
                               : 0.f);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mc = min(m0 + wm * 64 + i * 16 + min(rr0, 15), M - 1);
        rsr[i] = lnf ? ep.row_aff[2 * (int64_t)mc] : 1.f;
        ror[i] = lnf ? ep.row_aff[2 * (int64_t)mc + 1] : 0.f;
        if (ep.residual) {
          const uint16_t* rp = ep.residual + (int64_t)mc * ep.ldr + n;
          res[i][0] = *(const u32x4_t*)rp;
          res[i][1] = *(const u32x4_t*)(rp + 8);
        }
      }
    }
    Unroll<0, 4>::run([&](const int i) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) es[(g * 4 + r) * LDSTR + j * 16 + frow] = acc[i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        const int rr = p * RPP + lane / LPR;
        if (rr >= 16) continue;             // whole LPR-lane row groups skip together
        const int mt = wm * 64 + i * 16 + rr, m = m0 + mt;
        float rs = m < M ? (sa ? sa[m] : 1.f) : 0.f;
        if (mx.ssq_in) rs *= rstd_s[mt];
        if (fastep) {
          float v[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = t[e] * rs * cs[q * 4 + e];
              v[q * 4 + e] = lnf ? a * rsr[i] + (ror[i] * pa[q * 4 + e] + pb[q * 4 + e]) : a * ep.alpha + pb[q * 4 + e];
            }
          }
          if (ep.act) apply_act_n<16>(v, ep.act);
          if (ep.residual) {
            float f[8];
            unpack8(res[i][0], f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += f[q];
            unpack8(res[i][1], f);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[8 + q] += f[q];
          }
          if (m < M) {
            st16<false>(C, crs, ((int64_t)m * ldc + n) * 2, pack8(v));
            st16<false>(C, crs, ((int64_t)m * ldc + n + 8) * 2, pack8(v + 8));
          }
          continue;
        }
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
          v[q * 4 + 0] = t[0] * rs * cs[q * 4 + 0];
          v[q * 4 + 1] = t[1] * rs * cs[q * 4 + 1];
          v[q * 4 + 2] = t[2] * rs * cs[q * 4 + 2];
          v[q * 4 + 3] = t[3] * rs * cs[q * 4 + 3];
        }
        if (!mx_out) {
          epi_store16_t<false>(v, m, n, M, N, C, ldc, ep, crs);
          continue;
        }
        const bool valid = m < M && n < N;
        if (ep.glu) {
          // SwiGLU -> 8 outputs [n/2, n/2 + 8); a 4-lane row group owns one 32-output MX block
          if (ep.bias) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
              v[q] += valid ? (ep.bias_f32 ? ((const float*)ep.bias)[n + q] : bf2f(((const uint16_t*)ep.bias)[n + q]))
                            : 0.f;
          }
          float r[8], am = 0.f;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            r[q] = valid ? v[q] * fast_rcp(1.f + __expf(-v[q])) * v[8 + q] : 0.f;
            am = fmaxf(am, fabsf(r[q]));
          }
          if (valid && !mx.skip_c) st16<false>(C, crs, ((int64_t)m * ldc + (n >> 1)) * 2, pack8(r));
          if constexpr (LPR >= 4) if (mx.q8) {     // host: SwiGLU + q8 only on 64-column wave tiles
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            am = fmaxf(am, __shfl_xor(am, 2, 64));
            const int e = mx_exp(am);
            if (valid) {
              *(uint2*)(mx.q8 + (int64_t)m * mx.ldq + (n >> 1)) = fp8x8_scaled(r, mx_inv(e));
              if ((lane & 3) == 0) mx.qs[(int64_t)(n >> 8) * mx.ldqs + m * 4 + ((n >> 6) & 3)] = (uint8_t)(e + 127);
            }
          }
          continue;
        }
        if (valid && !mx.skip_c) {
          epi_store16_t<false>(v, m, n, M, N, C, ldc, ep, crs);   // v -> the stored values (fp32)
        } else if (valid) {      // MX output only: the same transforms, no bf16 store
          if (ep.row_aff) {
            const float ra = ep.row_aff[2 * (int64_t)m], rb = ep.row_aff[2 * (int64_t)m + 1];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = v[q] * ra + rb * ep.col_aff[n + q] + ep.col_aff[N + n + q];
          }
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] *= ep.alpha;
          if (ep.bias) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
              v[q] += ep.bias_f32 ? ((const float*)ep.bias)[n + q] : bf2f(((const uint16_t*)ep.bias)[n + q]);
          }
          if (ep.act) apply_act_n<16>(v, ep.act);
        }
        float f[16], am = 0.f, ss = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          // what the bf16 output now holds (the fp32 value when only the MX copy is written)
          f[q] = valid ? (mx.skip_c ? v[q] : bf2f(f2bf(v[q]))) : 0.f;
          am = fmaxf(am, fabsf(f[q]));
          ss += f[q] * f[q];
        }
        if (mx.q8) {
          am = fmaxf(am, __shfl_xor(am, 1, 64));     // lanes 2k, 2k+1: one 32-column block
          const int e = mx_exp(am);
          if (valid) {
            const float inv = mx_inv(e);
            const uint2 lo = fp8x8_scaled(f, inv), hi = fp8x8_scaled(f + 8, inv);
            *(u32x4_t*)(mx.q8 + (int64_t)m * mx.ldq + n) = (u32x4_t){lo.x, lo.y, hi.x, hi.y};
            if ((lane & 1) == 0) mx.qs[(int64_t)(n >> 7) * mx.ldqs + m * 4 + ((n >> 5) & 3)] = (uint8_t)(e + 127);
          }
        }
        if (mx.ssq_out) {
          ss += __shfl_xor(ss, 1, 64);
          if constexpr (LPR >= 4) ss += __shfl_xor(ss, 2, 64);
          if (lane % LPR == 0) ssq_s[mt * WN + wn] = ss;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    });
    if (mx.ssq_out) {   // fixed-order sum over the WN column slices -> one partial per (row, BN tile)
      __syncthreads();
      if (tid < 128 && m0 + tid < M) {
        float ss = 0.f;
#pragma unroll
        for (int w = 0; w < WN; ++w) ss += ssq_s[tid * WN + w];
        mx.ssq_out[(int64_t)(m0 + tid) * mx.ssq_out_tiles + n0 / BN] = ss;
      }
    }
  };

  if constexpr (!SK) {
    // XCD-aware: consecutive logical tiles share a W column panel (row tiles fastest), and
    // xcd_remap hands each XCD a contiguous run of them -> each W panel is read from HBM once
    const int lin = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int tm = lin % tiles_m, tn = lin / tiles_m;
    mainloop(tm * 128, tn * BN, 0, nk);
    epilogue(tm * 128, tn * BN);
  } else {
    // logical workgroup l (consecutive l on one XCD) takes iterations [l * ipw, (l + 1) * ipw)
    const int l = xcd_remap(blockIdx.x, gridDim.x);
    const int total = tiles_m * tiles_n * nk;
    int it = l * sk.ipw;
    const int end = min(total, it + sk.ipw);
    __shared__ int last_flag;
    while (it < end) {
      const int t = it / nk, k0 = it % nk, k1 = min(nk, k0 + (end - it));
      const int tm = t % tiles_m, tn = t / tiles_m;
      mainloop(tm * 128, tn * BN, k0, k1);
      it += k1 - k0;
      if (k0 != 0 || k1 != nk) {
        const int first = (t * nk) / sk.ipw, lastw = ((t + 1) * nk - 1) / sk.ipw;
        const int nc = lastw - first + 1;
        float* slabs = sk.ws + (int64_t)t * sk.maxc * (128 * BN);
        // accumulator-register layout: wave, fragment (i, j), lane -> 16 contiguous bytes
        const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
            slabs + (int64_t)(l - first) * (128 * BN), (short)0, 128 * BN * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, acc[i][j]), srs,
                                                   (((wid * 4 + i) * NR + j) * 64 + lane) * 16, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
        __syncthreads();
        if (tid == 0) {
          const uint32_t prev = __hip_atomic_fetch_add(sk.cnt + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const bool last = prev == (uint32_t)(nc - 1);
          if (last) {
            __hip_atomic_store(sk.cnt + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          last_flag = last ? 1 : 0;
        }
        __syncthreads();
        if (!last_flag) continue;
        // every slab (this workgroup's own too) summed in contributor order: the result does not
        // depend on which contributor arrived last (bit-identical launches and graph replays)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < nc; ++c) {
          const float* src = slabs + (int64_t)c * (128 * BN);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NR; ++j) {
              const f32x4_t v = *(const f32x4_t*)(src + (((wid * 4 + i) * NR + j) * 64 + lane) * 4);
              acc[i][j] += v;
            }
        }
      }
      epilogue(tm * 128, tn * BN);
      __syncthreads();   // the epilogue's LDS slabs are free before the next tile's staging
    }
  }
}

template <int NS, int WN, bool BS, int BN>
static constexpr size_t f8_lds() {
  return (size_t)NS * (128 * 128 + BN * 128 + (BS ? 2 * WN * 256 : 0));
}

template <int NS, int WN, bool F8 = true, int BN = 128, bool BS = false, bool PP = false>
static hipError_t launch_f8(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw,
                            const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep,
                            hipStream_t stream, int splits = 1, const MxArgs& mx = MxArgs{}) {
  constexpr size_t lds = f8_lds<NS, WN, BS, BN>();
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm_f8_kernel<NS, WN, F8, BN, false, BS, PP>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int tiles = ((M + 127) / 128) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_f8_kernel<NS, WN, F8, BN, false, BS, PP>), dim3(tiles, splits), dim3(128 * WN), lds, stream,
                     A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, SkArgs{}, mx);
  return hipGetLastError();
}

// Stream-K launch (see SkArgs): grid = min(CUs, iterations), slabs / tickets in the stream's
// workspace.  Returns hipErrorNotReady when no workspace is available (graph capture of a first
// call): the caller falls back to the tiled launch.
static uint32_t* sk_counters(size_t n, hipStream_t stream);
static float* sk_slabs(size_t bytes, hipStream_t stream);
static int f8_num_cus();

template <int NS, int WN, bool F8 = true, int BN = 128, bool BS = false, bool PP = false>
static hipError_t launch_f8_sk(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw,
                               const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep,
                               hipStream_t stream, const MxArgs& mx = MxArgs{}) {
  constexpr int ES = F8 ? 1 : 2;
  const int tiles = ((M + 127) / 128) * ((N + BN - 1) / BN);
  const int nk = K * ES / 128;
  const int total = tiles * nk;
  const int grid = std::min(f8_num_cus(), total);
  SkArgs sk{};
  sk.ipw = (total + grid - 1) / grid;
  sk.maxc = (nk + sk.ipw - 1) / sk.ipw + 1;
  sk.ws = sk_slabs((size_t)tiles * sk.maxc * 128 * BN * sizeof(float), stream);
  sk.cnt = sk_counters((size_t)tiles, stream);
  if (sk.ws == nullptr || sk.cnt == nullptr) return hipErrorNotReady;
  constexpr size_t lds = f8_lds<NS, WN, BS, BN>();
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm_f8_kernel<NS, WN, F8, BN, true, BS, PP>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int used = (total + sk.ipw - 1) / sk.ipw;   // workgroups with work
  hipLaunchKernelGGL((gemm_f8_kernel<NS, WN, F8, BN, true, BS, PP>), dim3(used), dim3(128 * WN), lds, stream, A, lda,
                     sa, W, ldw, sw, C, ldc, M, N, K, ep, sk, mx);
  return hipGetLastError();
}

// 256 x 256 ping-pong form (csrc/gemm_f8pp.hip); splits <= 0: automatic
hipError_t gemm_f8pp(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw, const float* sw,
                     void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, int splits, hipStream_t stream);
// intra-workgroup split-K form (csrc/gemm_f8ks.hip)
hipError_t gemm_f8ks(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw, const float* sw,
                     void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, hipStream_t stream,
                     int stream_k = -1);

// ---------------------------------------------------------------------------- split-K
// Mid-size GEMMs whose 128x128 tile count leaves CUs idle (LLaVA vision tower at 577 tokens:
// 40-160 tiles; 8B prefill o / down at 624 tokens: 160) split K over gridDim.y: each split
// writes scaled fp32 partials to its slab, one reduce pass sums the slabs in split order
// (deterministic) and runs the real epilogue (bias / act / SwiGLU / residual, 16 columns per
// thread).  Slabs live in a per-(device, stream) workspace; never during graph capture.
__global__ void __launch_bounds__(256)
splitk_reduce16_kernel(const float* __restrict__ slabs, int S, int M, int N, void* __restrict__ C, int64_t ldc,
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
  e.alpha = 1.f;   // scales were applied by the slab GEMM
  epi_store16_t<false>(v, m, n, M, N, C, ldc, e, c_rsrc(C));
}

static float* split_workspace(size_t bytes, hipStream_t stream) {
  return (float*)stream_workspace(bytes, stream, WS_F8_SPLIT, (size_t)32 << 20);
}

static float* sk_slabs(size_t bytes, hipStream_t stream) {
  return (float*)stream_workspace(bytes, stream, WS_SK_SLAB, (size_t)16 << 20);
}

static uint32_t* sk_counters(size_t n, hipStream_t stream) {
  return (uint32_t*)stream_workspace(n * sizeof(uint32_t), stream, WS_SK_CNT, 65536, true);
}

static int f8_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

// K splits for a 128x128-tile GEMM: only grids of at most half the CUs split, to ~1-2
// workgroups per CU, keeping >= 4 k tiles (128 B) per split
static int f8_pick_splits(int tiles, int nk, const GemmEpi& ep) {
  if (ep.out_group || ep.table || ep.split_koff || ep.prelu || ep.post_act) return 1;
  const int cus = f8_num_cus();
  int S = 1;
  // (r3, warm caches, M = 624: 2-way split of the 160-tile down projection 62.3 -> 59.4 us, K = 4096
  // shapes lose at S = 2: 23.8 -> 31.7 us, profiles/r3_f8_splits_v1.txt; in the cold-weight prefill
  // the down split did not show a TTFT gain, so the single-wave grid stays unsplit)
  if (2 * tiles <= cus && nk >= 32) {
    // deep K only: the fp32 slab round trip costs more than the idle CUs on K <= 1024 shapes
    // (577 x 3072 x 1024: 14.2 -> 28.2 us split; 577 x 1024 x 4096: 35.8 -> 25.8 us;
    // 624 x 4096 x 14336 fp8: 61.9 -> 57.4 us at S = 2; profiles/r2_splitk_mid_v1.txt)
    for (int c : {2, 3, 4, 6, 8})
      if (tiles * c <= 2 * cus && nk % c == 0 && nk / c >= 8) S = c;
  }
  while (S > 1 && (nk % S != 0 || nk / S < 2)) --S;
  return S;
}

template <int NS, int WN, bool F8, int BN = 128>
static hipError_t launch_f8_split(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw,
                                  const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep,
                                  int S, hipStream_t stream) {
  constexpr int ES = F8 ? 1 : 2;
  float* slabs = split_workspace((size_t)S * M * N * sizeof(float), stream);
  if (slabs == nullptr) return launch_f8<NS, WN, F8, BN>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
  GemmEpi e{};
  e.alpha = 1.f;
  e.out_f32 = 1;
  e.split_koff = (int64_t)(K / S);
  e.split_cstride = (int64_t)M * N;
  (void)ES;
  hipError_t err = launch_f8<NS, WN, F8, BN>(A, lda, sa, W, ldw, sw, slabs, N, M, N, K / S, e, stream, S);
  if (err != hipSuccess) return err;
  const int64_t work = (int64_t)M * (N / 16);
  hipLaunchKernelGGL(splitk_reduce16_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, slabs, S, M,
                     N, C, ldc, ep);
  return hipGetLastError();
}

// Pipeline shapes (NSTAGE x waves x tile width), selected by a variant code:
//   1 = <2 stages, 4 waves, 128>   2 = <3, 8, 128>   3 = <4, 8, 128>   4 = <4, 4, 128>
//   5 = <2, 8, 128>                6 = <3, 8, 256>   7 = <2, 8, 256>   8 = <5, 8, 128>
// 128 x 256 tiles halve the A/W staging bytes per MFMA of 128 x 128 ones; deeper rings keep
// more bytes in flight per CU for the cold-weight (HBM-latency-bound) regime of a layer stack.
// r4 also measured, and removed: a blocked weight layout (each K-step's W slice contiguous: no
// change, so not TLB-bound) and a software-pipelined loop (fragments of step k + 1 read during the
// MFMAs of step k: no change); every shape runs ~0.53 us per 128-byte K-step + ~7 us per launch
// (profiles/r4_cold_gemm_blocked_sp_v1.txt, r4_f8_gemm_time_vs_k_v1.txt).
//   9 = stream-K <3, 8, 128>   10 = stream-K <4, 4, 128>   11 = stream-K <4, 8, 128>
//  12 / 13 / 14 = ping-pong <3 / 4 / 5 stages, 8 waves, 128>   15 = stream-K ping-pong <4, 8, 128>
static int variant_bn(int v) { return v == 6 || v == 7 ? 256 : 128; }

template <bool F8>
static hipError_t launch_variant(int v, const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw,
                                 const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, int S,
                                 hipStream_t stream) {
  if (v == 17) {               // 256 x 256 ping-pong (fp8 only; its own split-K)
    if constexpr (F8) {
      if (ep.split_koff == 0) return gemm_f8pp(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S > 1 ? S : -1, stream);
    }
    v = 2;
  }
  if (v == 16 || v == 18) {    // intra-workgroup split-K (fp8 only; its own plain epilogues); 18: + Stream-K
    if constexpr (F8) {
      if (ep.split_koff == 0 && S == 1)
        return gemm_f8ks(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream, v == 18 ? 1 : 0);
    }
    v = 2;
  }
  if ((v >= 9 && v <= 11) || v == 15) {
    if (ep.split_koff == 0) {
      hipError_t e = v == 9 ? launch_f8_sk<3, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream)
                   : v == 10 ? launch_f8_sk<4, 2, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream)
                   : v == 11 ? launch_f8_sk<4, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream)
                             : launch_f8_sk<4, 4, F8, 128, false, true>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep,
                                                                          stream);
      if (e != hipErrorNotReady) return e;
    }
    v = v == 15 ? 13 : 2;      // no workspace (first call inside a graph capture): the tiled pipeline
    S = 1;
  }
  if (v >= 12 && v <= 14) {    // ping-pong forms: no split-K slabs
    if (v == 12) return launch_f8<3, 4, F8, 128, false, true>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    if (v == 13) return launch_f8<4, 4, F8, 128, false, true>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    return launch_f8<5, 4, F8, 128, false, true>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
  }
  if (S > 1) {
    switch (v) {
      case 1: return launch_f8_split<2, 2, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      case 3: return launch_f8_split<4, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      case 4: return launch_f8_split<4, 2, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      case 5: return launch_f8_split<2, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      case 6: return launch_f8_split<3, 4, F8, 256>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      case 7: return launch_f8_split<2, 4, F8, 256>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      case 8: return launch_f8_split<5, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
      default: return launch_f8_split<3, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
    }
  }
  switch (v) {
    case 1: return launch_f8<2, 2, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    case 3: return launch_f8<4, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    case 4: return launch_f8<4, 2, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    case 5: return launch_f8<2, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    case 6: return launch_f8<3, 4, F8, 256>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    case 7: return launch_f8<2, 4, F8, 256>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    case 8: return launch_f8<5, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
    default: return launch_f8<3, 4, F8>(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
  }
}

// bf16 operands on the same 128x128 LDS-DMA pipeline (K % 64 == 0, 16-byte aligned rows)
hipError_t gemm_lds128_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc,
                            int M, int N, int K, const GemmEpi& ep, int variant, hipStream_t stream) {
  if (K % 64 != 0 || N % 16 != 0 || M <= 0 || lda % 8 != 0 || ldw % 8 != 0) return hipErrorInvalidValue;
  const uint8_t* a = (const uint8_t*)A;
  const uint8_t* w = (const uint8_t*)W;
  // variant (bf16 tile codes 2000v): 0 = auto; 2 / 3 / 5 keep their r2 meaning (<2,2> / <3,4> / <2,4>);
  // 10 + v selects launch_variant's code v (deeper rings, 128 x 256 tiles)
  int code = variant >= 10 ? variant - 10 : variant == 2 ? 1 : variant == 5 ? 5 : variant == 0 ? 0 : 2;
  const int bn = variant_bn(code);
  const int tiles = ((M + 127) / 128) * ((N + bn - 1) / bn);
  int S = f8_pick_splits(tiles, K / 64, ep);
  if (code == 0) code = tiles * S > f8_num_cus() ? 1 : 2;
  return launch_variant<false>(code, a, lda, nullptr, w, ldw, nullptr, C, ldc, M, N, K, ep, S, stream);
}

hipError_t gemm_f8(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw, const float* sw,
                   void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, hipStream_t stream, int splits,
                   int variant) {
  if (K % 128 != 0 || N % 16 != 0 || M <= 0 || lda % 16 != 0 || ldw % 16 != 0) return hipErrorInvalidValue;
  // Measured at M = 624 on the Llama-3-8B projections (profiles/r2_f8_gemm_variants_v1.txt):
  // grids of more than one wave of workgroups (gate|up: 1120 tiles) run best at 2 stages x
  // 4 waves (64 KiB LDS -> 2 workgroups per CU overlap each other's barriers); grids that
  // fit in one wave (qkv / o / down: 160-240 tiles) at 3 stages x 8 waves (2 waves / SIMD).
  // (128x64 tiles were faster in isolation but slower over the whole weight-streaming prefill,
  // 9.87 vs 9.23-9.35 ms, profiles/r2_f8_bn64_v1.txt, and were removed.)
  const int bn = variant > 0 ? variant_bn(variant) : 128;
  const int tiles = ((M + 127) / 128) * ((N + bn - 1) / bn);
  int S = f8_pick_splits(tiles, K / 128, ep);
  if (splits > 0 && !(ep.out_group || ep.table || ep.split_koff || ep.prelu || ep.post_act)) {   // forced (benchmarks)
    S = splits;
    while (S > 1 && ((K / 128) % S != 0 || (K / 128) / S < 2)) --S;
  }
  const bool multi_wave = tiles * S > f8_num_cus();
  if (variant > 0) return launch_variant<true>(variant, A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
  // r5 (profiles/r5_f8_variants_cold_v1.txt): at prefill sizes (M <= 768) the intra-workgroup
  // split-K 128 x 128 form (code 16) runs the single-round grids (qkv / o / down: 23.8-66.1 us cold
  // vs 26.1-69.5 for code 2), the 256 x 256 ping-pong (code 17: twice the FLOP per staged byte) the
  // multi-round ones (gate|up, 1120 tiles of 128 x 128: 91.6 us vs 95.0 with its last partial
  // round on code 16 and 106.4 for code 1)
  const bool plain = !(ep.out_group || ep.table || ep.prelu || ep.post_act || ep.split_koff || ep.row_aff ||
                       (ep.glu && ep.out_f32));
  if (plain && splits <= 0 && M <= 768 && K >= 1024) {
    if (tiles > f8_num_cus() && N % 256 == 0) return gemm_f8pp(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, 1, stream);
    return gemm_f8ks(A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, stream);
  }
  return launch_variant<true>(multi_wave ? 1 : 2, A, lda, sa, W, ldw, sw, C, ldc, M, N, K, ep, S, stream);
}

// W8A8 with MX-scaled activations (ops.linear_mx, the fused prefill chain of LLM._layers_mx).
// No split-K (its slab reduce has no MX epilogue).  Codes as launch_variant; SwiGLU with an MX
// output needs 64-column wave tiles (codes 1, 4, 10), a sums-of-squares output 128-column tiles.
hipError_t gemm_mx(const uint8_t* A, int64_t lda, const uint8_t* a_bs, int64_t ld_bs, const uint8_t* W, int64_t ldw,
                   const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, MxArgs mx,
                   hipStream_t stream, int variant) {
  if (K % 128 != 0 || N % 16 != 0 || M <= 0 || lda % 16 != 0 || ldw % 16 != 0 || ld_bs < 4 * (int64_t)M ||
      ld_bs % 4 != 0)
    return hipErrorInvalidValue;
  if (ep.split_koff || ep.out_group || ep.table || ep.prelu || ep.post_act) return hipErrorInvalidValue;
  if (mx.skip_c && !mx.q8) return hipErrorInvalidValue;
  mx.a_bs = a_bs;
  mx.ld_bs = ld_bs;
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  const bool multi_wave = tiles > f8_num_cus();
  int v = variant > 0 ? variant : (multi_wave ? 1 : 2);
  if (ep.glu && mx.q8 && !(v == 1 || v == 4 || v == 10)) v = multi_wave ? 1 : 4;
  hipError_t e = hipErrorNotReady;
  switch (v) {
    case 9: e = launch_f8_sk<3, 4, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, mx); break;
    case 10: e = launch_f8_sk<4, 2, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, mx); break;
    case 11: e = launch_f8_sk<4, 4, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, mx); break;
    case 15:
      e = launch_f8_sk<4, 4, true, 128, true, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, mx);
      break;
    default: break;
  }
  if (e != hipErrorNotReady) return e;
  if (v >= 9 && v <= 11) v = v == 10 ? 4 : 2;    // no stream-K workspace (first call inside a graph capture)
  if (v == 15) v = 13;
  switch (v) {
    case 12:
      return launch_f8<3, 4, true, 128, true, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
    case 13:
      return launch_f8<4, 4, true, 128, true, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
    case 1: return launch_f8<2, 2, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
    case 3: return launch_f8<4, 4, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
    case 4: return launch_f8<4, 2, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
    case 5: return launch_f8<2, 4, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
    default: return launch_f8<3, 4, true, 128, true>(A, lda, nullptr, W, ldw, sw, C, ldc, M, N, K, ep, stream, 1, mx);
  }
}

// ============================================================================ quantisers
// Per-token dynamic quantisation: scale[m] = max|y[m, :]| / 448, out = e4m3(y / scale).
// One 256-thread workgroup per row; rows are re-read (L2-resident) instead of being held
// in registers so one kernel covers every hidden / intermediate width.

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  return v;
}
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  v = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return v;
}

// 8 floats (already divided by the scale) -> 8 e4m3 bytes
__device__ __forceinline__ uint2 to_fp8x8(const float* f) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}

__global__ void __launch_bounds__(256) quant_rows_fp8_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                             uint8_t* __restrict__ out, int64_t ldo,
                                                             float* __restrict__ scale, int K) {
  __shared__ float red[4];
  const int64_t m = blockIdx.x;
  const uint16_t* xr = x + m * ldx;
  // the row stays in registers (K <= 16384: 8 chunks of 8 per thread), every chunk's load in
  // flight at once: one round trip instead of one per 2048 columns per pass, and no second read
  constexpr int NC = 8;
  u32x4_t raw[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int k = (threadIdx.x + c * 256) * 8;
    raw[c] = k < K ? *(const u32x4_t*)(xr + k) : (u32x4_t){0u, 0u, 0u, 0u};
  }
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float f[8];
    unpack8(raw[c], f);
#pragma unroll
    for (int q = 0; q < 8; ++q) amax = fmaxf(amax, fabsf(f[q]));
  }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-12f) / FP8_MAX;
  if (threadIdx.x == 0) scale[m] = s;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int k = (threadIdx.x + c * 256) * 8;
    if (k >= K) break;
    float f[8];
    unpack8(raw[c], f);
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = fminf(fmaxf(f[q] / s, -FP8_MAX), FP8_MAX);   // IEEE divide: bit-identical to x / s on the host
    *(uint2*)(out + m * ldo + k) = to_fp8x8(f);
  }
}

// K > 16384: two passes over global memory
__global__ void __launch_bounds__(256) quant_rows_fp8_wide_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                                  uint8_t* __restrict__ out, int64_t ldo,
                                                                  float* __restrict__ scale, int K) {
  __shared__ float red[4];
  const int64_t m = blockIdx.x;
  const uint16_t* xr = x + m * ldx;
  float amax = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    float f[8];
    unpack8(*(const u32x4_t*)(xr + k), f);
#pragma unroll
    for (int q = 0; q < 8; ++q) amax = fmaxf(amax, fabsf(f[q]));
  }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-12f) / FP8_MAX;
  if (threadIdx.x == 0) scale[m] = s;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    float f[8];
    unpack8(*(const u32x4_t*)(xr + k), f);
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = fminf(fmaxf(f[q] / s, -FP8_MAX), FP8_MAX);
    *(uint2*)(out + m * ldo + k) = to_fp8x8(f);
  }
}

// RMSNorm (optionally after x += add, written back to resid_out) fused with the
// per-token fp8 quantisation of its output: the qkv / gate|up GEMM inputs of the decoder.
// Same numerics as norm_rows_kernel mode 1 (fp32 sum, y = x * rstd * gamma, no
// intermediate rounding).  The row stays in registers (K <= 16384: 8 chunks of 8 per thread).
__global__ void __launch_bounds__(256) rms_norm_quant_fp8_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                                 const uint16_t* __restrict__ add, int64_t ldadd,
                                                                 uint16_t* __restrict__ resid_out, int64_t ldr,
                                                                 const uint16_t* __restrict__ gamma, float eps,
                                                                 uint8_t* __restrict__ out, int64_t ldo,
                                                                 float* __restrict__ scale, int K) {
  __shared__ float red[4];
  const int64_t m = blockIdx.x;
  float v[8][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int k = (threadIdx.x + c * 256) * 8;
    if (k < K) {
      unpack8(*(const u32x4_t*)(x + m * ldx + k), v[c]);
      if (add) {
        float a[8];
        unpack8(*(const u32x4_t*)(add + m * ldadd + k), a);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[c][q] += a[q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) ss += v[c][q] * v[c][q];
    }
  }
  if (resid_out) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int k = (threadIdx.x + c * 256) * 8;
      if (k < K) *(u32x4_t*)(resid_out + m * ldr + k) = pack8(v[c]);
    }
  }
  const float rstd = rsqrtf(block_sum(ss, red) / (float)K + eps);
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int k = (threadIdx.x + c * 256) * 8;
    if (k < K) {
      float gm[8];
      unpack8(*(const u32x4_t*)(gamma + k), gm);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        v[c][q] = v[c][q] * rstd * gm[q];
        amax = fmaxf(amax, fabsf(v[c][q]));
      }
    }
  }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-12f) / FP8_MAX;
  if (threadIdx.x == 0) scale[m] = s;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int k = (threadIdx.x + c * 256) * 8;
    if (k < K) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[c][q] = fminf(fmaxf(v[c][q] / s, -FP8_MAX), FP8_MAX);
      *(uint2*)(out + m * ldo + k) = to_fp8x8(v[c]);
    }
  }
}

// bf16 rows -> MX fp8 (E8M0 per 32 columns) + per-(row, 128-column) sums of squares: the first
// layer's input of the MX prefill chain (later layers get theirs from the GEMM epilogues).
// One wave per row slice of 512 columns: lane -> 8 columns, 4 lanes per MX block, 16 per ssq tile.
__global__ void __launch_bounds__(256) quant_rows_mx_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                            uint8_t* __restrict__ q8, int64_t ldq,
                                                            uint8_t* __restrict__ qs, int64_t ldqs,
                                                            float* __restrict__ ssq, int64_t ldss, int M, int K) {
  const int lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // (row, 512-column slice)
  const int slices = (K + 511) / 512;
  if (item >= (int64_t)M * slices) return;
  const int64_t m = item / slices;
  const int k = (int)(item % slices) * 512 + lane * 8;
  const bool valid = k < K;
  float f[8], am = 0.f, ss = 0.f;
  if (valid) unpack8(*(const u32x4_t*)(x + m * ldx + k), f);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (!valid) f[q] = 0.f;
    am = fmaxf(am, fabsf(f[q]));
    ss += f[q] * f[q];
  }
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o, 64);
  if (!valid) return;
  const int e = mx_exp(am);
  *(uint2*)(q8 + m * ldq + k) = fp8x8_scaled(f, mx_inv(e));
  if ((lane & 3) == 0) qs[(k >> 7) * ldqs + m * 4 + ((k >> 5) & 3)] = (uint8_t)(e + 127);
  if (ssq && (lane & 15) == 0) ssq[m * ldss + (k >> 7)] = ss;
}

hipError_t quant_rows_mx(const uint16_t* x, int64_t ldx, uint8_t* q8, int64_t ldq, uint8_t* qs, int64_t ldqs,
                         float* ssq, int64_t ldss, int M, int K, hipStream_t stream) {
  if (K % 128 != 0 || M <= 0 || ldx % 8 != 0) return hipErrorInvalidValue;
  const int64_t items = (int64_t)M * ((K + 511) / 512);
  hipLaunchKernelGGL(quant_rows_mx_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, stream, x, ldx, q8, ldq, qs,
                     ldqs, ssq, ldss, M, K);
  return hipGetLastError();
}

hipError_t quant_rows_fp8(const uint16_t* x, int64_t ldx, uint8_t* out, int64_t ldo, float* scale, int M, int K,
                          hipStream_t stream) {
  if (K % 8 != 0 || M <= 0) return hipErrorInvalidValue;
  if (K <= 16384)
    hipLaunchKernelGGL(quant_rows_fp8_kernel, dim3(M), dim3(256), 0, stream, x, ldx, out, ldo, scale, K);
  else
    hipLaunchKernelGGL(quant_rows_fp8_wide_kernel, dim3(M), dim3(256), 0, stream, x, ldx, out, ldo, scale, K);
  return hipGetLastError();
}

hipError_t rms_norm_quant_fp8(const uint16_t* x, int64_t ldx, const uint16_t* add, int64_t ldadd, uint16_t* resid_out,
                              int64_t ldr, const uint16_t* gamma, float eps, uint8_t* out, int64_t ldo, float* scale,
                              int M, int K, hipStream_t stream) {
  if (K % 8 != 0 || K > 16384 || M <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rms_norm_quant_fp8_kernel, dim3(M), dim3(256), 0, stream, x, ldx, add, ldadd, resid_out, ldr,
                     gamma, eps, out, ldo, scale, K);
  return hipGetLastError();
}

}  // namespace lumen
