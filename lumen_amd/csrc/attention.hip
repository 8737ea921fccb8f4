// Fused multi-head attention forward (flash-style, online softmax) for gfx950.
//
// Transposed-score formulation so that P never leaves registers:
//   S^T[key][q]  = K . Q^T          (A = K rows from LDS via ds_read_b128,
//                                    B = Q^T fragment held in registers)
//   O^T[d][q]   += V^T . P^T        (A = V^T via ds_read_b64_tr_b16 hardware
//                                    transpose reads of the row-major V image,
//                                    B = P^T packed straight from the S^T
//                                    accumulators: the k-order of the two
//                                    operands is permuted identically)
// Each lane owns one query column (lane & 15), so the online-softmax row
// statistics are per-lane values reduced over the 4 lanes {l, l^16, l^32, l^48}.
//
// One workgroup = 4 waves = 64 queries of one (batch, head); each wave owns 16.
// K/V stream through LDS in 64-key chunks, double-buffered and filled by
// LDS-DMA (global_load_lds_dwordx4) with the XOR swizzle on the source address.
//
// Covers every attention the reference runs inside its ONNX graphs:
// non-causal ViT (CLIP/BioCLIP vision, seq 197/257/577), causal CLIP text (77),
// key-padded BERT (CN-CLIP), causal GQA decoder prefill (Qwen2 / Llama).
// Q/K/V are read in place from packed projections via strides, and O is
// written as [b, s, h, d] so the out-projection GEMM consumes it directly.
#include <cstdlib>
#include <type_traits>
#include "attention.h"
#include "common.h"
#include "tuning.h"

namespace lumen {

// AttnArgs: attention.h
typedef short s16x4v __attribute__((ext_vector_type(4)));

// K image: rows of D bf16; 16-byte chunk XOR so the ds_read_b128 A-fragment
// reads of 16 consecutive rows are conflict-free.
template <int D>
__device__ __forceinline__ int k_phys(int row, int chunk) {
  if constexpr (D == 64) return chunk ^ ((row >> 1) & 7);
  else if constexpr (D == 128) return chunk ^ (row & 15);
  else return chunk ^ ((row >> 2) & 3);
}
// V image: rows of D bf16; chunk XOR so that a 32-lane half of
// ds_read_b64_tr_b16 (8 rows x 32 bytes) covers all 64 banks.
template <int D>
__device__ __forceinline__ int v_phys(int row, int chunk) {
  if constexpr (D == 64) return chunk ^ (((row >> 1) & 3) << 1);
  else if constexpr (D == 128) return chunk ^ ((row & 7) << 1);
  else return chunk ^ (((row >> 2) & 1) << 1);
}

// max over the 4 lane groups (lane, lane ^ 16, lane ^ 32, lane ^ 48) with the gfx950 row swaps:
// v_permlane16_swap / v_permlane32_swap stay in the VALU (the __shfl_xor form is two
// ds_bpermute LDS round trips, each waited with lgkmcnt(0), in every chunk).  The max itself is
// a bare v_max_f32: the swapped values are finite or -inf scores, so the IEEE-mode
// canonicalisations hipcc inserts around fmaxf of an opaque value are not needed.
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float group4_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = vmax_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_raw(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

__device__ __forceinline__ s16x4v ds_read_tr16(const char* p) {
  typedef __attribute__((address_space(3))) s16x4v* lp;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(p));
}
typedef __attribute__((address_space(3))) const char lds_char;
__device__ __forceinline__ s16x4v ds_read_tr16(const lds_char* p) {
  typedef __attribute__((address_space(3))) s16x4v* lp;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(p));
}

// ----------------------------------------------------------------------------------------------
// Online-softmax step on one 64-key chunk of S^T (lane: query col, keys kb16*16 + 4g + r).
// VALU per score is what bounds D = 64 attention (0.25 MFMA cycles vs ~1 VALU cycle per
// score), so per score this costs one max (max3-fused) on the RAW score, one FMA folding
// the softmax scale and the max subtraction, one bare v_exp_f32 (exp2f adds a denormal
// range fix-up: cmp/cndmask/ldexp) and half a cvt_pk.  The row sum comes from an MFMA
// against a ones fragment in the PV loop (l4), and O / l4 are only rescaled when some
// lane's max grew by more than 8 in log2 units (lazy rescale: p <= 256 is exact enough in
// fp32 accumulators and bf16 P).
// ----------------------------------------------------------------------------------------------
template <int NB, int MASK>
__device__ __forceinline__ void softmax_chunk(f32x4_t (&sc)[4], f32x4_t (&o)[NB], f32x4_t& l4, float& mrow,
                                              const AttnArgs& a, bool need_mask, int k0, int g, int qi,
                                              int kv_len, int causal_off) {
  float mx = -INFINITY;
  // MASK: 0 = no key mask, 1 = masked, 2 = runtime need_mask.  As a runtime flag hipcc if-converts
  // the masked path into every chunk (~80 extra VALU per 18 MFMAs of the ViT K/V-resident kernel,
  // profiles/r6_attn_pmc_v1.txt): attn_res_kernel runs its clean chunks with 0; the streaming
  // attn_fwd_kernel keeps 2 (two inlined copies behind a branch measured worse there: 431 -> 577 VALU)
  if (MASK == 1 || (MASK == 2 && need_mask)) {
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kj = k0 + kb16 * 16 + g * 4 + r;
        bool ok = kj < kv_len;
        if (a.causal) ok = ok && (kj <= qi + causal_off);
        const float sv = ok ? sc[kb16][r] : -INFINITY;
        sc[kb16][r] = sv;
        mx = fmaxf(mx, sv);
      }
  } else {
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sc[kb16][r]);
  }
  mx = group4_max(mx);
  const float mcand = vmax_raw(mrow, mx * a.scale_log2);       // scale > 0 commutes with max
  if (__any(mcand > mrow + 8.f)) {                              // wave-uniform; first chunk: mrow = -inf
    const float mb = mcand == -INFINITY ? 0.f : mcand;
    const float alpha = __builtin_amdgcn_exp2f(mrow - mb);
#pragma unroll
    for (int j = 0; j < NB; ++j) o[j] *= alpha;
    l4 *= alpha;
    mrow = mcand;
  }
  const float nmb = mrow == -INFINITY ? 0.f : -mrow;
#pragma unroll
  for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
    for (int r = 0; r < 4; ++r) sc[kb16][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb16][r], a.scale_log2, nmb));
}

__device__ __forceinline__ bf16x8_t ones_bf16x8() {
  return __builtin_bit_cast(bf16x8_t, (s16x8_t){0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80});
}

// NW waves per workgroup, 16 queries each (a 16*NW-query block): NW = 2 doubles the workgroup
// count of the few-(batch, head) prefills (one LLaVA image: 16 heads x 10 blocks; 8B prefill:
// 32 heads x 10) at the price of staging each K/V chunk for half as many queries.
template <int D, int NW = 4>
__global__ void __launch_bounds__(64 * NW) attn_fwd_kernel(AttnArgs a) {
  constexpr int NCH = D / 8;        // 16-byte chunks per row
  constexpr int KS = D / 32;        // MFMA k-steps over head dim (S^T)
  constexpr int NB = D / 16;        // 16-wide d blocks (O^T)
  constexpr int KC = 64;            // keys per chunk
  constexpr int IMG = KC * D * 2;   // bytes per K (or V) chunk image
  constexpr int RPI = 1024 / (D * 2);  // rows per 1 KiB DMA wave-instruction
  constexpr int NI = KC / RPI / NW; // DMA instructions per wave per image
  constexpr int QB = 16 * NW;       // queries per workgroup
  static_assert(NI >= 1, "K/V staging");
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * IMG];  // [buf][K,V]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  // XCD-aware tile order: the query blocks of one (batch, head) get consecutive
  // logical ids on the same XCD, so their K/V reads hit that XCD's L2 instead of
  // being re-fetched from HBM by up to 8 different dies.
  const int nqb = gridDim.x;
  const int lin = xcd_remap(blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z), nqb * gridDim.y * gridDim.z);
  // causal: a head's query blocks in decreasing work order (the last block sees every key), so
  // each XCD starts its longest blocks first and the short ones fill in behind them
  const int qblk = a.causal ? nqb - 1 - lin % nqb : lin % nqb;
  const int h = (lin / nqb) % gridDim.y, b = lin / (nqb * gridDim.y);
  const int hk = h / (a.H / a.Hkv);
  const int q0 = qblk * QB + wid * 16;
  const int kv_len = a.kv_len ? min(a.kv_len[b], a.Sk) : a.Sk;
  const int causal_off = a.Sk - a.Sq;

  const uint16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const uint16_t* kb = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hk * a.v_sh;

  // ---- Q^T fragments (B operand): query q0 + col, dims 32t + 8g .. +8
  bf16x8_t qf[KS];
  {
    const int qr = min(q0 + col, a.Sq - 1);
#pragma unroll
    for (int t = 0; t < KS; ++t) qf[t] = *(const bf16x8_t*)(qb + (int64_t)qr * a.q_ss + t * 32 + g * 8);
  }

  // ---- DMA staging: wave wid fills rows [wid*NI*RPI, +NI*RPI) of each image.
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  int srow[NI], kch[NI], vch[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = (wid * NI + i) * RPI + lane / NCH;
    const int pc = lane % NCH;               // physical chunk this lane lands in
    srow[i] = r;
    kch[i] = k_phys<D>(r, pc);               // XOR is an involution: logical = phys ^ f
    vch[i] = v_phys<D>(r, pc);
  }
  auto stage = [&](int chunk, int buf) {
    const int k0 = chunk * KC;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int kr = min(k0 + srow[i], a.Sk - 1);
      char* dk = smem + buf * 2 * IMG + (wid * NI + i) * 1024;
      __builtin_amdgcn_global_load_lds((g_ptr_t)(kb + (int64_t)kr * a.k_ss + kch[i] * 8), (lds_ptr_t)dk, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((g_ptr_t)(vb + (int64_t)kr * a.v_ss + vch[i] * 8), (lds_ptr_t)(dk + IMG), 16,
                                       0, 0);
    }
  };

  f32x4_t o[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) o[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float mrow = -INFINITY;               // running max (scaled, log2) of query q0 + col (replicated over g)
  f32x4_t l4 = (f32x4_t){0.f, 0.f, 0.f, 0.f};   // running row sum (all 4 entries equal)
  const int qi = q0 + col;

  int kend = kv_len;
  if (a.causal) kend = min(kend, min(qblk * QB + QB, a.Sq) + causal_off);
  const int nkc = (kend + KC - 1) / KC;

  // waves whose 16 queries are all past the end (the ragged last q-block, e.g.
  // 257 = 4*64 + 1) still stage K/V and join the barriers but skip all math.
  const bool active = q0 < a.Sq;
  // causal: last key any query of this wave may see
  const int wave_kend = a.causal ? min(kend, min(q0 + 16, a.Sq) + causal_off) : kend;

  if (nkc > 0) stage(0, 0);
  for (int kc = 0; kc < nkc; ++kc) {
    const int buf = kc & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                       // chunk kc landed; chunk kc-1 fully consumed
    if (kc + 1 < nkc) stage(kc + 1, buf ^ 1);
    const int k0 = kc * KC;
    if (!active || k0 >= wave_kend) continue;
    const char* sK = smem + buf * 2 * IMG;
    const char* sV = sK + IMG;
    // all 4 key blocks always run (rows past Sk hold clamped, finite copies and are
    // masked): branch-free chunks keep S/O in fixed VGPRs — skipping the dead blocks of
    // the ragged tail chunk made hipcc shuffle ~30 v_mov per chunk around the branches

    // S^T = K Q^T : 4 key blocks of 16; lane holds keys kb*16 + 4g + r, query col
    f32x4_t sc[4];
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16) {
      sc[kb16] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      const int kr = kb16 * 16 + col;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        bf16x8_t kf = *(const bf16x8_t*)(sK + kr * D * 2 + (k_phys<D>(kr, t * 4 + g) << 4));
        sc[kb16] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[t], sc[kb16], 0, 0, 0);
      }
    }
    // mask (only on chunks that need it) + online softmax (per lane = per query)
    const bool need_mask = (k0 + KC > kv_len) || (a.causal && k0 + KC - 1 > q0 + causal_off);
    softmax_chunk<NB, 2>(sc, o, l4, mrow, a, need_mask, k0, g, qi, kv_len, causal_off);

    // O^T += V^T P^T over two 32-key steps
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t pf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = (__bf16)sc[2 * s][r];
        pf[4 + r] = (__bf16)sc[2 * s + 1][r];
      }
      // tr-read rows (keys): s*32 + 4g + q  and  s*32 + 16 + 4g + q ; lane 4q+p
      const int q = col >> 2, p = col & 3;
      const int r0 = s * 32 + 4 * g + q, r1 = r0 + 16;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int c0 = j * 16 + 4 * p;           // column (d) of this lane's 8-byte piece
        const char* a0 = sV + r0 * D * 2 + (v_phys<D>(r0, c0 >> 3) << 4) + (c0 & 7) * 2;
        const char* a1 = sV + r1 * D * 2 + (v_phys<D>(r1, c0 >> 3) << 4) + (c0 & 7) * 2;
        const s16x4v lo = ds_read_tr16(a0);
        const s16x4v hi = ds_read_tr16(a1);
        s16x8_t vv = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vv), pf, o[j], 0, 0, 0);
      }
      l4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones_bf16x8(), pf, l4, 0, 0, 0);   // row sums of P
    }
  }

  // ---- normalise and store O[b, q, h, d]: lane holds d = 16j + 4g + r for query col
  const float inv = l4[0] > 0.f ? __builtin_amdgcn_rcpf(l4[0]) : 0.f;
  if (a.o != nullptr && qi < a.Sq) {
    uint16_t* orow = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qi * a.o_ss;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      uint2 w;
      w.x = pack2bf(o[j][0] * inv, o[j][1] * inv);
      w.y = pack2bf(o[j][2] * inv, o[j][3] * inv);
      *(uint2*)(orow + j * 16 + 4 * g) = w;
    }
  }
  if constexpr (D >= 64) {
    if (a.o8 != nullptr) {
      // MX block m (d = 32m .. 32m+31) = fragments j = 2m, 2m+1 of the 4 lanes {l, l^16, l^32, l^48}
      // holding this query: amax over the lane's 8 values, then over the lane quartet (whole wave
      // takes part in the shuffles; lanes of one query share validity)
      constexpr int NM = D / 32;
      float am[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        float x = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) x = fmaxf(x, fmaxf(fabsf(o[2 * m][r]), fabsf(o[2 * m + 1][r])));
        x *= inv;
        x = fmaxf(x, __shfl_xor(x, 16, 64));
        am[m] = fmaxf(x, __shfl_xor(x, 32, 64));
      }
      if (qi < a.Sq) {
        uint8_t* o8 = a.o8 + b * a.o8_sb + (int64_t)qi * a.o8_ss + h * D;
        uint32_t sbytes = 0;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const int e = mx_exp(am[m]);
          const float sc = inv * mx_inv(e);
          sbytes |= (uint32_t)(e + 127) << (8 * m);
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * m + jj;
            float t[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] = fminf(fmaxf(o[j][r] * sc, -448.f), 448.f);
            int w = __builtin_amdgcn_cvt_pk_fp8_f32(t[0], t[1], 0, false);
            w = __builtin_amdgcn_cvt_pk_fp8_f32(t[2], t[3], w, true);
            *(uint32_t*)(o8 + j * 16 + 4 * g) = (uint32_t)w;
          }
        }
        // scale planes [H*D/128][rows][4]: head h's NM bytes at plane h*D/128, sub-block (h*NM) % 4
        uint8_t* os = a.os + b * a.os_sb + (int64_t)((h * D) >> 7) * a.os_ss + (int64_t)qi * 4 + ((h * NM) & 3);
        if (g == 0) {
          if constexpr (NM == 4) *(uint32_t*)os = sbytes;
          else *(uint16_t*)os = (uint16_t)sbytes;
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// K/V-resident variant for short sequences with many (batch, head) pairs (ViT S = 197 / 257,
// CLIP text S = 77): one workgroup per (batch, head) DMA-loads the WHOLE K and V (<= 80 KiB,
// two workgroups per CU) once, then its 4 waves walk 16-query blocks (wave w: blocks w, w+4,
// ...) over the LDS-resident chunks with no further barriers.  Versus the streaming kernel
// this reads K/V from HBM once instead of once per 64-query block and removes the per-chunk
// wait/barrier pairs; the ragged 257th query costs one 16-query block of one wave instead
// of a whole 64-query workgroup.
// NW waves per workgroup (4 or 8): with two K/V-resident workgroups per CU, 8 waves give 4 per
// SIMD to hide the LDS / MFMA latencies of the query-block walk (ViT S = 257: 17 blocks -> at most
// 3 per wave instead of 5).
template <int D, int NW>
__global__ void __launch_bounds__(64 * NW) attn_res_kernel(AttnArgs a, int nkc, int clean_split) {
  constexpr int NCH = D / 8;
  constexpr int KS = D / 32;
  constexpr int NB = D / 16;
  constexpr int KC = 64;
  constexpr int IMG = KC * D * 2;
  constexpr int RPI = 1024 / (D * 2);
  constexpr int NI = KC / RPI / NW;
  static_assert(NI >= 1, "K/V staging: at least one 1 KiB DMA piece per wave per chunk");
  extern __shared__ __attribute__((aligned(16))) char smem[];   // [nkc][K, V][IMG]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int lin = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int h = lin % a.H, b = lin / a.H;
  const int hk = h / (a.H / a.Hkv);
  const int kv_len = a.kv_len ? min(a.kv_len[b], a.Sk) : a.Sk;
  const int causal_off = a.Sk - a.Sq;
  const uint16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const uint16_t* kb = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hk * a.v_sh;
  const __amdgpu_buffer_rsrc_t o_rs = __builtin_amdgcn_make_buffer_rsrc(
      a.o + b * a.o_sb + h * a.o_sh, (short)0, (int)(((int64_t)(a.Sq - 1) * a.o_ss + D) * 2), 0x00020000);

  const int nq16 = (a.Sq + 15) / 16;
  // Q fragments are register-prefetched one query block ahead so their HBM latency
  // hides under the current block's chunks instead of stalling every block start.
  bf16x8_t qn[KS];
  auto load_q = [&](int blk) {
    const int qr = min(blk * 16 + col, a.Sq - 1);
#pragma unroll
    for (int t = 0; t < KS; ++t) qn[t] = *(const bf16x8_t*)(qb + (int64_t)qr * a.q_ss + t * 32 + g * 8);
  };
  load_q(wid);
  // ---- stage all K/V chunks (clamped rows past Sk keep the images finite)
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef const __attribute__((address_space(1))) void* g_ptr_t;
  for (int c = 0; c < nkc; ++c) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = (wid * NI + i) * RPI + lane / NCH;
      const int pc = lane % NCH;
      const int kr = min(c * KC + r, a.Sk - 1);
      char* dk = smem + c * 2 * IMG + (wid * NI + i) * 1024;
      __builtin_amdgcn_global_load_lds((g_ptr_t)(kb + (int64_t)kr * a.k_ss + k_phys<D>(r, pc) * 8), (lds_ptr_t)dk, 16,
                                       0, 0);
      __builtin_amdgcn_global_load_lds((g_ptr_t)(vb + (int64_t)kr * a.v_ss + v_phys<D>(r, pc) * 8),
                                       (lds_ptr_t)(dk + IMG), 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Per-lane byte offsets inside one chunk's K / V image (chunk independent: K rows kb16 * 16 + col
  // and V rows 32 s + 4 g + (col >> 2) (+ 16) differ from the kb16 = s = 0 rows by multiples of 16,
  // which leave the XOR swizzles unchanged), so every LDS address in the chunk loop is the chunk
  // base plus one of these plus an immediate.
  // the dynamic-LDS base as an opaque SGPR: with the symbol itself hipcc keeps one running pointer
  // per lane offset and re-adds the (zero) symbol to each in every chunk (12 VALU per chunk)
  int lds0 = (int)(size_t)(const lds_char*)smem;
  asm volatile("" : "+s"(lds0));
  int kofs[KS], vofs[NB];
#pragma unroll
  for (int t = 0; t < KS; ++t) kofs[t] = col * D * 2 + (k_phys<D>(col, t * 4 + g) << 4);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int r0 = 4 * g + (col >> 2), c0 = j * 16 + 4 * (col & 3);
    vofs[j] = r0 * D * 2 + (v_phys<D>(r0, c0 >> 3) << 4) + (c0 & 7) * 2;
  }
  // One 64-key chunk of S^T, online softmax, O^T += V^T P^T for the 16 queries of block q0 (qf).
  auto full_chunk = [&](auto maskc, int kc, const bf16x8_t (&qf)[KS], f32x4_t (&o)[NB], f32x4_t& l4, float& mrow,
                        int q0, int qi) __attribute__((always_inline)) {
    const int k0 = kc * KC;
    const int cb = lds0 + kc * 2 * IMG;   // wave-uniform chunk base (SGPR) + the hoisted lane offsets
    const lds_char* sK = (const lds_char*)(size_t)cb;
    const lds_char* sV = sK + IMG;
    f32x4_t sc[4];
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16) {
      sc[kb16] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        // row kb16 * 16 + col: the swizzle term of k_phys repeats every 16 rows
        bf16x8_t kf = *(const __attribute__((address_space(3))) bf16x8_t*)(sK + kofs[t] + kb16 * 16 * D * 2);
        sc[kb16] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[t], sc[kb16], 0, 0, 0);
      }
    }
    softmax_chunk<NB, decltype(maskc)::value ? 1 : 0>(sc, o, l4, mrow, a, true, k0, g, qi, kv_len, causal_off);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t pf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = (__bf16)sc[2 * s][r];
        pf[4 + r] = (__bf16)sc[2 * s + 1][r];
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        // rows r0 = 32 s + 4 g + (col >> 2) and r0 + 16: the swizzle term of v_phys repeats every 8 rows
        const s16x4v lo = ds_read_tr16(sV + vofs[j] + s * 32 * D * 2);
        const s16x4v hi = ds_read_tr16(sV + vofs[j] + (s * 32 + 16) * D * 2);
        s16x8_t vv = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vv), pf, o[j], 0, 0, 0);
      }
      l4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones_bf16x8(), pf, l4, 0, 0, 0);   // row sums of P
    }
  };
  // a ragged last chunk with <= 16 live keys (ViT S = 257: 1 key; CLIP text S = 77: 13): a 16-key
  // step, 7 MFMAs and 4 scores per lane instead of 18 and 16
  auto tail_chunk = [&](int kc, const bf16x8_t (&qf)[KS], f32x4_t (&o)[NB], f32x4_t& l4, float& mrow,
                        int qi) __attribute__((always_inline)) {
    const int k0 = kc * KC;
    const char* sK = smem + kc * 2 * IMG;
    const char* sV = sK + IMG;
    f32x4_t s0 = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      bf16x8_t kf = *(const bf16x8_t*)(sK + col * D * 2 + (k_phys<D>(col, t * 4 + g) << 4));
      s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[t], s0, 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kj = k0 + g * 4 + r;
      bool ok = kj < kv_len;
      if (a.causal) ok = ok && (kj <= qi + causal_off);
      s0[r] = ok ? s0[r] : -INFINITY;
      mx = fmaxf(mx, s0[r]);
    }
    mx = group4_max(mx);
    const float mcand = fmaxf(mrow, mx * a.scale_log2);
    if (__any(mcand > mrow + 8.f)) {
      const float mb = mcand == -INFINITY ? 0.f : mcand;
      const float alpha = __builtin_amdgcn_exp2f(mrow - mb);
#pragma unroll
      for (int j = 0; j < NB; ++j) o[j] *= alpha;
      l4 *= alpha;
      mrow = mcand;
    }
    const float nmb = mrow == -INFINITY ? 0.f : -mrow;
    bf16x8_t pf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pf[r] = (__bf16)__builtin_amdgcn_exp2f(__builtin_fmaf(s0[r], a.scale_log2, nmb));
      pf[4 + r] = (__bf16)0.f;                  // keys 16..31 of the chunk: past the tail
    }
    const int q = col >> 2, p = col & 3;
    const int r0 = 4 * g + q, r1 = r0 + 16;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int c0 = j * 16 + 4 * p;
      const char* a0 = sV + r0 * D * 2 + (v_phys<D>(r0, c0 >> 3) << 4) + (c0 & 7) * 2;
      const char* a1 = sV + r1 * D * 2 + (v_phys<D>(r1, c0 >> 3) << 4) + (c0 & 7) * 2;
      const s16x4v lo = ds_read_tr16(a0);
      const s16x4v hi = ds_read_tr16(a1);
      s16x8_t vv = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vv), pf, o[j], 0, 0, 0);
    }
    l4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones_bf16x8(), pf, l4, 0, 0, 0);
  };
  // Branch-free store through a per-(batch, head) buffer descriptor whose range ends at the last valid
  // query row: lanes of the ragged last block (qi >= Sq) are dropped by the range check.  A divergent
  // `if (qi < Sq)` store made hipcc merge its vmcnt bookkeeping conservatively and wait vmcnt(0) for the
  // prefetched Q at every block.
  auto store_o = [&](const f32x4_t (&o)[NB], float lsum, int qi) __attribute__((always_inline)) {
    const float inv = lsum > 0.f ? __builtin_amdgcn_rcpf(lsum) : 0.f;
    const int row_off = qi * (int)a.o_ss * 2;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
      const u32x2v w = {pack2bf(o[j][0] * inv, o[j][1] * inv), pack2bf(o[j][2] * inv, o[j][3] * inv)};
      __builtin_amdgcn_raw_buffer_store_b64(w, o_rs, row_off + (j * 16 + 4 * g) * 2, 0, 0);
    }
  };

  for (int qbk = wid; qbk < nq16; qbk += NW) {
    const int q0 = qbk * 16;
    const int qi = q0 + col;
    bf16x8_t qf[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) qf[t] = qn[t];
    if (qbk + NW < nq16) load_q(qbk + NW);
    f32x4_t o[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) o[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    float mrow = -INFINITY;
    f32x4_t l4 = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int wave_kend = a.causal ? min(kv_len, min(q0 + 16, a.Sq) + causal_off) : kv_len;
    const int nc = min(nkc, (wave_kend + KC - 1) / KC);
    const bool tail1 = nc > 0 && wave_kend - (nc - 1) * KC <= 16;
    const int nfull = tail1 ? nc - 1 : nc;
    // chunks needing no mask come first (key-length and causal masks grow with the chunk index):
    // an unmasked loop, then the masked remainder
    int nclean = clean_split ? nfull : 0;   // (0: every chunk takes the masked form -- the A/B arm)
    while (nclean > 0 && ((nclean * KC > kv_len) || (a.causal && nclean * KC - 1 > q0 + causal_off))) --nclean;
    for (int kc = 0; kc < nclean; ++kc) full_chunk(std::false_type{}, kc, qf, o, l4, mrow, q0, qi);
    for (int kc = nclean; kc < nfull; ++kc) full_chunk(std::true_type{}, kc, qf, o, l4, mrow, q0, qi);
    if (tail1) tail_chunk(nfull, qf, o, l4, mrow, qi);
    store_o(o, l4[0], qi);
  }
}

template <int D, int NW>
static hipError_t launch_res_nw(const AttnArgs& a, int B, int nkc, hipStream_t stream) {
  const size_t lds = (size_t)nkc * 2 * 64 * D * 2;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)attn_res_kernel<D, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((attn_res_kernel<D, NW>), dim3(a.H, B), dim3(64 * NW), lds, stream, a, nkc,
                     tuning(TUNE_ATTN_CLEAN_CHUNKS));
  return hipGetLastError();
}

template <int D>
static hipError_t launch_res(const AttnArgs& a, int B, int nkc, hipStream_t stream) {
  // 8 waves per workgroup once there are >= 10 query blocks to share (ViT-L/14 S = 257:
  // 0.416 -> 0.357 ms at b512, profiles/r2_attn_res_waves_v1.txt), 4 for short sequences
  // (CLIP text S = 77 has 5 blocks: extra waves would idle)
  const int nw = (a.Sq + 15) / 16 >= 10 ? 8 : 4;
  if constexpr (D >= 64) {
    if (nw == 8) return launch_res_nw<D, 8>(a, B, nkc, stream);
  }
  return launch_res_nw<D, 4>(a, B, nkc, stream);
}

hipError_t attn_fwd(const AttnArgs& a, int B, int D, hipStream_t stream) {
  // K/V-resident path when the whole K/V fits in 80 KiB and there are enough (batch, head) pairs
  const int nkc = (a.Sk + 63) / 64;
  if (a.o8 != nullptr && D < 64) return hipErrorInvalidValue;
  if (a.o == nullptr && a.o8 == nullptr) return hipErrorInvalidValue;
  const bool res_ok = a.o8 == nullptr && (int64_t)B * a.H >= 1024 && (size_t)nkc * 2 * 64 * D * 2 <= 80 * 1024 &&
                      a.Sq <= 1024;
  if (res_ok) {
    if (D == 64) return launch_res<64>(a, B, nkc, stream);
    if (D == 128) return launch_res<128>(a, B, nkc, stream);
    if (D == 32) return launch_res<32>(a, B, nkc, stream);
  }
  // streaming path: 64-query blocks, 4 waves (32-query / 2-wave blocks measured slower on the
  // few-(batch, head) prefills they were meant for, r2)
  dim3 grid((a.Sq + 63) / 64, a.H, B), block(256);
  if (D == 64) hipLaunchKernelGGL((attn_fwd_kernel<64, 4>), grid, block, 0, stream, a);
  else if (D == 128) hipLaunchKernelGGL((attn_fwd_kernel<128, 4>), grid, block, 0, stream, a);
  else if (D == 32) hipLaunchKernelGGL((attn_fwd_kernel<32, 4>), grid, block, 0, stream, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace lumen
