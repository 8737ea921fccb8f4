// Decoder-LLM kernels for the VLM (Qwen2 / Llama family):
//
//  * rope_kv: rotary embedding (rotate-half, HF convention) applied in place to
//    the q and k heads of the packed QKV projection, fused with the paged KV
//    cache write (k token-major, v transposed; layouts in llm.h).  Prefill
//    attention then reads q/k/v straight from the rotated QKV buffer.
//  * paged_decode: flash-decoding over the paged cache.  One workgroup per
//    (split, kv-head, sequence); the G = H / Hkv query heads sharing a kv head
//    are the 16 MFMA columns, each wave walks its own 64-token blocks with an
//    online softmax, the 4 wave states are merged through LDS and — when the
//    context is split across workgroups — the last split to finish merges them
//    (in-launch, ticket counter; no combine kernel).
//    Both MFMA operands come straight from HBM: S^T = K Q^T reads K rows in a
//    permuted token order chosen so that each lane's 8 P values are 8
//    consecutive tokens, which the transposed V cache serves with one 16-byte
//    load per MFMA (O^T = V^T P^T).
//  * rep_penalty: repetition penalty on the logits of previously generated
//    tokens (the reference accepts and ignores it, SURVEY V-7).
#include "common.h"
#include "llm.h"

namespace lumen {

// ------------------------------------------------------------------------------ RoPE + KV write
// grid (T, nrot_blocks + v_blocks): one (token, 256-element chunk) per workgroup and ONE
// rotation pair / V element per thread, so a decode step (T = 1..16) spreads over 14+
// workgroups per token instead of looping 10x inside one (each pass of that loop paid a
// dependent global round trip: 8 us per layer per token, measured)
__global__ void __launch_bounds__(256) rope_kv_kernel(RopeKVArgs a, int nrot_blocks) {
  const int t = blockIdx.x;
  const int half = a.D >> 1;
  uint16_t* row = a.qkv + (int64_t)t * a.ld;
  const int64_t slot = a.slots ? a.slots[t] : -1;
  const int64_t blk = slot >= 0 ? (slot >> 6) : 0;
  const int off = (int)(slot & 63);
  if ((int)blockIdx.y < nrot_blocks) {
    const int idx = blockIdx.y * 256 + threadIdx.x;
    if (idx >= (a.H + a.Hkv) * half) return;
    const int p = a.pos[t];
    const float2* cs = reinterpret_cast<const float2*>(a.cos_sin) + (int64_t)p * half;
    const int hh = idx / half, i = idx - hh * half;
    uint16_t* hp = row + hh * a.D;
    const float x1 = bf2f(hp[i]), x2 = bf2f(hp[i + half]);
    const float2 c = cs[i];
    const float y1 = x1 * c.x - x2 * c.y, y2 = x2 * c.x + x1 * c.y;
    const uint16_t b1 = f2bf(y1), b2 = f2bf(y2);
    hp[i] = b1;
    hp[i + half] = b2;
    if (hh >= a.H && slot >= 0) {
      const int64_t ko = ((blk * a.Hkv + (hh - a.H)) * KV_BLOCK + off) * a.D;
      if (a.kv_fp8) {
        uint8_t* kr = reinterpret_cast<uint8_t*>(a.k_cache) + ko;
        kr[i] = f2fp8(bf2f(b1));
        kr[i + half] = f2fp8(bf2f(b2));
      } else {
        uint16_t* kr = a.k_cache + ko;
        kr[i] = b1;
        kr[i + half] = b2;
      }
    }
    return;
  }
  if (slot < 0) return;
  const int idx = (blockIdx.y - nrot_blocks) * 256 + threadIdx.x;
  if (idx >= a.Hkv * a.D) return;
  const uint16_t* vr = row + (a.H + a.Hkv) * a.D;
  const int kh = idx / a.D, d = idx - kh * a.D;
  const int64_t vo = ((blk * a.Hkv + kh) * a.D + d) * KV_BLOCK + off;
  if (a.kv_fp8) reinterpret_cast<uint8_t*>(a.v_cache)[vo] = f2fp8(bf2f(vr[idx]));
  else a.v_cache[vo] = vr[idx];
}

// Prefill form (T >= 64): one workgroup per (64-token tile, head) with 16-byte accesses.  q / k
// heads: each thread rotates D/8 pairs of one token (4 threads per token) in place and writes the
// k cache rows; v heads: the [64 x D] tile goes through LDS and leaves d-major, 8 tokens (16 or
// 8 bytes) per store when their slots are consecutive in one block.  The per-element kernel above
// wrote V with 2-byte stores 128 bytes apart (11 us per 8B-prefill layer at 624 tokens).
template <int D>
__global__ void __launch_bounds__(256) rope_kv_tile_kernel(RopeKVArgs a) {
  constexpr int HALF = D / 2, PPT = D / 8;       // rotation pairs per thread
  __shared__ __attribute__((aligned(16))) uint16_t vt[64][D + 8];
  __shared__ int64_t sl[64];
  const int t0 = blockIdx.x * 64, hh = blockIdx.y, tid = threadIdx.x;
  if (hh < a.H + a.Hkv) {
    const int tt = tid >> 2, c0 = (tid & 3) * PPT, t = t0 + tt;
    if (t >= a.T) return;
    uint16_t* hp = a.qkv + (int64_t)t * a.ld + hh * D;
    const float2* cs = reinterpret_cast<const float2*>(a.cos_sin) + (int64_t)a.pos[t] * HALF + c0;
    float y1[PPT], y2[PPT];
#pragma unroll
    for (int u = 0; u < PPT; u += 8) {
      float x1[8], x2[8];
      unpack8(*(const u32x4_t*)(hp + c0 + u), x1);
      unpack8(*(const u32x4_t*)(hp + HALF + c0 + u), x2);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float2 c = cs[u + q];
        y1[u + q] = x1[q] * c.x - x2[q] * c.y;
        y2[u + q] = x2[q] * c.x + x1[q] * c.y;
      }
      *(u32x4_t*)(hp + c0 + u) = pack8(y1 + u);
      *(u32x4_t*)(hp + HALF + c0 + u) = pack8(y2 + u);
    }
    const int64_t slot = a.slots && hh >= a.H ? a.slots[t] : -1;
    if (slot >= 0) {
      const int64_t ko = (((slot >> 6) * a.Hkv + (hh - a.H)) * KV_BLOCK + (slot & 63)) * D;
#pragma unroll
      for (int u = 0; u < PPT; u += 8) {
        float r1[8], r2[8];   // the stored (bf16-rounded) values, as the per-element kernel caches them
        unpack8(pack8(y1 + u), r1);
        unpack8(pack8(y2 + u), r2);
        if (a.kv_fp8) {
          uint8_t* kr = reinterpret_cast<uint8_t*>(a.k_cache) + ko;
          *(uint2*)(kr + c0 + u) = fp8x8_scaled(r1, 1.f);
          *(uint2*)(kr + HALF + c0 + u) = fp8x8_scaled(r2, 1.f);
        } else {
          *(u32x4_t*)(a.k_cache + ko + c0 + u) = pack8(r1);
          *(u32x4_t*)(a.k_cache + ko + HALF + c0 + u) = pack8(r2);
        }
      }
    }
    return;
  }
  if (a.slots == nullptr) return;
  const int kh = hh - a.H - a.Hkv;
  if (tid < 64) sl[tid] = t0 + tid < a.T ? a.slots[t0 + tid] : -1;
  constexpr int CPR = D / 8;                       // 16-byte chunks per token row
  for (int c = tid; c < 64 * CPR; c += 256) {
    const int tt = c / CPR, ch = c % CPR;
    if (t0 + tt < a.T)
      *(u32x4_t*)&vt[tt][ch * 8] = *(const u32x4_t*)(a.qkv + (int64_t)(t0 + tt) * a.ld + (a.H + a.Hkv + kh) * D + ch * 8);
  }
  __syncthreads();
  // thread -> (d, run of 8 tokens)
  for (int w = tid; w < D * 8; w += 256) {
    const int d = w % D, g8 = w / D;
    const int64_t s0 = sl[g8 * 8];
    bool run = s0 >= 0 && (s0 & 7) == 0;
#pragma unroll
    for (int q = 1; q < 8; ++q) run = run && sl[g8 * 8 + q] == s0 + q;
    if (run) {
      const int64_t vo = (((s0 >> 6) * a.Hkv + kh) * D + d) * KV_BLOCK + (s0 & 63);
      float f[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = bf2f(vt[g8 * 8 + q][d]);
      if (a.kv_fp8) *(uint2*)(reinterpret_cast<uint8_t*>(a.v_cache) + vo) = fp8x8_scaled(f, 1.f);
      else *(u32x4_t*)(a.v_cache + vo) = pack8(f);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t s = sl[g8 * 8 + q];
        if (s < 0) continue;
        const int64_t vo = (((s >> 6) * a.Hkv + kh) * D + d) * KV_BLOCK + (s & 63);
        if (a.kv_fp8) reinterpret_cast<uint8_t*>(a.v_cache)[vo] = f2fp8(bf2f(vt[g8 * 8 + q][d]));
        else a.v_cache[vo] = vt[g8 * 8 + q][d];
      }
    }
  }
}

hipError_t rope_kv(const RopeKVArgs& a, hipStream_t stream) {
  if (a.T == 0) return hipSuccess;
  if (a.T >= 64 && (a.D == 64 || a.D == 128) && a.ld % 8 == 0) {
    const dim3 grid((a.T + 63) / 64, a.H + 2 * a.Hkv);
    if (a.D == 128) hipLaunchKernelGGL(rope_kv_tile_kernel<128>, grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL(rope_kv_tile_kernel<64>, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
  }
  const int nrot_blocks = ((a.H + a.Hkv) * (a.D / 2) + 255) / 256;
  const int v_blocks = a.slots ? (a.Hkv * a.D + 255) / 256 : 0;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(a.T, nrot_blocks + v_blocks), dim3(256), 0, stream, a, nrot_blocks);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ paged decode attention
// One workgroup of NW = 4 waves per (split, kv head, sequence); wave w takes the split's 64-token
// blocks w, w + 4, ... (up to 32 splits of 4 blocks -- 8k tokens -- one block per wave, so a
// context of <= 256 tokens is ONE workgroup per kv head; longer contexts loop with an online
// softmax).  The latency chain per wave is: block-table entry -> every K and V fragment of the
// block in flight at once -> S^T = K Q^T, online softmax, O^T += V^T P^T; the 8 wave states
// merge through LDS.  Fused RoPE mode (decode): q and the current token's k are rotated in
// registers, and the current token enters the wave that owns its block straight from registers
// (its score q . k_cur as a lane-group dot product, its v into the V fragment) -- the cache
// write of that token is fire-and-forget (the next step reads it), so no workgroup waits for a
// store round trip.  A context split over several workgroups is
// combined IN the launch: every split publishes its (m, l, o) partials with write-through (sc1)
// stores, draws a ticket from the (sequence, kv head) counter, and the last to arrive merges
// all splits (sc1 loads, 8 in flight) -- no combine launch, no fences (MI355X_MICROARCH.md
// hand-off rules); the last arriver re-zeroes the counter for the next launch.
// 4 waves = 1 per SIMD: the 512-VGPR budget holds a whole block's K and V fragments.  The launch
// fixes the number of splits (grid.x); blocks per split = max(a.blocks_per_split, ceil(blocks /
// grid.x)) is derived from each sequence's own ctx_len on the device, so a graph captured for the
// longest context spreads every shorter one over all its splits as well.  (One-wave workgroups with
// one block each measured 2x slower: their single-wave split combine is latency-serial,
// profiles/r3_decode_attn_splits_v1.txt.)
constexpr int PD_NW = 4;

// Prefetch workgroups (blockIdx.z >= B): stream a.pf[] once through the memory-side cache.
__device__ __forceinline__ void pd_prefetch(const DecodeArgs& a, int wg, int nwg) {
  uint32_t x = 0;
#pragma unroll 1
  for (int r = 0; r < 2; ++r) {
    if (a.pf[r] == nullptr || a.pf_bytes[r] <= 0) continue;
    const int64_t n16 = a.pf_bytes[r] >> 4;                     // whole 16-byte chunks
    const int64_t per = (n16 + nwg - 1) / nwg;
    const int64_t c0 = (int64_t)wg * per, c1 = min(n16, c0 + per);
    const u32x4_t* p = reinterpret_cast<const u32x4_t*>(a.pf[r]);
    int64_t c = c0 + threadIdx.x;
    for (; c + 7 * (int64_t)blockDim.x < c1; c += 8 * (int64_t)blockDim.x) {   // 8 loads in flight per lane
      u32x4_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[c + u * (int64_t)blockDim.x];
#pragma unroll
      for (int u = 0; u < 8; ++u) x ^= v[u][0] ^ v[u][3];
    }
    for (; c < c1; c += blockDim.x) x ^= p[c][0];
  }
  if (x == 0x9e3779b9u && a.pf_bytes[0] < 0) a.o[threadIdx.x] = 0;   // never true: keeps the loads
}

template <int D>
__device__ __forceinline__ void rope_chunks(u32x4_t (&w)[D / 32], const float2* cs, int g) {
  constexpr int KS = D / 32;
#pragma unroll
  for (int t = 0; t < KS / 2; ++t) {   // element e pairs with e + D/2: chunk t with t + KS/2
    float x1[8], x2[8];
    unpack8(w[t], x1);
    unpack8(w[t + KS / 2], x2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 c = cs[t * 32 + g * 8 + j];
      const float y1 = x1[j] * c.x - x2[j] * c.y, y2 = x2[j] * c.x + x1[j] * c.y;
      x1[j] = y1;
      x2[j] = y2;
    }
    w[t] = pack8(x1);
    w[t + KS / 2] = pack8(x2);
  }
}

// bf16 values as the cache stores them (fp8 cache: rounded through e4m3fn)
template <bool F8KV>
__device__ __forceinline__ __bf16 as_cached(__bf16 v) {
  if constexpr (F8KV) {
    const uint32_t b = f2fp8((float)v);
    return __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(b, 0u))[0];
  } else {
    return v;
  }
}

template <int D, bool F8KV>
__global__ void __launch_bounds__(64 * PD_NW) paged_decode_kernel(DecodeArgs a, int B) {
  constexpr int NW = PD_NW;
  if ((int)blockIdx.z >= B) {   // MALL prefetch workgroups
    pd_prefetch(a, ((blockIdx.z - B) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x,
                (gridDim.z - B) * gridDim.y * gridDim.x);
    return;
  }
  const int64_t t_start = a.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  constexpr int KS = D / 32;   // k-steps of S^T over the head dim
  constexpr int NB = D / 16;   // 16-wide d blocks of O^T
  __shared__ float sm_ml[NW][2][16];
  __shared__ float sm_o[NW][D][17];
  __shared__ int sm_last;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int G = a.H / a.Hkv;
  const int ctx = a.ctx_len[b];
  const int nblk = (ctx + KV_BLOCK - 1) / KV_BLOCK;
  const int bps = max(a.blocks_per_split, (nblk + (int)gridDim.x - 1) / (int)gridDim.x);
  const int blk0 = split * bps;
  const int blk1 = min(blk0 + bps, nblk);
  const int ns = max(1, (nblk + bps - 1) / bps);   // splits holding blocks
  if (split >= ns) return;
  // this wave's blocks: blk0 + wid, + NW, ... (one block per wave up to 512 tokens per split)
  int phys = blk0 + wid < blk1 ? a.block_table[(int64_t)b * a.bt_stride + blk0 + wid] : 0;   // first load of the chain

  // Q^T fragment (B operand): column = query head hk*G + col (zero beyond G).  Loaded here, rotated
  // (fused RoPE) only after the first block's K / V loads are in flight: its VALU then overlaps
  // that round trip instead of delaying the issue.
  bf16x8_t qf[KS];
  const bool fused = a.pos != nullptr;
  const float2* cs = fused ? reinterpret_cast<const float2*>(a.cos_sin) + (int64_t)a.pos[b] * (D / 2) : nullptr;
  const bool qv = col < G;
  u32x4_t qraw[KS];
  {
    const uint16_t* qp = a.q + (int64_t)b * a.q_sb + (int64_t)(hk * G + (qv ? col : 0)) * D;
#pragma unroll
    for (int t = 0; t < KS; ++t) qraw[t] = *(const u32x4_t*)(qp + t * 32 + g * 8);
  }
  bool q_ready = false;
  auto prep_q = [&]() {
#pragma unroll
    for (int t = 0; t < KS; ++t)
      if (!qv) qraw[t] = (u32x4_t){0u, 0u, 0u, 0u};
    if constexpr (KS >= 2) {
      if (fused) rope_chunks<D>(qraw, cs, g);
    }
#pragma unroll
    for (int t = 0; t < KS; ++t) qf[t] = __builtin_bit_cast(bf16x8_t, qraw[t]);
    q_ready = true;
  };
  // current token (position ctx - 1) in fused mode: the wave owning its block takes it from
  // registers; the owning split's workgroup also writes it to the cache AFTER its attention
  // (fire-and-forget: only the next decode step reads it)
  const int cur = ctx - 1;
  const bool owns_cur = fused && blk0 <= cur / KV_BLOCK && cur / KV_BLOCK < blk1;
  // the current token's k (rotated) and v as this lane's fragments need them, loaded BEFORE the
  // K / V stream (vmcnt retires in issue order; a load issued after it would wait behind it)
  u32x4_t kcur[KS];
  uint16_t vcur[NB];
  if (owns_cur) {
    const uint16_t* kp = a.q + (int64_t)b * a.q_sb + (int64_t)(a.H + hk) * D;
    const uint16_t* vp = a.q + (int64_t)b * a.q_sb + (int64_t)(a.H + a.Hkv + hk) * D;
#pragma unroll
    for (int t = 0; t < KS; ++t) kcur[t] = *(const u32x4_t*)(kp + t * 32 + g * 8);
#pragma unroll
    for (int j = 0; j < NB; ++j) vcur[j] = vp[j * 16 + col];
  }

  f32x4_t o[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) o[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float mrow = -INFINITY, lrow = 0.f;

  for (int bi = blk0 + wid; bi < blk1; bi += NW) {
    if (bi != blk0 + wid) phys = a.block_table[(int64_t)b * a.bt_stride + bi];
    const int64_t kvo = ((int64_t)phys * a.Hkv + hk) * KV_BLOCK * D;   // elements (= bytes for fp8)
    const uint16_t* kb = a.k_cache + kvo;
    const uint16_t* vb = a.v_cache + kvo;
    const uint8_t* kb8 = reinterpret_cast<const uint8_t*>(a.k_cache) + kvo;
    const uint8_t* vb8 = reinterpret_cast<const uint8_t*>(a.v_cache) + kvo;
    const int valid = min(KV_BLOCK, ctx - bi * KV_BLOCK);

    // ---- every K and V fragment of the block in flight at once
    // S^T tiles: tile kb16 = (s = kb16 >> 1, hf = kb16 & 1); MFMA row i <-> token
    // 32s + 8(i >> 2) + 4hf + (i & 3), so C row 4g + r holds token 32s + 8g + 4hf + r.
    bf16x8_t kf[4][KS];
    bf16x8_t vf[2][NB];
    const int64_t vro = (int64_t)col * KV_BLOCK + 8 * g;
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16) {
      const int tok = 32 * (kb16 >> 1) + 8 * (col >> 2) + 4 * (kb16 & 1) + (col & 3);
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        if constexpr (F8KV) {
          const uint2 w = *(const uint2*)(kb8 + (int64_t)tok * D + g * 8 + t * 32);
          kf[kb16][t] = __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(w.x, w.y));
        } else {
          kf[kb16][t] = *(const bf16x8_t*)(kb + (int64_t)tok * D + g * 8 + t * 32);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if constexpr (F8KV) {
          const uint2 w = *(const uint2*)(vb8 + vro + 32 * s + (int64_t)j * 16 * KV_BLOCK);
          vf[s][j] = __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(w.x, w.y));
        } else {
          vf[s][j] = *(const bf16x8_t*)(vb + vro + 32 * s + (int64_t)j * 16 * KV_BLOCK);
        }
      }
    // the current token's v from registers (the cache store above may not have landed)
    const bool cur_here = owns_cur && bi == cur / KV_BLOCK;
    const int coff = cur - bi * KV_BLOCK;
    if (cur_here) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int e = coff - 32 * s - 8 * g;   // lane-dependent: a select per element, no branch
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const __bf16 v = as_cached<F8KV>(__builtin_bit_cast(__bf16, vcur[j]));
#pragma unroll
          for (int ee = 0; ee < 8; ++ee) vf[s][j][ee] = ee == e ? v : vf[s][j][ee];
        }
      }
    }

    if (!q_ready) prep_q();
    f32x4_t sc[4];
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16) {
      sc[kb16] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KS; ++t) sc[kb16] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kb16][t], qf[t], sc[kb16], 0, 0, 0);
    }
    if (cur_here) {   // the current token's score q . k_cur from registers (rotated, rounded as cached)
      u32x4_t kw[KS];
#pragma unroll
      for (int t = 0; t < KS; ++t) kw[t] = kcur[t];
      if constexpr (KS >= 2) rope_chunks<D>(kw, cs, g);
      float dot = 0.f;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        const bf16x8_t kv8 = __builtin_bit_cast(bf16x8_t, kw[t]);
#pragma unroll
        for (int e = 0; e < 8; ++e) dot += (float)as_cached<F8KV>(kv8[e]) * (float)qf[t][e];
      }
      dot += __shfl_xor(dot, 16, 64);   // sum over the 4 lane groups (d ranges) of query col
      dot += __shfl_xor(dot, 32, 64);
#pragma unroll
      for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (32 * (kb16 >> 1) + 8 * g + 4 * (kb16 & 1) + r == coff) sc[kb16][r] = dot;
    }
    float mx = mrow;
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = 32 * (kb16 >> 1) + 8 * g + 4 * (kb16 & 1) + r;
        const float sv = tok < valid ? sc[kb16][r] * a.scale_log2 : -INFINITY;
        sc[kb16][r] = sv;
        mx = fmaxf(mx, sv);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mbase = mx == -INFINITY ? 0.f : mx;
    const float alpha = __builtin_amdgcn_exp2f(mrow - mbase);   // online softmax over a wave's blocks
    float rs = 0.f;
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(sc[kb16][r] - mbase);
        sc[kb16][r] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    lrow = lrow * alpha + rs;
    mrow = mx;
#pragma unroll
    for (int j = 0; j < NB; ++j) o[j] *= alpha;

    // a partial block: V columns past the context may hold any finite stale value (p = 0 there),
    // but zero them anyway so that a never-written slot cannot inject a NaN through 0 * NaN
    if (valid < KV_BLOCK) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (32 * s + 8 * g + e >= valid) {
#pragma unroll
            for (int j = 0; j < NB; ++j) vf[s][j][e] = (__bf16)0.f;
          }
    }
    // O^T += V^T P^T over two 32-token steps; lane's P k-slots 8g + j = tokens 32s + 8g + j
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t pf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = (__bf16)sc[2 * s][r];
        pf[4 + r] = (__bf16)sc[2 * s + 1][r];
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[s][j], pf, o[j], 0, 0, 0);
    }
  }

  if (owns_cur) {   // the current token's k (rotated) / v into the cache for the next step
    const int64_t slot = a.slots[b];
    if (slot >= 0) {
      const int64_t cblk = slot >> 6;
      const int coff = (int)(slot & 63);
      const uint16_t* kv = a.q + (int64_t)b * a.q_sb + (int64_t)(a.H + hk) * D;   // unrotated k head
      const int half = D / 2;
      for (int i = tid; i < half + D; i += 64 * NW) {   // k rotation pairs, then v elements
      if (i < half) {
        const float2 c = reinterpret_cast<const float2*>(a.cos_sin)[(int64_t)a.pos[b] * half + i];
        const float x1 = bf2f(kv[i]), x2 = bf2f(kv[i + half]);
        const uint16_t y1 = f2bf(x1 * c.x - x2 * c.y), y2 = f2bf(x2 * c.x + x1 * c.y);
        const int64_t ko = ((cblk * a.Hkv + hk) * KV_BLOCK + coff) * D;
        if constexpr (F8KV) {
          uint8_t* kr = reinterpret_cast<uint8_t*>(a.k_cache_w) + ko;
          kr[i] = f2fp8(bf2f(y1));
          kr[i + half] = f2fp8(bf2f(y2));
        } else {
          a.k_cache_w[ko + i] = y1;
          a.k_cache_w[ko + i + half] = y2;
        }
      } else {
        const int d = i - half;
        const uint16_t* vr = a.q + (int64_t)b * a.q_sb + (int64_t)(a.H + a.Hkv + hk) * D;
        const int64_t vo = ((cblk * a.Hkv + hk) * D + d) * KV_BLOCK + coff;
        if constexpr (F8KV) reinterpret_cast<uint8_t*>(a.v_cache_w)[vo] = f2fp8(bf2f(vr[d]));
        else a.v_cache_w[vo] = vr[d];
      }
      }
    }
  }

  int64_t* dbg = a.dbg ? a.dbg + ((((int64_t)b * a.Hkv + hk) * gridDim.x + split) << 3) : nullptr;
  if (dbg && lane == 0) {   // per wave: when its block loop ended (stamp 1 + wave)
    dbg[1 + wid] = (int64_t)__builtin_amdgcn_s_memrealtime();
    if (wid == 0) dbg[0] = t_start;
  }
  // ---- merge the NW wave states through LDS
  if (g == 0) {
    sm_ml[wid][0][col] = mrow;
    sm_ml[wid][1][col] = lrow;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) sm_o[wid][j * 16 + 4 * g + r][col] = o[j][r];
  __syncthreads();
  for (int idx = tid; idx < G * D; idx += 64 * NW) {
    const int q = idx / D, d = idx - q * D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sm_ml[w][0][q]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float e = __builtin_amdgcn_exp2f(sm_ml[w][0][q] - M);
        L += sm_ml[w][1][q] * e;
        O += sm_o[w][d][q] * e;
      }
    }
    const int h = hk * G + q;
    if (ns == 1) {
      a.o[(int64_t)b * a.o_sb + (int64_t)h * D + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const int64_t pi = ((int64_t)b * a.H + h) * a.nsplit + split;
      __hip_atomic_store(a.part_o + pi * D + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(a.part_ml + pi * 2, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.part_ml + pi * 2 + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (ns == 1) {
    if (dbg && tid == 0) dbg[5] = (int64_t)__builtin_amdgcn_s_memrealtime();
    return;
  }

  // ---- in-launch combine: the last split of (b, hk) to arrive merges all ns splits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (dbg && tid == 0) dbg[5] = (int64_t)__builtin_amdgcn_s_memrealtime();   // partials published
  if (tid == 0) {
    uint32_t* c = a.split_cnt + (int64_t)b * a.Hkv + hk;
    const uint32_t prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == (uint32_t)ns - 1;
    if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm_last = last ? 1 : 0;
  }
  __syncthreads();
  if (dbg && tid == 0) dbg[6] = (int64_t)__builtin_amdgcn_s_memrealtime();   // ticket back
  if (!sm_last) return;
  // one round trip per 8 splits: every (m, l) and o partial of a chunk is loaded before any is used
  // (the chunk's max rescales the running sums, online-softmax style); split order: deterministic
  for (int idx = tid; idx < G * D; idx += 64 * NW) {
    const int q = idx / D, d = idx - q * D;
    const int h = hk * G + q;
    const int64_t pi0 = ((int64_t)b * a.H + h) * a.nsplit;
    float M = -INFINITY, L = 0.f, O = 0.f;
    for (int s0 = 0; s0 < ns; s0 += 8) {
      float pm[8], pl[8], pv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t pi = pi0 + min(s0 + j, ns - 1);
        pm[j] = __hip_atomic_load(a.part_ml + pi * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pl[j] = __hip_atomic_load(a.part_ml + pi * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pv[j] = __hip_atomic_load(a.part_o + pi * D + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      float mc = M;
#pragma unroll
      for (int j = 0; j < 8; ++j) mc = s0 + j < ns ? fmaxf(mc, pm[j]) : mc;
      if (mc == -INFINITY) continue;
      const float r = __builtin_amdgcn_exp2f(M - mc);   // M = -inf: 0 (L, O still 0)
      L *= r;
      O *= r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (s0 + j < ns) {
          const float e = __builtin_amdgcn_exp2f(pm[j] - mc);
          L += pl[j] * e;
          O += pv[j] * e;
        }
      }
      M = mc;
    }
    a.o[(int64_t)b * a.o_sb + (int64_t)h * D + d] = f2bf(L > 0.f ? O / L : 0.f);
  }
  if (dbg && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dbg[7] = (int64_t)__builtin_amdgcn_s_memrealtime();   // combine done (last split only)
  }
}

hipError_t paged_decode(const DecodeArgs& a, int B, int D, hipStream_t stream) {
  if (a.nsplit > 32 || (a.nsplit > 1 && a.split_cnt == nullptr)) return hipErrorInvalidValue;
  // prefetch slices: enough z-slices of (nsplit x Hkv) workgroups for >= 192 prefetching CUs
  const bool pf = (a.pf[0] != nullptr && a.pf_bytes[0] > 0) || (a.pf[1] != nullptr && a.pf_bytes[1] > 0);
  const int per_z = a.nsplit * a.Hkv;
  const int pfz = pf ? (192 + per_z - 1) / per_z : 0;
  dim3 grid(a.nsplit, a.Hkv, B + pfz), block(64 * PD_NW);
#define PD_LAUNCH(D_)                                                                               \
  do {                                                                                              \
    if (a.kv_fp8) hipLaunchKernelGGL((paged_decode_kernel<D_, true>), grid, block, 0, stream, a, B);  \
    else hipLaunchKernelGGL((paged_decode_kernel<D_, false>), grid, block, 0, stream, a, B);          \
  } while (0)
  if (D == 64) PD_LAUNCH(64);
  else if (D == 128) PD_LAUNCH(128);
  else if (D == 32) PD_LAUNCH(32);
  else return hipErrorInvalidValue;
#undef PD_LAUNCH
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ repetition penalty
__global__ void rep_penalty_kernel(float* logits, int64_t ld, const int* ids, int maxn, const float* penalty, int V) {
  const int b = blockIdx.x;
  const float p = penalty[b];
  for (int j = threadIdx.x; j < maxn; j += blockDim.x) {
    const int id = ids[(int64_t)b * maxn + j];
    if (id < 0 || id >= V) continue;
    float* l = logits + (int64_t)b * ld + id;
    const float v = *l;
    *l = v > 0.f ? v / p : v * p;
  }
}

hipError_t rep_penalty(float* logits, int64_t ld, const int* ids, int maxn, const float* penalty, int B, int V,
                       hipStream_t stream) {
  if (B == 0 || maxn == 0) return hipSuccess;
  hipLaunchKernelGGL(rep_penalty_kernel, dim3(B), dim3(256), 0, stream, logits, ld, ids, maxn, penalty, V);
  return hipGetLastError();
}

// Small integer arrays (token ids, cache slots) uploaded through the kernel arguments: no copy
// engine / blit path, so behind a queue of kernels (a request's prefill inputs behind its image
// tower) the values land one tiny kernel after the queue drains instead of 20-70 us later per
// hipMemcpyAsync (profiles/r5_ttft_*).
__global__ void upload_i64_kernel(UploadArgs a, int64_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a.v[i];
}

hipError_t upload_i64(const UploadArgs& a, int64_t* out, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(upload_i64_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a, out, n);
  return hipGetLastError();
}

}  // namespace lumen
