// Fused multi-head attention forward (flash-style, online softmax) for gfx950.
//
// One workgroup = 4 waves = 64 query rows of one (batch, head); each wave owns
// 16 query rows.  K/V stream through LDS in 64-key chunks: K as an XOR-swizzled
// row-major image (B operand of S = Q.K^T, one ds_read_b128 per fragment), V
// transposed into [d][key] (B operand of O += P.V).  P is re-laid from the
// accumulator layout into an A fragment through a per-wave LDS tile.
//
// Covers every attention the reference runs inside its ONNX graphs:
// non-causal ViT (CLIP/BioCLIP vision, seq 197/257/577), causal CLIP text (77),
// key-padded BERT (CN-CLIP), causal GQA decoder prefill (Qwen2 / Llama).
// Q/K/V are read in place from packed projections via strides, and O is
// written as [b, s, h, d] so the out-projection GEMM consumes it directly.
#include "common.h"

namespace lumen {

struct AttnArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o;
  int64_t q_sb, q_ss, q_sh;   // strides (elements) batch / seq / head
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t o_sb, o_ss, o_sh;
  const int* kv_len;          // optional per-batch valid key count
  int Sq, Sk, H, Hkv;
  float scale_log2;           // softmax_scale * log2(e)
  int causal;                 // query i attends keys j <= i + (Sk - Sq)
};

__device__ __forceinline__ int kswz(int row, int chunk, int nchunk) {
  // rows of nchunk 16-byte chunks; XOR keeps a ds_read_b128 lane group on
  // distinct bank slots for both 128-B (D=64) and 256-B (D=128) rows.
  return nchunk == 8 ? (chunk ^ ((row >> 1) & 7))
                     : nchunk == 16 ? (chunk ^ (row & 15)) : (chunk ^ ((row >> 1) & 3));
}

template <int D>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  constexpr int NCH = D / 8;        // 16-byte chunks per K row
  constexpr int KS = D / 32;        // MFMA k-steps over head dim
  constexpr int NB = D / 16;        // 16-wide output column blocks
  constexpr int KC = 64;            // keys per chunk
  __shared__ __attribute__((aligned(16))) char smem[KC * D * 2 * 2 + 4 * 16 * KC * 2];
  char* sK = smem;                        // [KC][D]      swizzled
  char* sV = smem + KC * D * 2;           // [D][KC]      swizzled (8 chunks per row)
  char* sP = smem + KC * D * 2 * 2;       // [4 waves][16][KC]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int hk = h / (a.H / a.Hkv);
  const int q0 = blockIdx.x * 64 + wid * 16;
  const int kv_len = a.kv_len ? min(a.kv_len[b], a.Sk) : a.Sk;
  const int causal_off = a.Sk - a.Sq;

  const uint16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const uint16_t* kb = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hk * a.v_sh;

  // Q fragments (A operand): row q0 + frow, dims 32s + 8fq .. +8
  bf16x8_t qf[KS];
  {
    const int qr = min(q0 + frow, a.Sq - 1);
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *(const bf16x8_t*)(qb + (int64_t)qr * a.q_ss + s * 32 + fq * 8);
  }

  f32x4_t o[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) o[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrow[r] = -INFINITY; lrow[r] = 0.f; }

  int kend = kv_len;
  if (a.causal) kend = min(kend, blockIdx.x * 64 + 64 + causal_off);
  const int nkc = (kend + KC - 1) / KC;

  for (int kc = 0; kc < nkc; ++kc) {
    const int k0 = kc * KC;
    __syncthreads();  // previous chunk fully consumed
    // stage K chunk: KC*NCH 16-byte chunks over 256 threads
    for (int id = tid; id < KC * NCH; id += 256) {
      const int r = id / NCH, c = id % NCH;
      const int kr = min(k0 + r, a.Sk - 1);
      u32x4_t val = *(const u32x4_t*)(kb + (int64_t)kr * a.k_ss + c * 8);
      *(u32x4_t*)(sK + r * D * 2 + (kswz(r, c, NCH) << 4)) = val;
    }
    // stage V transposed: thread loads 8 dims of one key, scatters 8 bf16
    for (int id = tid; id < KC * NCH; id += 256) {
      const int r = id / NCH, c = id % NCH;   // key r, dims c*8..c*8+7
      const int kr = min(k0 + r, a.Sk - 1);
      u32x4_t val = *(const u32x4_t*)(vb + (int64_t)kr * a.v_ss + c * 8);
      const uint16_t* e = (const uint16_t*)&val;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int d = c * 8 + i;
        const int kch = r >> 3;
        *(uint16_t*)(sV + d * KC * 2 + (kswz(d, kch, 8) << 4) + (r & 7) * 2) = e[i];
      }
    }
    __syncthreads();

    // S = Q K^T for 4 key blocks of 16
    f32x4_t sc[4];
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16) {
      sc[kb16] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      const int kr = kb16 * 16 + frow;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8_t kf = *(const bf16x8_t*)(sK + kr * D * 2 + (kswz(kr, s * 4 + fq, NCH) << 4));
        sc[kb16] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], kf, sc[kb16], 0, 0, 0);
      }
    }
    // mask + online softmax.  lane holds S[row fq*4+r][key kb16*16+frow]
    float mnew[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = q0 + fq * 4 + r;
      float mx = mrow[r];
#pragma unroll
      for (int kb16 = 0; kb16 < 4; ++kb16) {
        const int kj = k0 + kb16 * 16 + frow;
        bool ok = kj < kv_len;
        if (a.causal) ok = ok && (kj <= qi + causal_off);
        float sv = ok ? sc[kb16][r] * a.scale_log2 : -INFINITY;
        sc[kb16][r] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      mnew[r] = mx;
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mbase = mnew[r] == -INFINITY ? 0.f : mnew[r];
      alpha[r] = exp2f(mrow[r] - mbase);
      float rs = 0.f;
#pragma unroll
      for (int kb16 = 0; kb16 < 4; ++kb16) {
        float p = exp2f(sc[kb16][r] - mbase);
        sc[kb16][r] = p;
        rs += p;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      lrow[r] = lrow[r] * alpha[r] + rs;
      mrow[r] = mnew[r];
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[j][r] *= alpha[r];

    // P (bf16) -> wave-private LDS tile [16][64], swizzled like K (8 chunks/row)
    char* pw = sP + wid * 16 * KC * 2;
#pragma unroll
    for (int kb16 = 0; kb16 < 4; ++kb16)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = fq * 4 + r, key = kb16 * 16 + frow;
        *(uint16_t*)(pw + pr * KC * 2 + (kswz(pr, key >> 3, 8) << 4) + (key & 7) * 2) = f2bf(sc[kb16][r]);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // O += P V : A = P[16 rows][32 keys] (2 k-steps), B = V[key][d] from sV (transposed image)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t pf = *(const bf16x8_t*)(pw + frow * KC * 2 + (kswz(frow, s * 4 + fq, 8) << 4));
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int d = j * 16 + frow;
        bf16x8_t vf = *(const bf16x8_t*)(sV + d * KC * 2 + (kswz(d, s * 4 + fq, 8) << 4));
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[j], 0, 0, 0);
      }
    }
  }

  // normalise and store O[b, q, h, :]
  uint16_t* ob = a.o + b * a.o_sb + h * a.o_sh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qi = q0 + fq * 4 + r;
    if (qi >= a.Sq) continue;
    const float inv = lrow[r] > 0.f ? 1.0f / lrow[r] : 0.f;
#pragma unroll
    for (int j = 0; j < NB; ++j) ob[(int64_t)qi * a.o_ss + j * 16 + frow] = f2bf(o[j][r] * inv);
  }
}

hipError_t attn_fwd(const AttnArgs& a, int B, int D, hipStream_t stream) {
  dim3 grid((a.Sq + 63) / 64, a.H, B), block(256);
  if (D == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, block, 0, stream, a);
  else if (D == 128) hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, block, 0, stream, a);
  else if (D == 32) hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, block, 0, stream, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace lumen
