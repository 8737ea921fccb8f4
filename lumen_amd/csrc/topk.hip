// Row top-k with fused softmax statistics, for zero-shot label-bank
// classification (CLIP / BioCLIP / scene) and vocab sampling candidates.
//
// scores [B, N] fp32 (the MFMA GEMM of query embeddings against the label bank)
// -> top-k values / indices per row (descending) and the row log-sum-exp of
// (scale * scores), so softmax probabilities of the winners are
// exp(scale*s - lse) without a second pass over N.
//
// One workgroup per row (chunk): every thread streams a strided slice keeping a
// sorted register list of its K best (compile-time K, unrolled compare-swap
// insertion) and an online (max, sum-exp); the block then merges by K rounds of a
// block arg-max over the list heads.  Long rows (LLM vocabularies, 128-152 k
// logits, or million-label banks) run in two phases so a single row still fills
// the GPU: phase 1 = one workgroup per (row, 4096-column chunk) writing k
// candidates + the chunk's (max, sum-exp); phase 2 = one workgroup per row merging
// the candidates (original indices carried along) and the partial statistics.
//
// Replaces the numpy `np.dot / softmax / argsort[::-1][:top_k]` of
// packages/lumen-clip/src/lumen_clip/general_clip/clip_model.py:289-315 and the
// raw-cosine top-k of expert_bioclip/bioclip_model.py:313-316.
#include "common.h"

namespace lumen {

constexpr int TOPK_CHUNK = 4096;

template <int K>
__global__ void __launch_bounds__(256)
row_topk_kernel(const float* __restrict__ scores, int64_t ld, int N, int k, float scale, float* __restrict__ out_v,
                int* __restrict__ out_i, float* __restrict__ out_lse, int index_offset, const int* __restrict__ in_idx,
                const float* __restrict__ in_ml, int nparts, int chunk, float* __restrict__ out_ml) {
  const int row = blockIdx.x, part = blockIdx.y, nblk = gridDim.y;
  const float* s = scores + (int64_t)row * ld;
  const int* ix = in_idx ? in_idx + (int64_t)row * ld : nullptr;
  const int j0 = part * chunk, j1 = min(N, j0 + chunk);
  float v[K];
  int id[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { v[i] = -INFINITY; id[i] = -1; }
  float m = -INFINITY, l = 0.f;
  auto take = [&](const float x, const int j) {
    if (!in_ml) {
      const float xs = x * scale;
      if (xs > m) { l = l * __expf(m - xs) + 1.f; m = xs; }
      else l += __expf(xs - m);
    }
    if (x > v[K - 1]) {
      v[K - 1] = x; id[K - 1] = j;
#pragma unroll
      for (int i = K - 1; i > 0; --i) {
        if (v[i] > v[i - 1]) {
          float tv = v[i]; v[i] = v[i - 1]; v[i - 1] = tv;
          int ti = id[i]; id[i] = id[i - 1]; id[i - 1] = ti;
        }
      }
    }
  };
  // 8 loads in flight per thread before any is consumed: a strided scalar loop paid one
  // dependent memory round trip per element (16 per thread on a 4096-column chunk)
  constexpr int LU = 8;
  for (int j = j0 + threadIdx.x; j < j1; j += 256 * LU) {
    float xv[LU];
    int iv[LU];
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const int jj = min(j + u * 256, j1 - 1);
      xv[u] = s[jj];
      iv[u] = ix ? ix[jj] : jj;
    }
#pragma unroll
    for (int u = 0; u < LU; ++u)
      if (j + u * 256 < j1) take(xv[u], iv[u]);
  }
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  __shared__ float red_m[4], red_l[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t obase = ((int64_t)row * nblk + part) * k;
  // block log-sum-exp (or the merge of phase-1 partials)
  if (in_ml) {
    if (out_lse) {   // merge the phase-1 (max, sum-exp) partials: one per thread, then a block reduction
      const float* pm = in_ml + (int64_t)row * nparts * 2;
      float pmx = -INFINITY, pl = 0.f;
      for (int p = threadIdx.x; p < nparts; p += 256) {
        const float qm = pm[2 * p], ql = pm[2 * p + 1];
        if (qm == -INFINITY) continue;
        if (qm > pmx) { pl = pl * __expf(pmx - qm) + ql; pmx = qm; }
        else pl += ql * __expf(qm - pmx);
      }
      float mm = pmx;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mm = fmaxf(mm, __shfl_xor(mm, o, 64));
      float ll = pmx == -INFINITY ? 0.f : pl * __expf(pmx - mm);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ll += __shfl_xor(ll, o, 64);
      if (lane == 0) { red_m[w] = mm; red_l[w] = ll; }
      __syncthreads();
      if (threadIdx.x == 0) {
        const float M = fmaxf(fmaxf(red_m[0], red_m[1]), fmaxf(red_m[2], red_m[3]));
        float L = 0.f;
        for (int i = 0; i < 4; ++i) L += red_m[i] == -INFINITY ? 0.f : red_l[i] * __expf(red_m[i] - M);
        out_lse[row] = M + logf(L);
      }
    }
  } else {
    float mm = m;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mm = fmaxf(mm, __shfl_xor(mm, o, 64));
    float ll = (m == -INFINITY) ? 0.f : l * __expf(m - mm);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ll += __shfl_xor(ll, o, 64);
    if (lane == 0) { red_m[w] = mm; red_l[w] = ll; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float M = fmaxf(fmaxf(red_m[0], red_m[1]), fmaxf(red_m[2], red_m[3]));
      float L = 0.f;
      for (int i = 0; i < 4; ++i) L += red_m[i] == -INFINITY ? 0.f : red_l[i] * __expf(red_m[i] - M);
      if (out_ml) { out_ml[((int64_t)row * nblk + part) * 2] = M; out_ml[((int64_t)row * nblk + part) * 2 + 1] = L; }
      else if (out_lse) out_lse[row] = M + logf(L);
    }
  }
  // K rounds of block arg-max over list heads
  for (int r = 0; r < k; ++r) {
    float bv = v[0];
    int bi = id[0], bt = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(bv, o, 64);
      int oi = __shfl_xor(bi, o, 64), ot = __shfl_xor(bt, o, 64);
      if (ov > bv || (ov == bv && oi >= 0 && (bi < 0 || oi < bi))) { bv = ov; bi = oi; bt = ot; }
    }
    __syncthreads();
    if (lane == 0) { red_v[w] = bv; red_i[w] = bi; red_l[w] = __int_as_float(bt); }
    __syncthreads();
    float fv = red_v[0];
    int fi = red_i[0], ft = __float_as_int(red_l[0]);
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      if (red_v[q] > fv || (red_v[q] == fv && red_i[q] >= 0 && (fi < 0 || red_i[q] < fi))) {
        fv = red_v[q]; fi = red_i[q]; ft = __float_as_int(red_l[q]);
      }
    }
    if (threadIdx.x == 0) {
      out_v[obase + r] = fv;
      out_i[obase + r] = fi < 0 ? -1 : fi + index_offset;
    }
    if (threadIdx.x == ft) {  // pop the winner's head
#pragma unroll
      for (int i = 0; i < K - 1; ++i) { v[i] = v[i + 1]; id[i] = id[i + 1]; }
      v[K - 1] = -INFINITY; id[K - 1] = -1;
    }
  }
}

template <int K>
static void launch_topk(dim3 grid, hipStream_t stream, const float* scores, int64_t ld, int N, int k, float scale,
                        float* out_v, int* out_i, float* out_lse, int index_offset, const int* in_idx,
                        const float* in_ml, int nparts, int chunk, float* out_ml) {
  hipLaunchKernelGGL(row_topk_kernel<K>, grid, dim3(256), 0, stream, scores, ld, N, k, scale, out_v, out_i, out_lse,
                     index_offset, in_idx, in_ml, nparts, chunk, out_ml);
}

static hipError_t topk_dispatch(dim3 grid, hipStream_t stream, const float* scores, int64_t ld, int N, int k,
                                float scale, float* out_v, int* out_i, float* out_lse, int index_offset,
                                const int* in_idx, const float* in_ml, int nparts, int chunk, float* out_ml) {
  if (k <= 8) launch_topk<8>(grid, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset, in_idx, in_ml, nparts, chunk, out_ml);
  else if (k <= 16) launch_topk<16>(grid, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset, in_idx, in_ml, nparts, chunk, out_ml);
  else if (k <= 32) launch_topk<32>(grid, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset, in_idx, in_ml, nparts, chunk, out_ml);
  else if (k <= 64) launch_topk<64>(grid, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset, in_idx, in_ml, nparts, chunk, out_ml);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

int topk_chunks(int N) { return N > 16384 ? (N + TOPK_CHUNK - 1) / TOPK_CHUNK : 1; }

// ws: float [B * nch * (2k + 2)] (candidate values, candidate indices as int bits, partial (m, l))
hipError_t row_topk(const float* scores, int64_t ld, int B, int N, int k, float scale, float* out_v, int* out_i,
                    float* out_lse, int index_offset, float* ws, hipStream_t stream) {
  const int nch = topk_chunks(N);
  if (nch == 1 || ws == nullptr)
    return topk_dispatch(dim3(B, 1), stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset, nullptr,
                         nullptr, 1, N, nullptr);
  float* cv = ws;
  int* ci = reinterpret_cast<int*>(ws + (int64_t)B * nch * k);
  float* pml = ws + (int64_t)B * nch * k * 2;
  hipError_t e = topk_dispatch(dim3(B, nch), stream, scores, ld, N, k, scale, cv, ci, nullptr, 0, nullptr, nullptr, 1,
                               TOPK_CHUNK, pml);
  if (e != hipSuccess) return e;
  return topk_dispatch(dim3(B, 1), stream, cv, (int64_t)nch * k, nch * k, k, 1.f, out_v, out_i, out_lse,
                       index_offset, ci, pml, nch, nch * k, nullptr);
}

}  // namespace lumen
