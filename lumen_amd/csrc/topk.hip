// Row top-k with fused softmax statistics, for zero-shot label-bank
// classification (CLIP / BioCLIP / scene) and vocab sampling candidates.
//
// scores [B, N] fp32 (the MFMA GEMM of query embeddings against the label bank)
// -> top-k values / indices per row (descending) and the row log-sum-exp of
// (scale * scores), so softmax probabilities of the winners are
// exp(scale*s - lse) without a second pass over N.
//
// One workgroup per row: every thread streams a strided slice keeping a sorted
// register list of its K best (compile-time K, unrolled compare-swap insertion)
// and an online (max, sum-exp); the block then merges by K rounds of a block
// arg-max over the list heads.
//
// Replaces the numpy `np.dot / softmax / argsort[::-1][:top_k]` of
// packages/lumen-clip/src/lumen_clip/general_clip/clip_model.py:289-315 and the
// raw-cosine top-k of expert_bioclip/bioclip_model.py:313-316.
#include "common.h"

namespace lumen {

template <int K>
__global__ void __launch_bounds__(256)
row_topk_kernel(const float* __restrict__ scores, int64_t ld, int N, int k, float scale, float* __restrict__ out_v,
                int* __restrict__ out_i, float* __restrict__ out_lse, int index_offset) {
  const int row = blockIdx.x;
  const float* s = scores + (int64_t)row * ld;
  float v[K];
  int id[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { v[i] = -INFINITY; id[i] = -1; }
  float m = -INFINITY, l = 0.f;
  for (int j = threadIdx.x; j < N; j += 256) {
    const float x = s[j];
    const float xs = x * scale;
    if (xs > m) { l = l * __expf(m - xs) + 1.f; m = xs; }
    else l += __expf(xs - m);
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
  }
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  __shared__ float red_m[4], red_l[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // block log-sum-exp
  {
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
      if (out_lse) out_lse[row] = M + logf(L);
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
    if (lane == 0) { red_v[w] = bv; red_i[w] = bt * 0 + bi; red_l[w] = __int_as_float(bt); }
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
      out_v[(int64_t)row * k + r] = fv;
      out_i[(int64_t)row * k + r] = fi < 0 ? -1 : fi + index_offset;
    }
    if (threadIdx.x == ft) {  // pop the winner's head
#pragma unroll
      for (int i = 0; i < K - 1; ++i) { v[i] = v[i + 1]; id[i] = id[i + 1]; }
      v[K - 1] = -INFINITY; id[K - 1] = -1;
    }
  }
}

hipError_t row_topk(const float* scores, int64_t ld, int B, int N, int k, float scale, float* out_v, int* out_i,
                    float* out_lse, int index_offset, hipStream_t stream) {
  dim3 grid(B), block(256);
  if (k <= 8) hipLaunchKernelGGL(row_topk_kernel<8>, grid, block, 0, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset);
  else if (k <= 16) hipLaunchKernelGGL(row_topk_kernel<16>, grid, block, 0, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset);
  else if (k <= 32) hipLaunchKernelGGL(row_topk_kernel<32>, grid, block, 0, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset);
  else if (k <= 64) hipLaunchKernelGGL(row_topk_kernel<64>, grid, block, 0, stream, scores, ld, N, k, scale, out_v, out_i, out_lse, index_offset);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace lumen
