// JPEG pixel reconstruction on the GPU: dequantise + 8x8 IDCT per block, then chroma
// upsampling (libjpeg's "fancy" triangle filter, h2v1 / h2v2) + YCbCr -> RGB (libjpeg's
// fixed-point tables) straight into a uint8 HWC image.  The coefficient planes come from the
// parallel entropy decoder (csrc/host/jpeg_decode.cpp); the reference decodes the whole file on
// one CPU thread with Pillow (packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:661-665,
// packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py:716-723).
#include "common.h"
#include "jpeg.h"

namespace lumen {

// JpegPlanes / JpegBatchEntry: jpeg.h

// cos((2x + 1) u pi / 16) * C(u) / 2 with C(0) = 1/sqrt(2)
__constant__ float kIdctCos[8][8] = {
    {0.35355339f, 0.35355339f, 0.35355339f, 0.35355339f, 0.35355339f, 0.35355339f, 0.35355339f, 0.35355339f},
    {0.49039264f, 0.41573481f, 0.27778512f, 0.09754516f, -0.09754516f, -0.27778512f, -0.41573481f, -0.49039264f},
    {0.46193977f, 0.19134172f, -0.19134172f, -0.46193977f, -0.46193977f, -0.19134172f, 0.19134172f, 0.46193977f},
    {0.41573481f, -0.09754516f, -0.49039264f, -0.27778512f, 0.27778512f, 0.49039264f, 0.09754516f, -0.41573481f},
    {0.35355339f, -0.35355339f, -0.35355339f, 0.35355339f, 0.35355339f, -0.35355339f, -0.35355339f, 0.35355339f},
    {0.27778512f, -0.49039264f, 0.09754516f, 0.41573481f, -0.41573481f, -0.09754516f, 0.49039264f, -0.27778512f},
    {0.19134172f, -0.46193977f, 0.46193977f, -0.19134172f, -0.19134172f, 0.46193977f, -0.46193977f, 0.19134172f},
    {0.09754516f, -0.27778512f, 0.41573481f, -0.49039264f, 0.49039264f, -0.41573481f, 0.27778512f, -0.09754516f}};

// 8x8 IDCT of block lbk of component c (threads t = 0..63 of one 64-lane group: row y, column x).
// Separable: the row pass (over u) goes through LDS, then the column pass (over v).
__device__ __forceinline__ void idct_block(const JpegPlanes& P, int c, int64_t lbk, bool live, int t,
                                           float (*sc)[8], float (*sr)[8]) {
  const int y = t >> 3, x = t & 7;
  if (live) sc[y][x] = (float)P.coef[P.coef_off[c] + lbk * 64 + t] * (float)P.qt[c * 64 + t];
  __syncthreads();
  if (live) {   // row pass: for row v = y, output column x
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += kIdctCos[u][x] * sc[y][u];
    sr[y][x] = s;
  }
  __syncthreads();
  if (!live) return;
  float s = 0.f;   // column pass: pixel (x, y)
#pragma unroll
  for (int v = 0; v < 8; ++v) s += kIdctCos[v][y] * sr[v][x];
  const int val = min(255, max(0, (int)rintf(s + 128.f)));
  const int bx = (int)(lbk % P.bw[c]), by = (int)(lbk / P.bw[c]);
  P.samp[P.samp_off[c] + (int64_t)(by * 8 + y) * (P.bw[c] * 8) + bx * 8 + x] = (uint8_t)val;
}

__device__ __forceinline__ void block_comp(const JpegPlanes& P, int64_t b, int& c, int64_t& lbk) {
  const int64_t n0 = (int64_t)P.bw[0] * P.bh[0], n1 = P.ncomp > 1 ? (int64_t)P.bw[1] * P.bh[1] : 0;
  c = b < n0 ? 0 : (b < n0 + n1 ? 1 : 2);
  lbk = b - (c == 0 ? 0 : (c == 1 ? n0 : n0 + n1));
}

__device__ __forceinline__ int64_t jpeg_blocks(const JpegPlanes& P) {
  int64_t n = 0;
  for (int c = 0; c < P.ncomp; ++c) n += (int64_t)P.bw[c] * P.bh[c];
  return n;
}

// 4 blocks per 256-thread workgroup; thread = (block, row y, column x)
__global__ void __launch_bounds__(256) jpeg_idct_kernel(JpegPlanes P, int64_t nblocks, int64_t b1, int64_t b2) {
  __shared__ float sc[4][8][8];   // dequantised coefficients [block][v][u]
  __shared__ float sr[4][8][8];   // after the horizontal pass [block][v][x]
  const int lb = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + lb;
  const bool live = b < nblocks;
  int c;
  int64_t lbk;
  block_comp(P, live ? b : 0, c, lbk);
  (void)b1;
  (void)b2;
  idct_block(P, c, lbk, live, t, sc[lb], sr[lb]);
}

// the entry owning global index i of a batch (entries sorted by start)
template <bool PIX>
__device__ __forceinline__ int batch_entry(const JpegBatchEntry* __restrict__ e, int n, int64_t i) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((PIX ? e[mid].pix0 : e[mid].blk0) <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Batched form: one launch for every image of a batch (each image's block range padded to 4 so a
// workgroup never straddles two images)
__global__ void __launch_bounds__(256) jpeg_idct_batch_kernel(const JpegBatchEntry* __restrict__ entries, int n) {
  __shared__ float sc[4][8][8];
  __shared__ float sr[4][8][8];
  __shared__ int img;
  const int lb = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int64_t b0 = (int64_t)blockIdx.x * 4;
  if (threadIdx.x == 0) img = batch_entry<false>(entries, n, b0);
  __syncthreads();
  const JpegPlanes& P = entries[img].P;
  const int64_t b = b0 - entries[img].blk0 + lb;
  const bool live = b < jpeg_blocks(P);
  int c;
  int64_t lbk;
  block_comp(P, live ? b : 0, c, lbk);
  idct_block(P, c, lbk, live, t, sc[lb], sr[lb]);
}

// libjpeg's fancy upsampling of one chroma sample at output (X, Y) of the full-resolution grid:
// 3/4 nearer + 1/4 farther per axis, edge samples replicated (jdsample.c h2v2 / h2v1)
__device__ __forceinline__ int chroma(const uint8_t* pl, int stride, int dw, int dh, int X, int Y, int h, int v,
                                      int hmax, int vmax) {
  const int sx = (h == hmax) ? 1 : 2, sy = (v == vmax) ? 1 : 2;
  if (sx == 1 && sy == 1) return pl[(int64_t)Y * stride + X];
  const int c = X / sx, r = Y / sy;
  if (sy == 2) {   // h2v2
    const int rf = (Y & 1) ? min(r + 1, dh - 1) : max(r - 1, 0);
    auto colsum = [&](int cc) { return 3 * pl[(int64_t)r * stride + cc] + pl[(int64_t)rf * stride + cc]; };
    const int cs = colsum(c);
    if (X & 1) return (3 * cs + colsum(min(c + 1, dw - 1)) + 7) >> 4;
    return (3 * cs + colsum(max(c - 1, 0)) + 8) >> 4;
  }
  // h2v1
  const int cs = pl[(int64_t)Y * stride + c];
  if (X & 1) return (3 * cs + pl[(int64_t)Y * stride + min(c + 1, dw - 1)] + 2) >> 2;
  return (3 * cs + pl[(int64_t)Y * stride + max(c - 1, 0)] + 1) >> 2;
}

__device__ __forceinline__ void color_pixel(const JpegPlanes& P, int64_t i, uint8_t* __restrict__ out) {
  if (i >= (int64_t)P.width * P.height) return;
  const int X = (int)(i % P.width), Y = (int)(i / P.width);
  const int y = P.samp[P.samp_off[0] + (int64_t)Y * (P.bw[0] * 8) + X];
  uint8_t* o = out + i * 3;
  if (P.ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)y;
    return;
  }
  int cb, cr;
  {
    const int dw = (P.width * P.h[1] + P.hmax - 1) / P.hmax, dh = (P.height * P.v[1] + P.vmax - 1) / P.vmax;
    cb = chroma(P.samp + P.samp_off[1], P.bw[1] * 8, dw, dh, X, Y, P.h[1], P.v[1], P.hmax, P.vmax) - 128;
  }
  {
    const int dw = (P.width * P.h[2] + P.hmax - 1) / P.hmax, dh = (P.height * P.v[2] + P.vmax - 1) / P.vmax;
    cr = chroma(P.samp + P.samp_off[2], P.bw[2] * 8, dw, dh, X, Y, P.h[2], P.v[2], P.hmax, P.vmax) - 128;
  }
  // jdcolor.c fixed point (SCALEBITS 16)
  const int r = y + ((91881 * cr + 32768) >> 16);
  const int g = y + ((-22554 * cb - 46802 * cr + 32768) >> 16);
  const int b = y + ((116130 * cb + 32768) >> 16);
  o[0] = (uint8_t)min(255, max(0, r));
  o[1] = (uint8_t)min(255, max(0, g));
  o[2] = (uint8_t)min(255, max(0, b));
}

__global__ void __launch_bounds__(256) jpeg_color_kernel(JpegPlanes P, uint8_t* __restrict__ out) {
  color_pixel(P, (int64_t)blockIdx.x * 256 + threadIdx.x, out);
}

// batched form (each image's pixel range padded to 256: one image per workgroup)
__global__ void __launch_bounds__(256) jpeg_color_batch_kernel(const JpegBatchEntry* __restrict__ entries, int n) {
  __shared__ int img;
  const int64_t p0 = (int64_t)blockIdx.x * 256;
  if (threadIdx.x == 0) img = batch_entry<true>(entries, n, p0);
  __syncthreads();
  const JpegBatchEntry& e = entries[img];
  color_pixel(e.P, p0 - e.pix0 + threadIdx.x, e.out);
}

hipError_t jpeg_reconstruct(const JpegPlanes& P, uint8_t* out, hipStream_t stream) {
  if (P.ncomp != 1 && P.ncomp != 3) return hipErrorInvalidValue;
  int64_t nb[3] = {0, 0, 0};
  for (int c = 0; c < P.ncomp; ++c) nb[c] = (int64_t)P.bw[c] * P.bh[c];
  const int64_t b1 = nb[0], b2 = nb[0] + nb[1], total = b2 + nb[2];
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((total + 3) / 4)), dim3(256), 0, stream, P, total, b1, b2);
  const int64_t px = (int64_t)P.width * P.height;
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((px + 255) / 256)), dim3(256), 0, stream, P, out);
  return hipGetLastError();
}

hipError_t jpeg_reconstruct_batch(const JpegBatchEntry* entries, int n, int64_t total_blk, int64_t total_pix,
                                  hipStream_t stream) {
  if (n <= 0 || total_blk % 4 != 0 || total_pix % 256 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(jpeg_idct_batch_kernel, dim3((unsigned)(total_blk / 4)), dim3(256), 0, stream, entries, n);
  hipLaunchKernelGGL(jpeg_color_batch_kernel, dim3((unsigned)(total_pix / 256)), dim3(256), 0, stream, entries, n);
  return hipGetLastError();
}

}  // namespace lumen
