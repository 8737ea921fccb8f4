// DBNet text-detection post-processing on the GPU: threshold + 8-connected component
// labelling + boundary extraction, and the box score of candidate rectangles.
//
// Reference: packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py:380-476
// (cv2.findContours on the thresholded bitmap, cv2.minAreaRect, box_score_fast).  The
// former path copied the whole probability map to the host and labelled it there
// (csrc/host/geometry.cpp: ~1M pixels per 960x960 map on one CPU thread).  Now:
//
//   db_label      lab[p] = p if prob[p] > thresh[img] else -1   (p = global pixel index)
//   db_merge      union-find over the 4 "earlier" 8-neighbours (W, NW, N, NE): roots are
//                 linked with atomicMin, so every component's root is its smallest pixel
//                 index -- the raster-order first pixel, i.e. the same component order
//                 as the host two-pass labelling (max_candidates cuts identically)
//   db_flatten    lab[p] = root(p)
//   db_boundary   (root, x, y) of every pixel with a 4-neighbour outside its component
//                 (or on the map border), appended with one atomic per wave
//   db_quad_score mean probability inside each candidate rectangle (one workgroup each)
//
// Only the boundary list (a few % of the pixels) and the per-box scores cross PCIe; the
// host keeps the cheap geometry (convex hull, rotating calipers, unclip, ordering).
// Atomics are vector-memory (global_atomic_*) operations.
#include "common.h"

namespace lumen {

template <typename T>
__device__ __forceinline__ float ld_prob(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld_prob<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ld_prob<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }

template <typename T>
__global__ void db_label_kernel(const T* __restrict__ prob, const float* __restrict__ thresh, int* __restrict__ lab,
                                int HW, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int img = (int)(i / HW);
  lab[i] = ld_prob<T>(prob, i) > thresh[img] ? (int)i : -1;
}

// L2-coherent reads: other workgroups relink roots with atomics while finds walk the trees
// (every link points to a smaller index, so a stale read only costs an extra step)
__device__ __forceinline__ int db_ld(const int* lab, int i) {
  return __hip_atomic_load(lab + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int db_find(const int* lab, int i) {
  int p = db_ld(lab, i);
  while (p != i) {
    i = p;
    p = db_ld(lab, i);
  }
  return i;
}

__device__ __forceinline__ void db_union(int* lab, int a, int b) {
  while (true) {
    a = db_find(lab, a);
    b = db_find(lab, b);
    if (a == b) return;
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    // link the larger root under the smaller one; if a stopped being a root meanwhile, retry
    const int old = atomicMin(lab + a, b);
    if (old == a) return;
    a = old;
  }
}

__global__ void db_merge_kernel(int* __restrict__ lab, int H, int W, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total || lab[i] < 0) return;
  const int HW = H * W;
  const int p = (int)(i % HW), x = p % W, y = p / W;
  const int dx[4] = {-1, -1, 0, 1}, dy[4] = {0, -1, -1, -1};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = x + dx[k], yy = y + dy[k];
    if (xx < 0 || yy < 0 || xx >= W) continue;
    const int64_t j = i + (int64_t)dy[k] * W + dx[k];
    if (lab[j] >= 0) db_union(lab, (int)i, (int)j);
  }
}

__global__ void db_flatten_kernel(int* __restrict__ lab, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total || lab[i] < 0) return;
  lab[i] = db_find(lab, (int)i);
}

__global__ void db_boundary_kernel(const int* __restrict__ lab, int H, int W, int64_t total, int* __restrict__ out,
                                   int* __restrict__ count, int cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool emit = false;
  int x = 0, y = 0, l = -1;
  if (i < total) {
    l = lab[i];
    if (l >= 0) {
      const int HW = H * W;
      const int p = (int)(i % HW);
      x = p % W;
      y = p / W;
      emit = x == 0 || y == 0 || x == W - 1 || y == H - 1 || lab[i - 1] < 0 || lab[i + 1] < 0 || lab[i - W] < 0 ||
             lab[i + W] < 0;
    }
  }
  // one atomic per wave: ballot the emitting lanes, lane 0 reserves, each lane takes its rank
  const uint64_t m = __ballot(emit);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(m));
  base = __shfl(base, leader, 64);
  if (!emit) return;
  const int k = base + __popcll(m & ((1ull << lane) - 1ull));
  if (k < cap) {
    out[3 * k] = l;
    out[3 * k + 1] = x;
    out[3 * k + 2] = y;
  }
}

// quads [m, 8] (x0,y0 .. x3,y3 in map pixels), img[m] -> score[m] = mean prob of the pixel
// centres inside the quad (host in_quad test, box_score_fast)
template <typename T>
__global__ void __launch_bounds__(256) db_quad_score_kernel(const T* __restrict__ prob, int H, int W,
                                                            const float* __restrict__ quads,
                                                            const int* __restrict__ img, float* __restrict__ score) {
  __shared__ float rs[4], rc[4];
  const int q = blockIdx.x;
  float px[4], py[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    px[k] = quads[q * 8 + 2 * k];
    py[k] = quads[q * 8 + 2 * k + 1];
  }
  float xmin = px[0], xmax = px[0], ymin = py[0], ymax = py[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    xmin = fminf(xmin, px[k]); xmax = fmaxf(xmax, px[k]);
    ymin = fminf(ymin, py[k]); ymax = fmaxf(ymax, py[k]);
  }
  const int x0 = max(0, (int)floorf(xmin)), x1 = min(W - 1, (int)ceilf(xmax));
  const int y0 = max(0, (int)floorf(ymin)), y1 = min(H - 1, (int)ceilf(ymax));
  const int bw = x1 - x0 + 1, bh = y1 - y0 + 1;
  const T* pm = prob + (int64_t)img[q] * H * W;
  float s = 0.f, c = 0.f;
  if (bw > 0 && bh > 0) {
    for (int t = threadIdx.x; t < bw * bh; t += blockDim.x) {
      const float xx = (float)(x0 + t % bw), yy = (float)(y0 + t / bw);
      bool pos = false, neg = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int k1 = (k + 1) & 3;
        // same orientation test as the host path (double there; the corners are pixel-scale floats)
        const float cr = (px[k1] - px[k]) * (yy - py[k]) - (py[k1] - py[k]) * (xx - px[k]);
        pos |= cr > 0.f;
        neg |= cr < 0.f;
      }
      if (!(pos && neg)) {
        s += ld_prob<T>(pm, (int64_t)(y0 + t / bw) * W + x0 + t % bw);
        c += 1.f;
      }
    }
  }
  s = wave_sum(s);
  c = wave_sum(c);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { rs[wid] = s; rc[wid] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S = rs[0] + rs[1] + rs[2] + rs[3], C = rc[0] + rc[1] + rc[2] + rc[3];
    score[q] = C > 0.f ? S / C : 0.f;
  }
}

// prob: [n, H, W] (bf16 if is_bf16 else f32); thresh [n] f32; lab: int32 workspace [n*H*W];
// out: int32 [cap, 3]; count: int32 [1] (zeroed here).
hipError_t db_components(const void* prob, int is_bf16, const float* thresh, int n, int H, int W, int* lab,
                         int* out, int* count, int cap, hipStream_t stream) {
  const int64_t total = (int64_t)n * H * W;
  if (total <= 0 || total >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  const int blocks = (int)((total + 255) / 256);
  (void)hipMemsetAsync(count, 0, sizeof(int), stream);
  if (is_bf16)
    hipLaunchKernelGGL(db_label_kernel<uint16_t>, dim3(blocks), dim3(256), 0, stream, (const uint16_t*)prob, thresh,
                       lab, H * W, total);
  else
    hipLaunchKernelGGL(db_label_kernel<float>, dim3(blocks), dim3(256), 0, stream, (const float*)prob, thresh, lab,
                       H * W, total);
  hipLaunchKernelGGL(db_merge_kernel, dim3(blocks), dim3(256), 0, stream, lab, H, W, total);
  hipLaunchKernelGGL(db_flatten_kernel, dim3(blocks), dim3(256), 0, stream, lab, total);
  hipLaunchKernelGGL(db_boundary_kernel, dim3(blocks), dim3(256), 0, stream, lab, H, W, total, out, count, cap);
  return hipGetLastError();
}

hipError_t db_quad_score(const void* prob, int is_bf16, int H, int W, const float* quads, const int* img, float* score,
                         int m, hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  if (is_bf16)
    hipLaunchKernelGGL(db_quad_score_kernel<uint16_t>, dim3(m), dim3(256), 0, stream, (const uint16_t*)prob, H, W,
                       quads, img, score);
  else
    hipLaunchKernelGGL(db_quad_score_kernel<float>, dim3(m), dim3(256), 0, stream, (const float*)prob, H, W, quads,
                       img, score);
  return hipGetLastError();
}

}  // namespace lumen
