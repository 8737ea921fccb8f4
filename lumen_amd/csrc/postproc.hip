// Detection / recognition post-processing kernels.
//
//  * det_decode: SCRFD-style anchor decode of one FPN stride, fused with the
//    score threshold, distance2bbox / distance2kps, un-letterbox rescale, clip
//    and face-size filter; survivors are appended to a per-image candidate list
//    through an atomic counter (reference face onnxrt_backend.py:425-468,
//    882-1153, 1208-1259; SURVEY F-3/F-5).  Also decodes RetinaFace-style
//    prior-box outputs (F-4: centre/size regression with variances) and already-decoded
//    (boxes, scores, landmarks) exports (reference onnxrt_backend.py:810-880).
//  * nms: per-image greedy NMS on the candidate list (one workgroup per image:
//    bitonic sort by score in LDS, then the kept set is swept in score order
//    with a block-parallel IoU suppression per kept box; reference _nms
//    onnxrt_backend.py:391-422).
//  * warp_affine_batch: bilinear warpAffine (cv2 INTER_LINEAR, constant-0
//    border) of every detected face into the 112x112 recogniser batch, fused
//    with RGB->BGR and (x/255 - 0.5)/0.5 (F-7/F-8), and the same kernel with a
//    3x3 matrix for OCR perspective crops into the padded recogniser batch (O-5/O-6).
//  * ctc_greedy: per (sequence, timestep) arg-max over the class axis and the
//    blank/repeat collapse with the mean confidence (O-8).
#include "common.h"
#include "workspace.h"
#include "postproc.h"

namespace lumen {



__global__ void det_decode_kernel(DetDecodeArgs a) {
  const int n = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.P) return;
  const int loc_i = i / a.A, anc = i % a.A;
  const bool strided = a.sL > 0;
  float s = strided ? a.scores[n * a.sN + loc_i * a.sL + anc] : a.scores[(int64_t)n * a.P + i];
  if (a.apply_sigmoid) s = 1.f / (1.f + __expf(-s));
  if (!(s >= a.thresh)) return;
  const float* bb = strided ? a.bbox + n * a.sN + loc_i * a.sL + anc * 4 : a.bbox + ((int64_t)n * a.P + i) * 4;
  float x1, y1, x2, y2, cx, cy, pw = 0.f, ph = 0.f;
  const bool decoded = a.priors == nullptr && a.stride < 0;
  // decoded mode (generic detector exports that emit boxes directly, reference
  // _decode_detection_outputs non-SCRFD branch): bbox = (x1, y1, x2, y2) in network-input pixels
  // times (in_w, in_h), or, with in_w < 0, normalised to the ORIGINAL image (reference
  // normalized_boxes): scaled by the image size here and by the letterbox scale so the common
  // "/ sc" below cancels
  const float fx = decoded ? (a.in_w < 0.f ? a.img_hw[n * 2 + 1] * a.img_scale[n] : a.in_w) : 0.f;
  const float fy = decoded ? (a.in_h < 0.f ? a.img_hw[n * 2 + 0] * a.img_scale[n] : a.in_h) : 0.f;
  if (decoded) {
    cx = cy = 0.f;
    x1 = bb[0] * fx; y1 = bb[1] * fy; x2 = bb[2] * fx; y2 = bb[3] * fy;
  } else if (a.priors == nullptr) {
    const int loc = i / a.A;
    cx = (float)((loc % a.W) * a.stride);
    cy = (float)((loc / a.W) * a.stride);
    x1 = cx - bb[0] * a.stride; y1 = cy - bb[1] * a.stride;
    x2 = cx + bb[2] * a.stride; y2 = cy + bb[3] * a.stride;
  } else {
    const float* pr = a.priors + (int64_t)i * 4;
    cx = pr[0] + bb[0] * a.var0 * pr[2];
    cy = pr[1] + bb[1] * a.var0 * pr[3];
    pw = pr[2] * __expf(bb[2] * a.var1);
    ph = pr[3] * __expf(bb[3] * a.var1);
    x1 = (cx - pw * 0.5f) * a.in_w; y1 = (cy - ph * 0.5f) * a.in_h;
    x2 = (cx + pw * 0.5f) * a.in_w; y2 = (cy + ph * 0.5f) * a.in_h;
  }
  const float sc = a.img_scale[n];
  const float ih = a.img_hw[n * 2 + 0], iw = a.img_hw[n * 2 + 1];
  x1 = fminf(fmaxf(x1 / sc, 0.f), iw); x2 = fminf(fmaxf(x2 / sc, 0.f), iw);
  y1 = fminf(fmaxf(y1 / sc, 0.f), ih); y2 = fminf(fmaxf(y2 / sc, 0.f), ih);
  const float fw = x2 - x1, fh = y2 - y1;
  const float side = fminf(fw, fh);
  if (side < a.min_size || fmaxf(fw, fh) > a.max_size) return;
  const int slot = atomicAdd(&a.count[n], 1);
  if (slot >= a.max_cand) return;
  float* o = a.cand + ((int64_t)n * a.max_cand + slot) * 16;
  o[0] = x1; o[1] = y1; o[2] = x2; o[3] = y2; o[4] = s;
  if (a.kps) {
    const float* kp = strided ? a.kps + n * a.sN + loc_i * a.sL + anc * 10 : a.kps + ((int64_t)n * a.P + i) * 10;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      float kx, ky;
      if (decoded) {
        kx = kp[2 * k] * fx; ky = kp[2 * k + 1] * fy;
      } else if (a.priors == nullptr) {
        kx = cx + kp[2 * k] * a.stride; ky = cy + kp[2 * k + 1] * a.stride;
      } else {
        const float* pr = a.priors + (int64_t)i * 4;
        kx = (pr[0] + kp[2 * k] * a.var0 * pr[2]) * a.in_w;
        ky = (pr[1] + kp[2 * k + 1] * a.var0 * pr[3]) * a.in_h;
      }
      o[5 + 2 * k] = kx / sc; o[6 + 2 * k] = ky / sc;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 10; ++k) o[5 + k] = -1.f;
  }
  o[15] = 0.f;
}

hipError_t det_decode(const DetDecodeArgs& a, hipStream_t stream) {
  dim3 grid((a.P + 255) / 256, a.N), block(256);
  hipLaunchKernelGGL(det_decode_kernel, grid, block, 0, stream, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- NMS
// one workgroup (256 threads) per image; up to 1024 candidates
__global__ void __launch_bounds__(256)
nms_kernel(const float* __restrict__ cand, const int* __restrict__ count, int max_cand, float iou_thr, int max_out,
           int* __restrict__ keep, int* __restrict__ keep_n) {
  constexpr int CAP = 1024;
  __shared__ float sc[CAP];
  __shared__ int id[CAP];
  __shared__ float bx[CAP][4];
  __shared__ unsigned char alive[CAP];
  __shared__ int nkeep;
  const int n = blockIdx.x;
  const int cnt = min(min(count[n], max_cand), CAP);
  int P2 = 1;
  while (P2 < cnt) P2 <<= 1;
  for (int i = threadIdx.x; i < P2; i += 256) {
    sc[i] = i < cnt ? cand[((int64_t)n * max_cand + i) * 16 + 4] : -INFINITY;
    id[i] = i;
  }
  __syncthreads();
  // bitonic sort descending by score
  for (int k = 2; k <= P2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P2; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool desc = (i & k) == 0;
          const bool sw = desc ? (sc[i] < sc[ixj]) : (sc[i] > sc[ixj]);
          if (sw) {
            float t = sc[i]; sc[i] = sc[ixj]; sc[ixj] = t;
            int u = id[i]; id[i] = id[ixj]; id[ixj] = u;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < cnt; i += 256) {
    const float* c = cand + ((int64_t)n * max_cand + id[i]) * 16;
    bx[i][0] = c[0]; bx[i][1] = c[1]; bx[i][2] = c[2]; bx[i][3] = c[3];
    alive[i] = 1;
  }
  if (threadIdx.x == 0) nkeep = 0;
  __syncthreads();
  for (int i = 0; i < cnt; ++i) {
    if (!alive[i]) continue;  // uniform: alive[] only changes between barriers
    if (threadIdx.x == 0) {
      if (nkeep < max_out) keep[n * max_out + nkeep] = id[i];
      nkeep++;
    }
    const float ax1 = bx[i][0], ay1 = bx[i][1], ax2 = bx[i][2], ay2 = bx[i][3];
    const float aa = (ax2 - ax1) * (ay2 - ay1);  // continuous-area IoU, +1e-8 (reference _nms)
    for (int j = i + 1 + threadIdx.x; j < cnt; j += 256) {
      if (!alive[j]) continue;
      const float xx1 = fmaxf(ax1, bx[j][0]), yy1 = fmaxf(ay1, bx[j][1]);
      const float xx2 = fminf(ax2, bx[j][2]), yy2 = fminf(ay2, bx[j][3]);
      const float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
      const float inter = w * h;
      const float ab = (bx[j][2] - bx[j][0]) * (bx[j][3] - bx[j][1]);
      if (inter / (aa + ab - inter + 1e-8f) > iou_thr) alive[j] = 0;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) keep_n[n] = min(nkeep, max_out);
}

hipError_t nms(const float* cand, const int* count, int N, int max_cand, float iou_thr, int max_out, int* keep,
               int* keep_n, hipStream_t stream) {
  hipLaunchKernelGGL(nms_kernel, dim3(N), dim3(256), 0, stream, cand, count, max_cand, iou_thr, max_out, keep, keep_n);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- warps
// out[f, y, x, c] for c < 3 (channel-padded to cpad) =
//   ((sample(src_f, Minv * (x, y, 1)) [c or 2-c]) * scale - mean) * inv_std
// M is a 3x3 inverse map (affine: last row 0 0 1).  bilinear, constant 0 border
// (cv2 warpAffine/warpPerspective defaults) or replicate.  Output region [0, ow_f) x [0, OH)
// of a (OH x OW) canvas; columns beyond ow_f are zero (OCR width bucketing).


__device__ __forceinline__ float cub(float x) {
  const float a = -0.75f;
  x = fabsf(x);
  if (x < 1.f) return ((a + 2.f) * x - (a + 3.f)) * x * x + 1.f;
  if (x < 2.f) return (((x - 5.f) * x + 8.f) * x - 4.f) * a;
  return 0.f;
}

__global__ void warp_kernel(WarpArgs a) {
  const int f = blockIdx.z;
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= a.OW || y >= a.OH) return;
  const int64_t off = a.meta[f * 4 + 0];
  const int h = (int)a.meta[f * 4 + 1], w = (int)a.meta[f * 4 + 2], ow = (int)a.meta[f * 4 + 3];
  const float* M = a.minv + f * 9;
  float v[3] = {0.f, 0.f, 0.f};
  bool inside = x < ow;
  if (inside) {
    const float X = M[0] * x + M[1] * y + M[2], Y = M[3] * x + M[4] * y + M[5];
    const float Z = M[6] * x + M[7] * y + M[8];
    const float sx = X / Z, sy = Y / Z;
    const uint8_t* img = a.src + off;
    if (!a.cubic) {
      const int x0 = (int)floorf(sx), y0 = (int)floorf(sy);
      const float fx = sx - x0, fy = sy - y0;
      for (int dy = 0; dy < 2; ++dy)
        for (int dx = 0; dx < 2; ++dx) {
          int xx = x0 + dx, yy = y0 + dy;
          if (a.replicate) { xx = min(max(xx, 0), w - 1); yy = min(max(yy, 0), h - 1); }
          else if (xx < 0 || yy < 0 || xx >= w || yy >= h) continue;
          const float wt = (dx ? fx : 1.f - fx) * (dy ? fy : 1.f - fy);
          const uint8_t* p = img + ((int64_t)yy * w + xx) * 3;
          v[0] += wt * p[0]; v[1] += wt * p[1]; v[2] += wt * p[2];
        }
    } else {
      const int x0 = (int)floorf(sx), y0 = (int)floorf(sy);
      const float fx = sx - x0, fy = sy - y0;
      for (int dy = -1; dy < 3; ++dy)
        for (int dx = -1; dx < 3; ++dx) {
          int xx = x0 + dx, yy = y0 + dy;
          if (a.replicate) { xx = min(max(xx, 0), w - 1); yy = min(max(yy, 0), h - 1); }
          else if (xx < 0 || yy < 0 || xx >= w || yy >= h) continue;
          const float wt = cub(dx - fx) * cub(dy - fy);
          const uint8_t* p = img + ((int64_t)yy * w + xx) * 3;
          v[0] += wt * p[0]; v[1] += wt * p[1]; v[2] += wt * p[2];
        }
    }
  }
  uint16_t* o = a.out + (((int64_t)f * a.OH + y) * a.OW + x) * a.cpad;
  for (int c = 0; c < a.cpad; ++c) {
    float r = 0.f;
    if (c < 3 && inside) {
      const float px = fminf(fmaxf(rintf(v[a.swap_rb ? 2 - c : c]), 0.f), 255.f);
      r = (px * a.scale - a.mean) * a.inv_std;
    }
    o[c] = f2bf(r);
  }
}

hipError_t warp_batch(const WarpArgs& a, hipStream_t stream) {
  dim3 grid((a.OW + 127) / 128, a.OH, a.F), block(128);
  hipLaunchKernelGGL(warp_kernel, grid, block, 0, stream, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- CTC
// probs [B, T, C] fp32 -> idx [B, T] (arg-max), conf [B, T] (max prob).  With from_logits
// the row holds raw logits and conf = softmax(row)[argmax] = 1 / sum_j exp(l_j - l_max),
// computed with a per-lane online sum — the recogniser's softmax is fused away.
__global__ void ctc_argmax_kernel(const float* __restrict__ probs, int rows, int C, int from_logits,
                                  int* __restrict__ idx, float* __restrict__ conf) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;  // wave-uniform
  const float* p = probs + (int64_t)row * C;
  float best = -INFINITY, sum = 0.f;
  int bi = 0;
  for (int c = lane; c < C; c += 64) {
    const float v = p[c];
    if (v > best) {
      if (from_logits) sum = sum * __expf(best - v) + 1.f;
      best = v;
      bi = c;
    } else if (from_logits) {
      sum += __expf(v - best);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    const float os = __shfl_xor(sum, o, 64);
    if (from_logits) {
      const float m = fmaxf(best, ov);
      sum = (best == -INFINITY ? 0.f : sum * __expf(best - m)) + (ov == -INFINITY ? 0.f : os * __expf(ov - m));
    }
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if (lane == 0) { idx[row] = bi; conf[row] = from_logits ? 1.f / sum : best; }
}

// collapse: one wave per sequence (4 per workgroup); out_ids [B, T] (-1 padded), out_len [B],
// out_conf [B] (mean prob).  tlen (optional) = valid time steps per sequence (width-bucketed
// batches).  64 time steps per pass: keep = not blank and not the previous step's class, the kept
// steps' output slots from a ballot prefix count.  (The former thread-per-sequence loop was a chain
// of ~T dependent global round trips: ~85 us for 64 crops x 108 steps, more than the classifier.)
__global__ void __launch_bounds__(256) ctc_collapse_kernel(const int* __restrict__ idx, const float* __restrict__ conf,
                                                           int B, int T, int blank, const int* __restrict__ tlen,
                                                           int* __restrict__ out_ids, int* __restrict__ out_len,
                                                           float* __restrict__ out_conf) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;      // wave-uniform
  const int Tb = tlen ? min(max(tlen[b], 0), T) : T;
  const int64_t row = (int64_t)b * T;
  int n = 0, carry = -1;   // carry: the class of the step before this pass
  float s = 0.f;
  for (int t0 = 0; t0 < Tb; t0 += 64) {
    const int t = t0 + lane;
    const bool in = t < Tb;
    const int c = in ? idx[row + t] : blank;
    int cp = __shfl_up(c, 1, 64);
    if (lane == 0) cp = carry;
    const bool keep = in && c != blank && c != cp;
    const unsigned long long mask = __ballot(keep);
    if (keep) out_ids[row + n + __popcll(mask & ((1ull << lane) - 1ull))] = c;
    s += wave_sum(keep ? conf[row + t] : 0.f);
    n += __popcll(mask);
    carry = __shfl(c, 63, 64);
  }
  for (int t = n + lane; t < T; t += 64) out_ids[row + t] = -1;
  if (lane == 0) {
    out_len[b] = n;
    out_conf[b] = n > 0 ? s / n : 0.f;
  }
}

// Recogniser classifier fused with the CTC arg-max (O-8): logits = h . W^T + bias are never
// stored.  For the PP-OCR recogniser (6625 classes, ~25k time steps per batch) the fp32 logits
// are ~650 MB; here each workgroup keeps 128 rows of h in registers (4 waves x 2 MFMA row
// fragments), streams W (L2-resident, [N, K] bf16) through a double-buffered, XOR-swizzled LDS
// tile of 64 classes, and folds every tile into per-row online (max, arg-max, sum of exp)
// states; one 16-lane reduction at the end gives idx[row] and conf[row] = 1 / sum (the softmax
// probability of the arg-max, what ctc_argmax_kernel computes from stored logits).  Ties keep the
// smaller class index.  K in {64, 128, 256}; classes >= C (padding) never win.
// Split form (gridDim.y = S > 1): workgroup (x, y) folds the class tiles of split y only and writes its
// per-row (max, sum, arg-max) state to part[y][row]; cls_argmax_combine merges the S states per row.  A
// batch of 320 crops x 40 steps is 100 row blocks: one workgroup per CU for a fifth of the CUs and
// 104 class tiles each (VALU-bound fold, one wave per SIMD) -- S = 8 spreads it over the chip.
struct ClsPart {
  float m, s;
  int idx, pad;
};

template <int K>
__global__ void __launch_bounds__(256) cls_argmax_kernel(const uint16_t* __restrict__ h, int64_t ldh,
                                                         const uint16_t* __restrict__ w, const float* __restrict__ bias,
                                                         int M, int N, int C, int* __restrict__ idx_out,
                                                         float* __restrict__ conf_out, ClsPart* __restrict__ part) {
  constexpr int KS = K / 32;          // MFMA k-steps
  constexpr int CPR = K / 8;          // 16-byte chunks per W row
  constexpr int TILE = 64 * K * 2;    // bytes of one 64-class W tile
  constexpr int LPT = TILE / (256 * 16);   // 16-byte loads per thread per tile
  __shared__ __attribute__((aligned(16))) char sw[2][TILE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 15, g = lane >> 4;
  const int row0 = blockIdx.x * 128 + wid * 32;
  // A fragments of the wave's 2 x 16 rows, whole K, kept in registers
  bf16x8_t fa[2][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = min(row0 + i * 16 + frow, M - 1);
#pragma unroll
    for (int t = 0; t < KS; ++t) fa[i][t] = *(const bf16x8_t*)(h + (int64_t)r * ldh + t * 32 + g * 8);
  }
  const int ntile_all = (N + 63) / 64;
  const int tps = (ntile_all + (int)gridDim.y - 1) / (int)gridDim.y;   // class tiles of this split
  const int t0 = (int)blockIdx.y * tps;
  const int ntile = max(0, min(ntile_all - t0, tps));
  auto load_tile = [&](int nt_, u32x4_t (&v)[LPT]) {
    const int nt = t0 + nt_;
#pragma unroll
    for (int q = 0; q < LPT; ++q) {
      const int c = tid + q * 256;                 // 16-byte chunk of the tile
      const int r = c / CPR, ch = c % CPR;
      const int n = min(nt * 64 + r, N - 1);
      v[q] = *(const u32x4_t*)(w + (int64_t)n * K + ch * 8);
    }
  };
  auto store_tile = [&](int buf, const u32x4_t (&v)[LPT]) {
#pragma unroll
    for (int q = 0; q < LPT; ++q) {
      const int c = tid + q * 256;
      const int r = c / CPR, ch = c % CPR;
      *(u32x4_t*)(sw[buf] + r * (K * 2) + ((ch ^ (r % CPR)) << 4)) = v[q];
    }
  };
  const float L2E = 1.4426950408889634f;
  float m[2][4], s[2][4];
  int bi[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      m[i][r] = -1e30f;      // finite: the branch-free fold never forms -inf - -inf
      s[i][r] = 0.f;
      bi[i][r] = 0;
    }
  u32x4_t stage[LPT];
  if (ntile > 0) {
    load_tile(0, stage);
    store_tile(0, stage);
  }
  __syncthreads();
  for (int nt_ = 0; nt_ < ntile; ++nt_) {
    const int buf = nt_ & 1;
    const int nt = t0 + nt_;
    if (nt_ + 1 < ntile) load_tile(nt_ + 1, stage);   // lands while this tile computes
    f32x4_t acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KS; ++t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = j * 16 + frow, ch = t * 4 + g;
        const bf16x8_t fb = *(const bf16x8_t*)(sw[buf] + r * (K * 2) + ((ch ^ (r % CPR)) << 4));
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][t], fb, acc[i][j], 0, 0, 0);
      }
    }
    // fold the tile, branch-free: lane column n_j = nt*64 + 16j + frow, rows 16i + 4g + r.  Per row slot
    // the 4 columns' max / first arg-max and the rescaled sum of exp; a per-value branch (the old form)
    // put ~50 instructions of exec-mask juggling on every logit (profiles/r6_ocr_kernel_stats).
    int col[4];
    float bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      col[j] = nt * 64 + j * 16 + frow;
      bl[j] = col[j] < C ? (bias ? bias[col[j]] * L2E : 0.f) : -INFINITY;   // padding classes never win
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaf(acc[i][j][r], L2E, bl[j]);
        const float tm = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        int tc = col[3];
        tc = v[2] == tm ? col[2] : tc;
        tc = v[1] == tm ? col[1] : tc;
        tc = v[0] == tm ? col[0] : tc;
        const float mo = m[i][r], mn = fmaxf(mo, tm);
        bi[i][r] = tm > mo ? tc : bi[i][r];      // strict: an equal later column keeps the earlier index
        s[i][r] = s[i][r] * __builtin_amdgcn_exp2f(mo - mn) + __builtin_amdgcn_exp2f(v[0] - mn) +
                  __builtin_amdgcn_exp2f(v[1] - mn) + __builtin_amdgcn_exp2f(v[2] - mn) +
                  __builtin_amdgcn_exp2f(v[3] - mn);
        m[i][r] = mn;
      }
    if (nt_ + 1 < ntile) {
      __syncthreads();                 // every wave is done reading buf ^ 1 (tile nt - 1)
      store_tile(buf ^ 1, stage);
      __syncthreads();
    }
  }
  // reduce the 16 lanes (frow) that share each row
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float bm = m[i][r], bs = s[i][r];
      int bx = bi[i][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float om = __shfl_xor(bm, o, 64), os = __shfl_xor(bs, o, 64);
        const int ox = __shfl_xor(bx, o, 64);
        const float mm = fmaxf(bm, om);
        const float ns = (bm == -INFINITY ? 0.f : bs * __builtin_amdgcn_exp2f(bm - mm)) +
                         (om == -INFINITY ? 0.f : os * __builtin_amdgcn_exp2f(om - mm));
        if (om > bm || (om == bm && ox < bx)) bx = ox;
        bm = mm;
        bs = ns;
      }
      const int row = row0 + i * 16 + 4 * g + r;
      if (frow == 0 && row < M) {
        if (part != nullptr) {
          part[(int64_t)blockIdx.y * M + row] = ClsPart{bm, bs, bx, 0};
        } else {
          idx_out[row] = bx;
          conf_out[row] = bs > 0.f ? 1.f / bs : 0.f;
        }
      }
    }
}

// merge the S split states of every row (split order: deterministic; ties keep the smaller class)
__global__ void __launch_bounds__(256) cls_argmax_combine_kernel(const ClsPart* __restrict__ part, int S, int M,
                                                                 int* __restrict__ idx_out,
                                                                 float* __restrict__ conf_out) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= M) return;
  float bm = -INFINITY, bs = 0.f;
  int bx = 0;
  for (int y = 0; y < S; ++y) {
    const ClsPart p = part[(int64_t)y * M + row];
    if (p.m == -INFINITY) continue;
    const float mm = fmaxf(bm, p.m);
    bs = (bm == -INFINITY ? 0.f : bs * __builtin_amdgcn_exp2f(bm - mm)) + p.s * __builtin_amdgcn_exp2f(p.m - mm);
    if (p.m > bm || (p.m == bm && p.idx < bx)) bx = p.idx;
    bm = mm;
  }
  idx_out[row] = bx;
  conf_out[row] = bs > 0.f ? 1.f / bs : 0.f;
}

hipError_t cls_argmax(const uint16_t* h, int64_t ldh, const uint16_t* w, const float* bias, int M, int N, int K, int C,
                      int* idx_out, float* conf_out, hipStream_t stream) {
  if (M <= 0) return hipSuccess;
  const int rb = (M + 127) / 128, ntile = (N + 63) / 64;
  // class splits: ~3 workgroups per CU of 256, at least 4 class tiles each
  int S = (768 + rb - 1) / rb;
  S = S < 1 ? 1 : S > 16 ? 16 : S;
  while (S > 1 && ntile / S < 4) --S;
  ClsPart* part = nullptr;
  if (S > 1) {
    part = (ClsPart*)stream_workspace((size_t)S * M * sizeof(ClsPart), stream, WS_CLS_PART, (size_t)1 << 20);
    if (part == nullptr) S = 1;
  }
  const dim3 grid(rb, S);
  switch (K) {
    case 64: hipLaunchKernelGGL(cls_argmax_kernel<64>, grid, dim3(256), 0, stream, h, ldh, w, bias, M, N, C, idx_out, conf_out, part); break;
    case 128: hipLaunchKernelGGL(cls_argmax_kernel<128>, grid, dim3(256), 0, stream, h, ldh, w, bias, M, N, C, idx_out, conf_out, part); break;
    case 256: hipLaunchKernelGGL(cls_argmax_kernel<256>, grid, dim3(256), 0, stream, h, ldh, w, bias, M, N, C, idx_out, conf_out, part); break;
    default: return hipErrorInvalidValue;
  }
  if (part != nullptr)
    hipLaunchKernelGGL(cls_argmax_combine_kernel, dim3((M + 255) / 256), dim3(256), 0, stream, part, S, M, idx_out,
                       conf_out);
  return hipGetLastError();
}

hipError_t ctc_collapse(const int* idx, const float* conf, int B, int T, int blank, const int* tlen, int* out_ids,
                        int* out_len, float* out_conf, hipStream_t stream) {
  hipLaunchKernelGGL(ctc_collapse_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, idx, conf, B, T, blank, tlen,
                     out_ids, out_len, out_conf);
  return hipGetLastError();
}

hipError_t ctc_greedy(const float* probs, int B, int T, int C, int blank, int from_logits, const int* tlen,
                      int* tmp_idx, float* tmp_conf, int* out_ids, int* out_len, float* out_conf, hipStream_t stream) {
  const int rows = B * T;
  hipLaunchKernelGGL(ctc_argmax_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, probs, rows, C, from_logits,
                     tmp_idx, tmp_conf);
  hipLaunchKernelGGL(ctc_collapse_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, tmp_idx, tmp_conf, B, T, blank,
                     tlen, out_ids, out_len, out_conf);
  return hipGetLastError();
}

}  // namespace lumen
