// Shared host/device declarations of the post-processing kernels (postproc.hip)
// and their torch bindings (ops_post.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lumen {

struct DetDecodeArgs {
  const float* scores;   // [N, H*W*A]           (already sigmoid'ed) — or [N, P] priors mode
  const float* bbox;     // [N, H*W*A, 4]        distances (in stride units) or prior deltas
  const float* kps;      // [N, H*W*A, 10] or null
  const float* priors;   // [P, 4] (cx, cy, w, h) normalised, RetinaFace mode; null = SCRFD anchors
  int N, H, W, A, stride;  // stride < 0 with priors null: already-decoded boxes (x1 y1 x2 y2) * (in_w, in_h)
  int P;                 // candidates per image in this level
  float thresh;
  const float* img_scale;  // [N] letterbox scale (det size / original)
  const float* img_hw;     // [N, 2] original (h, w)
  float min_size, max_size;
  float var0, var1;        // RetinaFace variances
  float in_w, in_h;        // network input size (priors mode)
  float* cand;             // [N, max_cand, 16]: x1 y1 x2 y2 score kps*10 pad
  int* count;              // [N]
  int max_cand;
  // generalised addressing (fused head conv outputs, NHWC): element (n, loc, a, j) of
  // scores/bbox/kps lives at base + n*sN + loc*sL + a*{1,4,10} + j
  int64_t sN, sL;
  int apply_sigmoid;
};
hipError_t det_decode(const DetDecodeArgs& a, hipStream_t stream);
hipError_t nms(const float* cand, const int* count, int N, int max_cand, float iou_thr, int max_out, int* keep,
               int* keep_n, hipStream_t stream);

struct WarpArgs {
  const uint8_t* src;
  const int64_t* meta;   // [F, 4]: byte offset, h, w, out_w (valid output width)
  const float* minv;     // [F, 9]
  uint16_t* out;         // [F, OH, OW, cpad] bf16
  int F, OH, OW, cpad;
  float scale, mean, inv_std;
  int swap_rb;
  int cubic;             // 0 bilinear, 1 bicubic (cv2 a=-0.75)
  int replicate;         // border: 0 constant 0, 1 replicate (cv2 BORDER_REPLICATE)
};
hipError_t warp_batch(const WarpArgs& a, hipStream_t stream);
hipError_t cls_argmax(const uint16_t* h, int64_t ldh, const uint16_t* w, const float* bias, int M, int N, int K, int C,
                      int* idx_out, float* conf_out, hipStream_t stream);
hipError_t ctc_collapse(const int* idx, const float* conf, int B, int T, int blank, const int* tlen, int* out_ids,
                        int* out_len, float* out_conf, hipStream_t stream);
hipError_t ctc_greedy(const float* probs, int B, int T, int C, int blank, int from_logits, const int* tlen,
                      int* tmp_idx, float* tmp_conf, int* out_ids, int* out_len, float* out_conf, hipStream_t stream);

}  // namespace lumen
