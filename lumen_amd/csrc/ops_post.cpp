// torch.ops.lumen.* registration of the detection / recognition post-processing
// kernels (postproc.hip): anchor/prior decode, NMS, batched affine/perspective
// warps into recogniser batches, CTC greedy decode.
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <vector>

#include "postproc.h"

namespace lumen {
hipError_t db_components(const void* prob, int is_bf16, const float* thresh, int n, int H, int W, int* lab,
                         int* out, int* count, int cap, int min_size, hipStream_t stream);
hipError_t db_quad_score(const void* prob, int is_bf16, int n, int H, int W, const float* quads, const int* img, float* score,
                         double* pre,
                         int m, hipStream_t stream);
}  // namespace lumen
#include "jpeg.h"
#include "jpeg_huff.h"

namespace {

#define CHECK_HIP2(expr)                                                                   \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "lumen HIP error: ", hipGetErrorString(_e), " @ ", #expr); \
  } while (0)

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void f32c(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), n, ": f32 contiguous GPU tensor");
}

// scores [N, P], bbox [N, P, 4], kps [N, P, 10]?; priors [P, 4]? ; cand [N, max_cand, 16]; count [N] (int32, zeroed)
void det_decode(const at::Tensor& scores, const at::Tensor& bbox, const c10::optional<at::Tensor>& kps,
                const c10::optional<at::Tensor>& priors, int64_t H, int64_t W, int64_t A, int64_t stride_,
                double thresh, const at::Tensor& img_scale, const at::Tensor& img_hw, double min_size,
                double max_size, double var0, double var1, double in_w, double in_h, at::Tensor cand,
                at::Tensor count, int64_t P, int64_t sN, int64_t sL, bool apply_sigmoid) {
  f32c(img_scale, "img_scale"); f32c(img_scale, "img_scale"); f32c(img_hw, "img_hw"); f32c(cand, "cand");
  TORCH_CHECK(count.scalar_type() == at::kInt && count.is_contiguous(), "count int32");
  lumen::DetDecodeArgs a{};
  TORCH_CHECK(scores.is_cuda() && scores.scalar_type() == at::kFloat && bbox.scalar_type() == at::kFloat, "f32 GPU");
  a.scores = scores.data_ptr<float>(); a.bbox = bbox.data_ptr<float>();
  if (kps.has_value() && kps->defined()) a.kps = kps->data_ptr<float>();
  if (priors.has_value() && priors->defined()) { f32c(*priors, "priors"); a.priors = priors->data_ptr<float>(); }
  a.N = (int)img_scale.size(0); a.P = (int)P;
  a.sN = sN; a.sL = sL; a.apply_sigmoid = apply_sigmoid ? 1 : 0;
  a.H = (int)H; a.W = (int)W; a.A = (int)A; a.stride = (int)stride_;
  a.thresh = (float)thresh; a.img_scale = img_scale.data_ptr<float>(); a.img_hw = img_hw.data_ptr<float>();
  a.min_size = (float)min_size; a.max_size = (float)max_size; a.var0 = (float)var0; a.var1 = (float)var1;
  a.in_w = (float)in_w; a.in_h = (float)in_h;
  a.cand = cand.data_ptr<float>(); a.count = count.data_ptr<int>(); a.max_cand = (int)cand.size(1);
  TORCH_CHECK(cand.size(2) == 16 && cand.size(0) == a.N, "cand [N, max_cand, 16]");
  const at::DeviceGuard g(scores.device());
  CHECK_HIP2(lumen::det_decode(a, stream()));
}

void nms(const at::Tensor& cand, const at::Tensor& count, double iou_thr, at::Tensor keep, at::Tensor keep_n) {
  f32c(cand, "cand");
  TORCH_CHECK(cand.size(1) <= 1024, "nms: at most 1024 candidates per image");
  TORCH_CHECK(keep.scalar_type() == at::kInt && keep_n.scalar_type() == at::kInt, "nms: int32 outputs");
  const at::DeviceGuard g(cand.device());
  CHECK_HIP2(lumen::nms(cand.data_ptr<float>(), count.data_ptr<int>(), (int)cand.size(0), (int)cand.size(1),
                        (float)iou_thr, (int)keep.size(1), keep.data_ptr<int>(), keep_n.data_ptr<int>(), stream()));
}

// src flat uint8; meta int64 [F, 4] (offset, h, w, out_w); minv f32 [F, 9]; out bf16 [F, OH, OW, cpad]
void warp_batch(const at::Tensor& src, const at::Tensor& meta, const at::Tensor& minv, at::Tensor out, double scale,
                double mean, double std_, bool swap_rb, bool cubic, bool replicate) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte, "warp: uint8 src");
  TORCH_CHECK(meta.is_cuda() && meta.scalar_type() == at::kLong && meta.is_contiguous() && meta.size(1) == 4, "meta");
  f32c(minv, "minv");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kBFloat16 && out.dim() == 4, "warp: out bf16 [F,H,W,C]");
  lumen::WarpArgs a{};
  a.src = src.data_ptr<uint8_t>(); a.meta = meta.data_ptr<int64_t>(); a.minv = minv.data_ptr<float>();
  a.out = reinterpret_cast<uint16_t*>(out.data_ptr());
  a.F = (int)out.size(0); a.OH = (int)out.size(1); a.OW = (int)out.size(2); a.cpad = (int)out.size(3);
  a.scale = (float)scale; a.mean = (float)mean; a.inv_std = (float)(1.0 / std_);
  a.swap_rb = swap_rb ? 1 : 0; a.cubic = cubic ? 1 : 0; a.replicate = replicate ? 1 : 0;
  const at::DeviceGuard g(src.device());
  CHECK_HIP2(lumen::warp_batch(a, stream()));
}

void ctc_greedy(const at::Tensor& probs, int64_t blank, at::Tensor out_ids, at::Tensor out_len, at::Tensor out_conf,
                bool from_logits, const c10::optional<at::Tensor>& tlen) {
  f32c(probs, "probs");
  const int B = (int)probs.size(0), T = (int)probs.size(1), C = (int)probs.size(2);
  TORCH_CHECK(out_ids.is_contiguous() && out_ids.scalar_type() == at::kInt && out_ids.numel() == (int64_t)B * T, "ids");
  TORCH_CHECK(out_len.scalar_type() == at::kInt && out_len.numel() == B, "len");
  TORCH_CHECK(out_conf.scalar_type() == at::kFloat && out_conf.numel() == B, "conf");
  const int* tl = nullptr;
  if (tlen.has_value()) {
    TORCH_CHECK(tlen->is_cuda() && tlen->scalar_type() == at::kInt && tlen->numel() == B && tlen->is_contiguous(), "tlen");
    tl = tlen->data_ptr<int>();
  }
  auto idx = at::empty({B, T}, probs.options().dtype(at::kInt));
  auto conf = at::empty({B, T}, probs.options());
  const at::DeviceGuard g(probs.device());
  CHECK_HIP2(lumen::ctc_greedy(probs.data_ptr<float>(), B, T, C, (int)blank, from_logits ? 1 : 0, tl, idx.data_ptr<int>(),
                               conf.data_ptr<float>(), out_ids.data_ptr<int>(), out_len.data_ptr<int>(),
                               out_conf.data_ptr<float>(), stream()));
}

// Recogniser classifier + CTC greedy decode without stored logits: h [B*T, K] bf16 rows, w [N, K]
// bf16, bias f32 [N] (optional), C real classes (<= N) -> out_ids [B, T] (-1 padded), out_len [B],
// out_conf [B]; top1_idx / top1_conf [B*T] receive the per-step arg-max and its probability.
void cls_ctc(const at::Tensor& h, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t C, int64_t B,
             int64_t T, int64_t blank, const c10::optional<at::Tensor>& tlen, at::Tensor top1_idx, at::Tensor top1_conf,
             at::Tensor out_ids, at::Tensor out_len, at::Tensor out_conf) {
  TORCH_CHECK(h.is_cuda() && h.scalar_type() == at::kBFloat16 && h.dim() == 2 && h.stride(1) == 1 &&
                  h.stride(0) % 8 == 0, "cls_ctc: h bf16 rows");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.size(1) == h.size(1),
              "cls_ctc: w bf16 [N, K]");
  const int64_t M = h.size(0), K = h.size(1), N = w.size(0);
  TORCH_CHECK(K == 64 || K == 128 || K == 256, "cls_ctc: K must be 64, 128 or 256");
  TORCH_CHECK(M == B * T && C >= 1 && C <= N, "cls_ctc: shapes");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() >= N, "cls_ctc: bias f32 [N]");
    bp = bias->data_ptr<float>();
  }
  TORCH_CHECK(top1_idx.scalar_type() == at::kInt && top1_idx.numel() == M && top1_idx.is_contiguous(), "top1_idx");
  TORCH_CHECK(top1_conf.scalar_type() == at::kFloat && top1_conf.numel() == M && top1_conf.is_contiguous(), "top1_conf");
  TORCH_CHECK(out_ids.scalar_type() == at::kInt && out_ids.numel() == M && out_ids.is_contiguous(), "ids");
  TORCH_CHECK(out_len.scalar_type() == at::kInt && out_len.numel() == B, "len");
  TORCH_CHECK(out_conf.scalar_type() == at::kFloat && out_conf.numel() == B, "conf");
  const int* tl = nullptr;
  if (tlen.has_value() && tlen->defined()) {
    TORCH_CHECK(tlen->is_cuda() && tlen->scalar_type() == at::kInt && tlen->numel() == B && tlen->is_contiguous(), "tlen");
    tl = tlen->data_ptr<int>();
  }
  const at::DeviceGuard g(h.device());
  CHECK_HIP2(lumen::cls_argmax(reinterpret_cast<const uint16_t*>(h.data_ptr()), h.stride(0),
                               reinterpret_cast<const uint16_t*>(w.data_ptr()), bp, (int)M, (int)N, (int)K, (int)C,
                               top1_idx.data_ptr<int>(), top1_conf.data_ptr<float>(), stream()));
  CHECK_HIP2(lumen::ctc_collapse(top1_idx.data_ptr<int>(), top1_conf.data_ptr<float>(), (int)B, (int)T, (int)blank, tl,
                                 out_ids.data_ptr<int>(), out_len.data_ptr<int>(), out_conf.data_ptr<float>(), stream()));
}

// DB post-processing on the GPU (db_post.hip): prob [n, H, W] bf16/f32, thresh f32 [n];
// lab int32 [n*H*W] workspace; out int32 [cap, 3] (root, x, y); count int32 [1]
void db_components(const at::Tensor& prob, const at::Tensor& thresh, at::Tensor lab, at::Tensor out, at::Tensor count,
                   int64_t min_size) {
  TORCH_CHECK(prob.is_cuda() && prob.is_contiguous() && prob.dim() == 3 &&
              (prob.scalar_type() == at::kBFloat16 || prob.scalar_type() == at::kFloat), "db_components: prob");
  f32c(thresh, "thresh");
  const int64_t n = prob.size(0), H = prob.size(1), W = prob.size(2);
  TORCH_CHECK(thresh.numel() == n, "db_components: thresh [n]");
  TORCH_CHECK(lab.is_cuda() && lab.scalar_type() == at::kInt && lab.numel() >= 5 * n * H * W && lab.is_contiguous(),
              "db_components: lab workspace int32 [5*n*H*W]");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.dim() == 2 && out.size(1) == 3 &&
              out.is_contiguous(), "db_components: out int32 [cap, 3]");
  TORCH_CHECK(count.is_cuda() && count.scalar_type() == at::kInt && count.numel() >= 1, "db_components: count");
  const at::DeviceGuard g(prob.device());
  CHECK_HIP2(lumen::db_components(prob.data_ptr(), prob.scalar_type() == at::kBFloat16, thresh.data_ptr<float>(),
                                  (int)n, (int)H, (int)W, lab.data_ptr<int>(), out.data_ptr<int>(),
                                  count.data_ptr<int>(), (int)out.size(0), (int)min_size, stream()));
}

void db_quad_score(const at::Tensor& prob, const at::Tensor& quads, const at::Tensor& img, at::Tensor score) {
  TORCH_CHECK(prob.is_cuda() && prob.is_contiguous() && prob.dim() == 3 &&
              (prob.scalar_type() == at::kBFloat16 || prob.scalar_type() == at::kFloat), "db_quad_score: prob");
  f32c(quads, "quads");
  f32c(score, "score");
  const int64_t m = quads.size(0);
  TORCH_CHECK(quads.dim() == 2 && quads.size(1) == 8 && score.numel() >= 3 * m,
              "db_quad_score: quads [m, 8], score f32 [3m] (scores + accumulators)");
  TORCH_CHECK(img.is_cuda() && img.scalar_type() == at::kInt && img.numel() == m && img.is_contiguous(),
              "db_quad_score: img int32 [m]");
  const at::DeviceGuard g(prob.device());
  // fp64 row prefix sums of every map (the O(rows) span sums of the score kernel)
  auto pre = at::empty({prob.size(0) * prob.size(1) * (prob.size(2) + 1)}, prob.options().dtype(at::kDouble));
  CHECK_HIP2(lumen::db_quad_score(prob.data_ptr(), prob.scalar_type() == at::kBFloat16, (int)prob.size(0),
                                  (int)prob.size(1), (int)prob.size(2), quads.data_ptr<float>(), img.data_ptr<int>(),
                                  score.data_ptr<float>(), pre.data_ptr<double>(), (int)m, stream()));
}

// JPEG pixels from entropy-decoded coefficient planes (host/jpeg_decode.cpp): coef int16 (all
// planes), qt uint16 [ncomp, 64], meta [ncomp, hmax, vmax, width, height, (h, v, bw, bh) x ncomp],
// samp uint8 scratch (sum of bw * bh * 64), out uint8 [height, width, 3].
void jpeg_reconstruct(const at::Tensor& coef, const at::Tensor& qt, at::IntArrayRef meta, at::Tensor samp,
                      at::Tensor out) {
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kShort && coef.is_contiguous(), "jpeg: coef int16");
  TORCH_CHECK(qt.is_cuda() && qt.scalar_type() == at::kShort && qt.is_contiguous(), "jpeg: qt int16 (uint16 bits)");
  TORCH_CHECK(samp.is_cuda() && samp.scalar_type() == at::kByte && samp.is_contiguous(), "jpeg: samp uint8");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kByte && out.is_contiguous(), "jpeg: out uint8");
  TORCH_CHECK(meta.size() >= 5, "jpeg: meta");
  lumen::JpegPlanes P{};
  P.ncomp = (int)meta[0];
  P.hmax = (int)meta[1];
  P.vmax = (int)meta[2];
  P.width = (int)meta[3];
  P.height = (int)meta[4];
  TORCH_CHECK((P.ncomp == 1 || P.ncomp == 3) && (int64_t)meta.size() == 5 + 4 * P.ncomp, "jpeg: meta size");
  TORCH_CHECK(out.numel() == (int64_t)P.width * P.height * 3, "jpeg: out must be [height, width, 3]");
  int64_t co = 0;
  for (int c = 0; c < P.ncomp; ++c) {
    P.h[c] = (int)meta[5 + 4 * c];
    P.v[c] = (int)meta[6 + 4 * c];
    P.bw[c] = (int)meta[7 + 4 * c];
    P.bh[c] = (int)meta[8 + 4 * c];
    TORCH_CHECK(P.bw[c] * 8 >= (P.width * P.h[c] + P.hmax - 1) / P.hmax &&
                P.bh[c] * 8 >= (P.height * P.v[c] + P.vmax - 1) / P.vmax, "jpeg: plane smaller than the image");
    P.coef_off[c] = co;
    P.samp_off[c] = co;
    co += (int64_t)P.bw[c] * P.bh[c] * 64;
  }
  TORCH_CHECK(coef.numel() >= co && samp.numel() >= co && qt.numel() >= 64 * P.ncomp, "jpeg: buffer sizes");
  P.coef = coef.data_ptr<int16_t>();
  P.qt = reinterpret_cast<const uint16_t*>(qt.data_ptr<int16_t>());
  P.samp = samp.data_ptr<uint8_t>();
  const at::DeviceGuard g(coef.device());
  CHECK_HIP2(lumen::jpeg_reconstruct(P, out.data_ptr<uint8_t>(), stream()));
}

// Batched JPEG pixels: every image of a serving batch in one IDCT and one colour launch.
// coef_all int16 / samp_all uint8: all images' planes back to back; qt_all int16 [n, 3, 64];
// meta int64 CPU [n, 21] = (coef_base, samp_base, out_off, ncomp, hmax, vmax, width, height,
// (h, v, bw, bh) x 3, qt_index); out_flat uint8 (each image [height, width, 3] at out_off);
// entries: uint8 device scratch >= n * sizeof(JpegBatchEntry); entries_host: pinned uint8 CPU staging of
// the same size, which the caller keeps (and does not rewrite) until this stream has passed the launch.
void jpeg_reconstruct_batch(const at::Tensor& coef_all, const at::Tensor& qt_all, const at::Tensor& meta,
                            at::Tensor samp_all, at::Tensor out_flat, at::Tensor entries, at::Tensor entries_host) {
  TORCH_CHECK(coef_all.is_cuda() && coef_all.scalar_type() == at::kShort && coef_all.is_contiguous(), "jpeg: coef int16");
  TORCH_CHECK(qt_all.is_cuda() && qt_all.scalar_type() == at::kShort && qt_all.is_contiguous(), "jpeg: qt int16");
  TORCH_CHECK(samp_all.is_cuda() && samp_all.scalar_type() == at::kByte && samp_all.is_contiguous(), "jpeg: samp");
  TORCH_CHECK(out_flat.is_cuda() && out_flat.scalar_type() == at::kByte && out_flat.is_contiguous(), "jpeg: out");
  TORCH_CHECK(entries.is_cuda() && entries.scalar_type() == at::kByte && entries.is_contiguous(), "jpeg: entries");
  TORCH_CHECK(!meta.is_cuda() && meta.scalar_type() == at::kLong && meta.dim() == 2 && meta.size(1) == 21 &&
              meta.is_contiguous(), "jpeg: meta int64 CPU [n, 21]");
  const int64_t n = meta.size(0);
  TORCH_CHECK(n > 0 && entries.numel() >= n * (int64_t)sizeof(lumen::JpegBatchEntry), "jpeg: entries scratch");
  TORCH_CHECK(!entries_host.is_cuda() && entries_host.is_pinned() && entries_host.scalar_type() == at::kByte &&
              entries_host.is_contiguous() && entries_host.numel() >= n * (int64_t)sizeof(lumen::JpegBatchEntry),
              "jpeg: entries_host pinned uint8 staging");
  const int64_t* m = meta.data_ptr<int64_t>();
  lumen::JpegBatchEntry* es = reinterpret_cast<lumen::JpegBatchEntry*>(entries_host.data_ptr());
  int64_t blk = 0, pix = 0;
  for (int64_t i = 0; i < n; ++i, m += 21) {
    lumen::JpegBatchEntry& e = es[i];
    lumen::JpegPlanes& P = e.P;
    P = lumen::JpegPlanes{};
    P.ncomp = (int)m[3]; P.hmax = (int)m[4]; P.vmax = (int)m[5]; P.width = (int)m[6]; P.height = (int)m[7];
    TORCH_CHECK(P.ncomp == 1 || P.ncomp == 3, "jpeg: components");
    int64_t co = 0;
    for (int c = 0; c < P.ncomp; ++c) {
      P.h[c] = (int)m[8 + 4 * c]; P.v[c] = (int)m[9 + 4 * c]; P.bw[c] = (int)m[10 + 4 * c]; P.bh[c] = (int)m[11 + 4 * c];
      TORCH_CHECK(P.bw[c] * 8 >= (P.width * P.h[c] + P.hmax - 1) / P.hmax &&
                  P.bh[c] * 8 >= (P.height * P.v[c] + P.vmax - 1) / P.vmax, "jpeg: plane smaller than the image");
      P.coef_off[c] = m[0] + co;
      P.samp_off[c] = m[1] + co;
      co += (int64_t)P.bw[c] * P.bh[c] * 64;
    }
    TORCH_CHECK(m[0] + co <= coef_all.numel() && m[1] + co <= samp_all.numel() &&
                m[2] + (int64_t)P.width * P.height * 3 <= out_flat.numel() && (m[20] + 1) * 192 <= qt_all.numel(),
                "jpeg: image ", i, " exceeds the batch buffers");
    P.coef = coef_all.data_ptr<int16_t>();
    P.qt = reinterpret_cast<const uint16_t*>(qt_all.data_ptr<int16_t>()) + m[20] * 192;
    P.samp = samp_all.data_ptr<uint8_t>();
    e.out = out_flat.data_ptr<uint8_t>() + m[2];
    e.blk0 = blk;
    e.pix0 = pix;
    blk += (co / 64 + 3) / 4 * 4;
    pix += ((int64_t)P.width * P.height + 255) / 256 * 256;
  }
  const at::DeviceGuard g(coef_all.device());
  CHECK_HIP2(hipMemcpyAsync(entries.data_ptr(), es, (size_t)n * sizeof(lumen::JpegBatchEntry), hipMemcpyHostToDevice,
                            stream()));
  CHECK_HIP2(lumen::jpeg_reconstruct_batch(reinterpret_cast<const lumen::JpegBatchEntry*>(entries.data_ptr()), (int)n,
                                           blk, pix, stream()));
}

// GPU entropy decode of n prepared JPEGs (host/jpeg_decode.cpp:lumen_jpeg_prepare_gpu).  blob: the
// device copy of the pinned upload blob_host; every job's descriptor, stream, restart table and
// coefficient range is bounds-checked on the host copy before the launch.
void jpeg_huff_decode(const at::Tensor& blob, const at::Tensor& blob_host, int64_t n, at::Tensor coefs,
                      at::Tensor err, const c10::optional<at::Tensor>& ticks) {
  TORCH_CHECK(blob.is_cuda() && blob.scalar_type() == at::kByte && blob.is_contiguous(), "jpeg_huff: blob uint8");
  TORCH_CHECK(!blob_host.is_cuda() && blob_host.scalar_type() == at::kByte && blob_host.is_contiguous() &&
              blob_host.numel() == blob.numel(), "jpeg_huff: blob_host must be the host copy of blob");
  TORCH_CHECK(coefs.is_cuda() && coefs.scalar_type() == at::kShort && coefs.is_contiguous(), "jpeg_huff: coefs int16");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt && err.numel() >= 2 * n, "jpeg_huff: err int32 [2n]");
  TORCH_CHECK(n > 0 && (int64_t)sizeof(lumen::JHuffJob) * n <= blob.numel(), "jpeg_huff: jobs");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(blob.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(coefs.data_ptr()) % 16 == 0, "jpeg_huff: 16-byte aligned buffers");
  const uint8_t* hb = blob_host.data_ptr<uint8_t>();
  const int64_t bn = blob.numel();
  int max_wg = 1, max_lanes = 1, max_window = 0;
  for (int64_t i = 0; i < n; ++i) {
    const lumen::JHuffJob& j = reinterpret_cast<const lumen::JHuffJob*>(hb)[i];
    TORCH_CHECK(j.desc_off >= 0 && j.desc_off % 16 == 0 && j.desc_off + (int64_t)sizeof(lumen::JHuffDesc) <= bn,
                "jpeg_huff: descriptor ", i, " outside the blob");
    const lumen::JHuffHead& H = reinterpret_cast<const lumen::JHuffDesc*>(hb + j.desc_off)->h;
    TORCH_CHECK(H.ncomp >= 1 && H.ncomp <= 3 && H.bpm >= 1 && H.bpm <= 10 && H.mcux >= 1 && H.total >= 0 &&
                H.nbits >= 0 && H.nwords >= 0 && H.ndc >= 1 && H.ndc <= 3 && H.nac >= 1 && H.nac <= 3,
                "jpeg_huff: descriptor ", i, " header");
    TORCH_CHECK(H.stream_off % 16 == 0 && j.desc_off + H.stream_off + 4 * (int64_t)H.nwords <= bn &&
                4 * (int64_t)H.nwords * 8 >= (int64_t)H.nbits && H.nbits < (1 << 28),
                "jpeg_huff: stream ", i, " outside the blob");
    if (H.restart_blocks == 0) {
      max_wg = std::max(max_wg, (H.nsub + lumen::kJHuffWgLanes - 1) / lumen::kJHuffWgLanes);
      max_lanes = std::max(max_lanes, H.nsub);
      max_window = std::max<int64_t>(max_window, std::min<int64_t>(H.nwords, (int64_t)lumen::kJHuffWgLanes * H.sub_bits / 32 + 256));
    }
    for (int k = 0; k < H.bpm; ++k)
      TORCH_CHECK(H.pcomp[k] >= 0 && H.pcomp[k] < H.ncomp && H.pdc[k] >= 0 && H.pdc[k] < H.ndc && H.pac[k] >= 0 &&
                  H.pac[k] < H.nac && H.px[k] >= 0 && H.px[k] < H.hh[H.pcomp[k]] && H.py[k] >= 0 &&
                  H.py[k] < H.vv[H.pcomp[k]], "jpeg_huff: MCU layout ", i);
    int64_t blocks = 0;
    for (int c = 0; c < H.ncomp; ++c) {
      TORCH_CHECK(H.hh[c] >= 1 && H.hh[c] <= 2 && H.vv[c] >= 1 && H.vv[c] <= 2 && H.bw[c] == H.mcux * H.hh[c] &&
                  H.plane_off[c] == 64 * blocks, "jpeg_huff: planes ", i);
      blocks += (int64_t)H.bw[c] * (H.total / H.bpm / H.mcux) * H.vv[c];
    }
    TORCH_CHECK(blocks == H.total && j.coef_off >= 0 && j.coef_off % 64 == 0 && j.coef_off + 64 * blocks <= coefs.numel(),
                "jpeg_huff: coefficients of image ", i, " outside the buffer");
    if (H.restart_blocks > 0) {
      TORCH_CHECK(H.nseg >= 1 && H.seg_off % 4 == 0 && j.desc_off + H.seg_off + 4 * (int64_t)H.nseg <= bn &&
                  (int64_t)H.nseg * H.restart_blocks >= H.total, "jpeg_huff: restart table ", i);
    } else {
      TORCH_CHECK(H.sub_bits >= 32 && H.sub_bits % 32 == 0 && H.nsub >= 1 && H.nsub <= lumen::kJHuffMaxLanes &&
                  (int64_t)H.nsub * H.sub_bits >= (int64_t)H.nbits, "jpeg_huff: subsequences ", i);
    }
  }
  // the workgroups of an image meet at a spin barrier: all of them must be resident at once
  int cus = 0;
  CHECK_HIP2(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, blob.get_device()));
  TORCH_CHECK(max_wg == 1 || n * max_wg <= cus, "jpeg_huff: ", n, " images x ", max_wg,
              " workgroups exceed the ", cus, " CUs (prepare with fewer lanes per image)");
  auto scratch = at::zeros({(int64_t)lumen::jpeg_huff_scratch_bytes((int)n, max_lanes)}, blob.options());
  err.zero_();
  coefs.zero_();   // the decoder writes only the nonzero coefficients
  int64_t* tp = nullptr;
  if (ticks.has_value()) {
    TORCH_CHECK(ticks->is_cuda() && ticks->scalar_type() == at::kLong && ticks->numel() >= 128 * n, "jpeg_huff: ticks");
    tp = ticks->data_ptr<int64_t>();
  }
  CHECK_HIP2(lumen::jpeg_huff_decode(blob.data_ptr<uint8_t>(), (int)n, max_wg, coefs.data_ptr<int16_t>(),
                                     err.data_ptr<int32_t>(), scratch.data_ptr(), max_lanes, max_window, tp, stream()));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(lumen, m) {
  m.def("jpeg_huff_decode(Tensor blob, Tensor blob_host, int n, Tensor(c!) coefs, Tensor(e!) err, "
        "Tensor(t!)? ticks=None) -> ()");
  m.def("jpeg_reconstruct(Tensor coef, Tensor qt, int[] meta, Tensor(s!) samp, Tensor(o!) out) -> ()");
  m.def("jpeg_reconstruct_batch(Tensor coef_all, Tensor qt_all, Tensor meta, Tensor(s!) samp_all, Tensor(o!) out_flat, "
        "Tensor(e!) entries, Tensor(h!) entries_host) -> ()");
  m.def("db_components(Tensor prob, Tensor thresh, Tensor(l!) lab, Tensor(o!) out, Tensor(c!) count, "
        "int min_size) -> ()");
  m.def("db_quad_score(Tensor prob, Tensor quads, Tensor img, Tensor(s!) score) -> ()");
  m.def("det_decode(Tensor scores, Tensor bbox, Tensor? kps, Tensor? priors, int H, int W, int A, int stride, "
        "float thresh, Tensor img_scale, Tensor img_hw, float min_size, float max_size, float var0, float var1, "
        "float in_w, float in_h, Tensor(c!) cand, Tensor(n!) count, int P, int sN, int sL, bool apply_sigmoid) -> ()");
  m.def("nms(Tensor cand, Tensor count, float iou_thr, Tensor(k!) keep, Tensor(n!) keep_n) -> ()");
  m.def("warp_batch(Tensor src, Tensor meta, Tensor minv, Tensor(o!) out, float scale, float mean, float std, "
        "bool swap_rb, bool cubic, bool replicate=False) -> ()");
  m.def("cls_ctc(Tensor h, Tensor w, Tensor? bias, int C, int B, int T, int blank, Tensor? tlen, Tensor(a!) top1_idx, "
        "Tensor(b!) top1_conf, Tensor(i!) out_ids, Tensor(l!) out_len, Tensor(c!) out_conf) -> ()");
  m.def("ctc_greedy(Tensor probs, int blank, Tensor(i!) out_ids, Tensor(l!) out_len, Tensor(c!) out_conf, "
        "bool from_logits=False, Tensor? tlen=None) -> ()");
}

TORCH_LIBRARY_IMPL(lumen, CUDA, m) {
  m.impl("jpeg_reconstruct", &jpeg_reconstruct);
  m.impl("jpeg_reconstruct_batch", &jpeg_reconstruct_batch);
  m.impl("jpeg_huff_decode", &jpeg_huff_decode);
  m.impl("det_decode", &det_decode);
  m.impl("nms", &nms);
  m.impl("warp_batch", &warp_batch);
  m.impl("ctc_greedy", &ctc_greedy);
  m.impl("cls_ctc", &cls_ctc);
  m.impl("db_components", &db_components);
  m.impl("db_quad_score", &db_quad_score);
}
