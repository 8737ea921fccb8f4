// PyTorch-ROCm operator registration for the lumen_amd HIP kernel library.
//
// Every op is registered under the `lumen` namespace (torch.ops.lumen.*) with
// a CUDA (= HIP on ROCm) implementation only: on a GPU tensor the hand-written
// gfx950 kernel runs on the current HIP stream (so the ops compose with
// torch.cuda graphs and stream semantics); CPU tensors are rejected here and
// handled by the Python reference path in lumen_amd.ops.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <ATen/DeviceGuard.h>
#include <torch/library.h>
#include <hip/hip_runtime.h>

#include <vector>
#include <mutex>
#include <unordered_map>
#include <algorithm>

#include "gemm_epi.h"
#include "attention.h"
#include "tuning.h"
#include "conv.h"

namespace lumen {
hipError_t gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C,
                     int64_t ldc, int M, int N, int K, const GemmEpi& ep, int tile, hipStream_t stream);
hipError_t gemm_w8(const uint16_t* A, int64_t lda, const uint8_t* W, int64_t ldw, const float* scale, void* C,
                   int64_t ldc, int M, int N, int K, const GemmEpi& ep, float* ws, uint32_t* cnt, int ksplit,
                   hipStream_t stream);
hipError_t gemm_f8(const uint8_t* A, int64_t lda, const float* sa, const uint8_t* W, int64_t ldw, const float* sw,
                   void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, hipStream_t stream, int splits = -1,
                   int variant = 0);
hipError_t quant_rows_fp8(const uint16_t* x, int64_t ldx, uint8_t* out, int64_t ldo, float* scale, int M, int K,
                          hipStream_t stream);
hipError_t gemm_mx(const uint8_t* A, int64_t lda, const uint8_t* a_bs, int64_t ld_bs, const uint8_t* W, int64_t ldw,
                   const float* sw, void* C, int64_t ldc, int M, int N, int K, const GemmEpi& ep, MxArgs mx,
                   hipStream_t stream, int variant);
hipError_t quant_rows_mx(const uint16_t* x, int64_t ldx, uint8_t* q8, int64_t ldq, uint8_t* qs, int64_t ldqs,
                         float* ssq, int64_t ldss, int M, int K, hipStream_t stream);
hipError_t rms_norm_quant_fp8(const uint16_t* x, int64_t ldx, const uint16_t* add, int64_t ldadd, uint16_t* resid_out,
                              int64_t ldr, const uint16_t* gamma, float eps, uint8_t* out, int64_t ldo, float* scale,
                              int M, int K, hipStream_t stream);
hipError_t gemm_skinny(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, void* C, int64_t ldc, int M,
                       int N, int K, const GemmEpi& ep, float* ws, uint32_t* cnt, int ksplit, hipStream_t stream);
int skinny_ksplit(int N, int K);
hipError_t norm_rows(const uint16_t* x, int64_t x_stride, const int64_t* row_idx, const uint16_t* add,
                     int64_t add_stride, uint16_t* resid_out, int64_t resid_stride, const uint16_t* w,
                     const uint16_t* b, void* out, int64_t out_stride, int out_f32, int rows, int D,
                     float eps, int mode, hipStream_t stream);
hipError_t l2norm_f32(float* x, int rows, int D, float eps, hipStream_t stream);
hipError_t ln_row_stats(const uint16_t* x, int64_t x_stride, float* out, int rows, int D, float eps,
                        hipStream_t stream, uint8_t* q8 = nullptr, int64_t ldq = 0, uint8_t* qs = nullptr,
                        int64_t ldqs = 0);
hipError_t cls_fill(uint16_t* x, int64_t seq_stride, const uint16_t* cls, const uint16_t* pos, int B, int D,
                    hipStream_t stream);
hipError_t embed_gather(const int64_t* ids, const uint16_t* table, const uint16_t* pos, int S, uint16_t* out,
                        int rows, int D, int64_t vocab, int64_t id_offset, hipStream_t stream);
struct ImgGeomRaw;
struct PrepArgs {
  const uint8_t* src; const ImgGeomRaw* geom; float* tmp; int tmp_h, tmp_w; void* out; int OH, OW;
  int filter; int swap_rb; float mean[3], inv_std[3]; float scale; float pad; int layout; int patch;
  int kpad; int out_bf16;
};
hipError_t image_prep(const PrepArgs& a, int B, int max_ch, int max_dw, hipStream_t stream);
hipError_t image_prep_band(const PrepArgs& a, int B, int rcap, int cwcap, int T, hipStream_t stream);
hipError_t row_topk(const float* scores, int64_t ld, int B, int N, int k, float scale, float* out_v, int* out_i,
                    float* out_lse, int index_offset, float* ws, hipStream_t stream);
int topk_chunks(int N);
}  // namespace lumen

namespace lumen {
// Split-K arrival counters of the skinny (decode) GEMMs (one per 16-column tile) and of the
// decode attention's in-launch split combine (one per sequence x kv head).  The
// last K-split workgroup of a tile to arrive reduces the slabs and resets its counter
// to 0, so the buffer is all-zero between kernels.  Kept per (device, stream): split-K
// GEMMs on different streams may run concurrently and must not share tiles.  A buffer
// first requested inside a stream capture comes from the graph's pool and its zero-fill
// is captured too (harmless on replay: the counters are zero between kernels anyway).
uint32_t* splitk_counters(const at::Tensor& like, int64_t tiles) {
  static std::mutex mu;
  static std::unordered_map<uint64_t, at::Tensor> bufs;
  const auto st = c10::hip::getCurrentHIPStream();
  const uint64_t key = ((uint64_t)(uint8_t)like.device().index() << 56) ^ (uint64_t)st.id();
  std::lock_guard<std::mutex> g(mu);
  at::Tensor& t = bufs[key];
  if (!t.defined() || t.numel() < tiles)
    t = at::zeros({std::max<int64_t>(tiles, 16384)}, like.options().dtype(at::kInt));
  return reinterpret_cast<uint32_t*>(t.data_ptr());
}
static int g_tuning[TUNE_COUNT] = {1, 1};
int tuning(int flag) { return flag >= 0 && flag < TUNE_COUNT ? g_tuning[flag] : 0; }
void set_tuning(int flag, int value) {
  if (flag >= 0 && flag < TUNE_COUNT) g_tuning[flag] = value;
}
}  // namespace lumen

namespace {

int64_t* g_gemm_dbg = nullptr;   // profiling only (gemm_set_dbg)

#define LM_CHECK_HIP(expr)                                                        \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    TORCH_CHECK(_e == hipSuccess, "lumen HIP error: ", hipGetErrorString(_e), " @ ", #expr); \
  } while (0)

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

using lumen::splitk_counters;
inline const uint16_t* bf(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
inline uint16_t* bfm(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

void check_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "lumen op: ", name, " must be a GPU tensor");
}
void check_bf16_rows(const at::Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be 2-D with unit inner stride");
  TORCH_CHECK(t.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0,
              name, " rows must be 16-byte aligned");
}

// ---------------------------------------------------------------- gemm
void gemm(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
          const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& table,
          int64_t table_period, int64_t table_offset, int64_t act, double alpha, at::Tensor out,
          int64_t out_group, int64_t out_group_stride, int64_t out_row_offset, int64_t tile,
          const c10::optional<at::Tensor>& prelu, int64_t glu) {
  check_bf16_rows(a, "a");
  check_bf16_rows(w, "w");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm: K mismatch ", w.size(1), " vs ", K);
  TORCH_CHECK(K % 64 == 0, "gemm: K must be a multiple of 64 (pad weights), got ", K);
  TORCH_CHECK(N % 16 == 0, "gemm: N must be a multiple of 16, got ", N);
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) >= (glu ? N / 2 : N), "gemm: bad out");
  TORCH_CHECK(!glu || (out.scalar_type() == at::kBFloat16 && out_group == 0 && !(residual.has_value() && residual->defined())),
              "gemm: glu epilogue writes bf16 rows without residual / row remap");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "gemm: out dtype");
  const int64_t last = M - 1;
  const int64_t need_rows = out_group > 0 ? (last / out_group) * out_group_stride + out_row_offset + last % out_group + 1 : M;
  TORCH_CHECK(out.size(0) >= need_rows, "gemm: out has ", out.size(0), " rows, needs ", need_rows);
  lumen::GemmEpi ep{};
  ep.alpha = (float)alpha;
  ep.act = (int)act;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N && bias->is_contiguous(), "gemm: bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16, "gemm: bias dtype");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (residual.has_value() && residual->defined()) {
    check_bf16_rows(*residual, "residual");
    ep.residual = bf(*residual);
    ep.ldr = residual->stride(0);
  }
  if (table.has_value() && table->defined()) {
    check_bf16_rows(*table, "table");
    TORCH_CHECK(table_period > 0, "gemm: table_period");
    ep.table = bf(*table);
    ep.ldt = table->stride(0);
    ep.table_period = (int)table_period;
    ep.table_offset = (int)table_offset;
  }
  ep.out_group = (int)out_group;
  ep.out_group_stride = out_group_stride;
  ep.out_row_offset = (int)out_row_offset;
  ep.out_f32 = out.scalar_type() == at::kFloat;
  ep.glu = (int)glu;
  if (glu) TORCH_CHECK(out.stride(0) % 8 == 0, "gemm: glu out rows must be 16-byte aligned");
  if (prelu.has_value() && prelu->defined()) {
    TORCH_CHECK(prelu->scalar_type() == at::kBFloat16 && prelu->numel() >= N && prelu->is_contiguous(), "gemm: prelu");
    ep.prelu = bf(*prelu);
  }
  ep.dbg = g_gemm_dbg;
  const at::DeviceGuard guard(a.device());
  // decode-shaped GEMMs (M <= 32): bandwidth-bound split-K kernel (tile -1 = auto, 9 = force)
  if ((tile == -1 || tile == 9) && M <= 32 && M > 0) {
    const int ks = lumen::skinny_ksplit((int)N, (int)K);
    at::Tensor ws;
    if (ks > 1) ws = at::empty({ks, M, N}, a.options().dtype(at::kFloat));   // per-split slabs, no zero-fill
    uint32_t* cnt = ks > 1 ? splitk_counters(a, (N + 15) / 16) : nullptr;
    LM_CHECK_HIP(lumen::gemm_skinny(bf(a), a.stride(0), bf(w), w.stride(0), out.data_ptr(), out.stride(0), (int)M,
                                       (int)N, (int)K, ep, ks > 1 ? ws.data_ptr<float>() : nullptr, cnt, ks,
                                       cur_stream()));
    return;
  }
  LM_CHECK_HIP(lumen::gemm_bf16(bf(a), a.stride(0), bf(w), w.stride(0), out.data_ptr(), out.stride(0),
                                   (int)M, (int)N, (int)K, ep, (int)tile, cur_stream()));
}

// LayerNorm folded into the projection: out = act(rstd * (a . w'^T) - mean * rstd * colsum(w') + bias')
// with w' = w * gamma; col_aff [2, N] fp32 = (colsum(w'), bias'), row_aff [M, 2] fp32 = (rstd, -mean * rstd)
// from ln_row_stats over the same rows of a.  Never the skinny path (it has its own folded-norm form).
void gemm_lnf(const at::Tensor& a, const at::Tensor& w, const at::Tensor& col_aff, const at::Tensor& row_aff,
              int64_t act, at::Tensor out, int64_t tile) {
  check_bf16_rows(a, "a");
  check_bf16_rows(w, "w");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 16 == 0, "gemm_lnf: shapes");
  TORCH_CHECK(col_aff.is_cuda() && col_aff.scalar_type() == at::kFloat && col_aff.is_contiguous() &&
                  col_aff.numel() == 2 * N, "gemm_lnf: col_aff must be fp32 [2, N]");
  TORCH_CHECK(row_aff.is_cuda() && row_aff.scalar_type() == at::kFloat && row_aff.is_contiguous() &&
                  row_aff.numel() >= 2 * M, "gemm_lnf: row_aff must be fp32 [M, 2]");
  check_bf16_rows(out, "out");
  TORCH_CHECK(out.size(0) >= M && out.size(1) >= N, "gemm_lnf: out");
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.act = (int)act;
  ep.row_aff = row_aff.data_ptr<float>();
  ep.col_aff = col_aff.data_ptr<float>();
  ep.dbg = g_gemm_dbg;
  const at::DeviceGuard guard(a.device());
  LM_CHECK_HIP(lumen::gemm_bf16(bf(a), a.stride(0), bf(w), w.stride(0), out.data_ptr(), out.stride(0),
                                   (int)M, (int)N, (int)K, ep, (int)tile, cur_stream()));
}

static int64_t check_planes(const at::Tensor& t, int64_t planes, int64_t M, const char* name);
static void check_f8_rows(const at::Tensor& t, const char* name);

// q8 / qs (optional): the raw rows as MX fp8 + E8M0 planes (the LN-folded gemm_mx operand)
void ln_row_stats(const at::Tensor& x, at::Tensor out, double eps, const c10::optional<at::Tensor>& q8,
                  const c10::optional<at::Tensor>& qs) {
  check_bf16_rows(x, "x");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() >= 2 * x.size(0),
              "ln_row_stats: out must be fp32 [rows, 2]");
  uint8_t* qp = nullptr;
  uint8_t* sp = nullptr;
  int64_t ldq = 0, ldqs = 0;
  if (q8.has_value() && q8->defined()) {
    const int64_t M = x.size(0), D = x.size(1);
    check_f8_rows(*q8, "ln_row_stats: q8");
    TORCH_CHECK(q8->size(0) >= M && q8->size(1) == D && D % 128 == 0 && qs.has_value() && qs->defined(),
                "ln_row_stats: q8 [rows, D] (D % 128 == 0) needs qs");
    ldqs = check_planes(*qs, D / 128, M, "ln_row_stats: qs");
    qp = reinterpret_cast<uint8_t*>(q8->data_ptr());
    ldq = q8->stride(0);
    sp = qs->data_ptr<uint8_t>();
  }
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::ln_row_stats(bf(x), x.stride(0), out.data_ptr<float>(), (int)x.size(0), (int)x.size(1),
                                      (float)eps, cur_stream(), qp, ldq, sp, ldqs));
}

// ---------------------------------------------------------------- fp8 (e4m3fn) weight GEMM
// out = epi((a @ w8^T) * scale[n]): bias -> act | SwiGLU -> + residual.  w8 [N, K] float8_e4m3fn.
void gemm_w8(const at::Tensor& a, const at::Tensor& w8, const at::Tensor& scale, const c10::optional<at::Tensor>& bias,
             const c10::optional<at::Tensor>& residual, int64_t act, at::Tensor out, int64_t glu) {
  check_bf16_rows(a, "a");
  TORCH_CHECK(w8.is_cuda() && w8.scalar_type() == at::kFloat8_e4m3fn && w8.dim() == 2 && w8.stride(1) == 1 &&
              w8.stride(0) % 16 == 0, "gemm_w8: w8 must be float8_e4m3fn [N, K] with 16-byte aligned rows");
  const int64_t M = a.size(0), K = a.size(1), N = w8.size(0);
  TORCH_CHECK(w8.size(1) == K && K % 64 == 0 && N % 16 == 0, "gemm_w8: K % 64 == 0, N % 16 == 0");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() == N && scale.is_contiguous(),
              "gemm_w8: scale f32 [N]");
  check_gpu(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "gemm_w8: out dtype");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(0) >= M && out.size(1) >= (glu ? N / 2 : N), "gemm_w8: out");
  TORCH_CHECK(!glu || out.scalar_type() == at::kBFloat16, "gemm_w8: glu writes bf16");
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.act = (int)act;
  ep.glu = (int)glu;
  ep.out_f32 = out.scalar_type() == at::kFloat;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N && bias->is_contiguous() &&
                (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16), "gemm_w8: bias");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (residual.has_value() && residual->defined()) {
    check_bf16_rows(*residual, "residual");
    ep.residual = bf(*residual);
    ep.ldr = residual->stride(0);
  }
  const at::DeviceGuard guard(a.device());
  int ks = 1;
  at::Tensor ws;
  uint32_t* cnt = nullptr;
  if (M <= 32) {
    ks = lumen::w8_dec_plan((int)M, (int)N, (int)K).ks;
    if (ks > 1) {
      ws = at::empty({ks, M, N}, a.options().dtype(at::kFloat));
      cnt = splitk_counters(a, (N + 15) / 16);
    }
  }
  LM_CHECK_HIP(lumen::gemm_w8(bf(a), a.stride(0), reinterpret_cast<const uint8_t*>(w8.data_ptr()), w8.stride(0),
                                 scale.data_ptr<float>(), out.data_ptr(), out.stride(0), (int)M, (int)N, (int)K, ep,
                                 ks > 1 ? ws.data_ptr<float>() : nullptr, cnt, ks, cur_stream()));
}

// ---------------------------------------------------------------- decode GEMM (norm folding)
// out = epi(rstd(a) * (a @ w^T) [* scale]) for M <= 32 rows on the skinny decode kernels.
// norm = 1: rows are scaled by rstd = rsqrt(mean(a^2) + eps) before the bias (RMSNorm with
// its gamma folded into w, see LLM.fold_norms), rstd from ssq_in [M, tiles] (sums of squares
// the producing GEMM wrote) or from a itself.  ssq_out [M, N/16]: this GEMM's epilogue writes
// the per-16-column sums of squares of its stored bf16 rows (the residual stream), for the
// next norm-folded GEMM.  w bf16 [N, K], or float8_e4m3fn with fp32 per-row scale.
void gemm_dec(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& scale,
              const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& residual, at::Tensor out,
              int64_t glu, int64_t norm, double eps, const c10::optional<at::Tensor>& ssq_in,
              const c10::optional<at::Tensor>& ssq_out) {
  check_bf16_rows(a, "a");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(M > 0 && M <= 32, "gemm_dec: decode rows only (1..32)");
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && w.stride(1) == 1 && N % 16 == 0, "gemm_dec: w [N, K], N % 16 == 0");
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(0) >= M && out.size(1) >= (glu ? N / 2 : N),
              "gemm_dec: out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || (out.scalar_type() == at::kFloat && !glu), "gemm_dec: out dtype");
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.glu = (int)glu;
  ep.out_f32 = out.scalar_type() == at::kFloat;
  ep.norm = (int)norm;
  ep.norm_eps = (float)eps;
  if (norm && ssq_in.has_value() && ssq_in->defined()) {
    TORCH_CHECK(ssq_in->is_cuda() && ssq_in->scalar_type() == at::kFloat && ssq_in->dim() == 2 &&
                ssq_in->size(0) >= M && ssq_in->is_contiguous(), "gemm_dec: ssq_in f32 [>= M, tiles]");
    TORCH_CHECK(ssq_in->size(1) * 16 == K, "gemm_dec: ssq_in tiles * 16 must equal K");
    ep.ssq_in = ssq_in->data_ptr<float>();
    ep.ssq_tiles = (int)ssq_in->size(1);
  }
  if (ssq_out.has_value() && ssq_out->defined()) {
    TORCH_CHECK(!norm || !ep.ssq_in, "gemm_dec: ssq_in and ssq_out share the tile count field");
    TORCH_CHECK(!glu && out.scalar_type() == at::kBFloat16, "gemm_dec: ssq_out needs a bf16 non-GLU output");
    TORCH_CHECK(ssq_out->is_cuda() && ssq_out->scalar_type() == at::kFloat && ssq_out->dim() == 2 &&
                ssq_out->size(0) >= M && ssq_out->size(1) * 16 == N && ssq_out->is_contiguous(),
                "gemm_dec: ssq_out f32 [>= M, N / 16]");
    ep.ssq_out = ssq_out->data_ptr<float>();
    ep.ssq_tiles = (int)ssq_out->size(1);
  }
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N && bias->is_contiguous() &&
                (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16), "gemm_dec: bias");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (residual.has_value() && residual->defined()) {
    check_bf16_rows(*residual, "residual");
    ep.residual = bf(*residual);
    ep.ldr = residual->stride(0);
  }
  const at::DeviceGuard guard(a.device());
  const bool is_f8 = w.scalar_type() == at::kFloat8_e4m3fn;
  const int ks = is_f8 ? lumen::w8_dec_plan((int)M, (int)N, (int)K).ks : lumen::skinny_ksplit((int)N, (int)K);
  at::Tensor ws;
  if (ks > 1) ws = at::empty({ks, M, N}, a.options().dtype(at::kFloat));
  uint32_t* cnt = ks > 1 ? splitk_counters(a, (N + 15) / 16) : nullptr;
  float* wsp = ks > 1 ? ws.data_ptr<float>() : nullptr;
  if (w.scalar_type() == at::kFloat8_e4m3fn) {
    TORCH_CHECK(scale.has_value() && scale->defined() && scale->scalar_type() == at::kFloat && scale->numel() == N,
                "gemm_dec: fp8 weights need scale f32 [N]");
    TORCH_CHECK(K % 64 == 0 && w.stride(0) % 16 == 0, "gemm_dec: fp8 K % 64");
    LM_CHECK_HIP(lumen::gemm_w8(bf(a), a.stride(0), reinterpret_cast<const uint8_t*>(w.data_ptr()), w.stride(0),
                                   scale->data_ptr<float>(), out.data_ptr(), out.stride(0), (int)M, (int)N, (int)K, ep,
                                   wsp, cnt, ks, cur_stream()));
  } else {
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && K % 32 == 0, "gemm_dec: bf16 weights, K % 32");
    LM_CHECK_HIP(lumen::gemm_skinny(bf(a), a.stride(0), bf(w), w.stride(0), out.data_ptr(), out.stride(0), (int)M,
                                       (int)N, (int)K, ep, wsp, cnt, ks, cur_stream()));
  }
}

// ---------------------------------------------------------------- fp8 x fp8 (W8A8) GEMM
// out = epi((a8 @ w8^T) * sa[m] * sw[n]): fp32 bias | SwiGLU -> + residual; a8 [M, K] and
// w8 [N, K] float8_e4m3fn, sa [M] / sw [N] fp32 (per-token / per-channel scales).
static void check_f8_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat8_e4m3fn && t.dim() == 2 && t.stride(1) == 1 &&
              t.stride(0) % 16 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              ": float8_e4m3fn [rows, K] with 16-byte aligned rows");
}
void gemm_f8(const at::Tensor& a8, const at::Tensor& sa, const at::Tensor& w8, const at::Tensor& sw,
             const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& residual, at::Tensor out,
             int64_t glu, int64_t splits, int64_t variant) {
  check_f8_rows(a8, "gemm_f8: a8");
  check_f8_rows(w8, "gemm_f8: w8");
  const int64_t M = a8.size(0), K = a8.size(1), N = w8.size(0);
  TORCH_CHECK(w8.size(1) == K && K % 128 == 0 && N % 16 == 0, "gemm_f8: K % 128 == 0, N % 16 == 0");
  TORCH_CHECK(variant >= 0 && variant <= 18, "gemm_f8: variant 0..18");
  TORCH_CHECK(sa.is_cuda() && sa.scalar_type() == at::kFloat && sa.numel() >= M && sa.is_contiguous(),
              "gemm_f8: sa f32 [M]");
  TORCH_CHECK(sw.is_cuda() && sw.scalar_type() == at::kFloat && sw.numel() == N && sw.is_contiguous(),
              "gemm_f8: sw f32 [N]");
  check_gpu(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "gemm_f8: out dtype");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(0) >= M && out.size(1) >= (glu ? N / 2 : N),
              "gemm_f8: out");
  TORCH_CHECK(!glu || out.scalar_type() == at::kBFloat16, "gemm_f8: glu writes bf16");
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.glu = (int)glu;
  ep.out_f32 = out.scalar_type() == at::kFloat;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N && bias->is_contiguous() &&
                (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16), "gemm_f8: bias");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (residual.has_value() && residual->defined()) {
    check_bf16_rows(*residual, "residual");
    ep.residual = bf(*residual);
    ep.ldr = residual->stride(0);
  }
  const at::DeviceGuard guard(a8.device());
  LM_CHECK_HIP(lumen::gemm_f8(reinterpret_cast<const uint8_t*>(a8.data_ptr()), a8.stride(0), sa.data_ptr<float>(),
                                 reinterpret_cast<const uint8_t*>(w8.data_ptr()), w8.stride(0), sw.data_ptr<float>(),
                                 out.data_ptr(), out.stride(0), (int)M, (int)N, (int)K, ep, cur_stream(),
                                 (int)splits, (int)variant));
}

// ---------------------------------------------------------------- MX W8A8 (block-scaled activations)
// MX scale planes: uint8 [K/128, >= M, 4] (byte of row m, 32-column block b at [b/4][m][b%4]); returns
// the plane stride in bytes
static int64_t check_planes(const at::Tensor& t, int64_t planes, int64_t M, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kByte && t.dim() == 3 && t.size(0) == planes && t.size(1) >= M &&
              t.size(2) == 4 && t.stride(2) == 1 && t.stride(1) == 4 && (t.stride(0) % 4 == 0 || t.size(0) == 1) &&
              reinterpret_cast<uintptr_t>(t.data_ptr()) % 4 == 0, name, ": uint8 scale planes [", planes,
              ", >= ", M, ", 4]");
  return t.size(0) == 1 ? std::max<int64_t>(t.stride(0), 4 * t.size(1)) : t.stride(0);   // size-1 dim: any stride
}
static void check_f32_rows(const at::Tensor& t, int64_t M, int64_t cols, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= M &&
              t.size(1) >= cols, name, ": f32 [rows, >= ", cols, "]");
}

// out = epi(rstd? * (A . W^T) * sw[n]) with A = a8 [M, K] e4m3fn x 2^(a_bs - 127) per 32 columns;
// optional MX fp8 copy of the output (q8 / qs), per-(row, 128-column) sums of squares (ssq_out),
// RMSNorm row scale from the producer's sums of squares (ssq_in [M, K/128], norm_eps).
void gemm_mx(const at::Tensor& a8, const at::Tensor& a_bs, const at::Tensor& w8, const at::Tensor& sw,
             const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& residual,
             const c10::optional<at::Tensor>& out, int64_t glu, const c10::optional<at::Tensor>& ssq_in, double norm_eps,
             const c10::optional<at::Tensor>& q8, const c10::optional<at::Tensor>& qs,
             const c10::optional<at::Tensor>& ssq_out, int64_t variant, int64_t act,
             const c10::optional<at::Tensor>& row_aff, const c10::optional<at::Tensor>& col_aff) {
  check_f8_rows(a8, "gemm_mx: a8");
  check_f8_rows(w8, "gemm_mx: w8");
  const int64_t M = a8.size(0), K = a8.size(1), N = w8.size(0);
  TORCH_CHECK(w8.size(1) == K && K % 128 == 0 && N % 128 == 0, "gemm_mx: K % 128 == 0, N % 128 == 0");
  TORCH_CHECK(variant >= 0 && variant <= 15 && variant != 6 && variant != 7 && variant != 8 && variant != 14,
              "gemm_mx: variant");
  const int64_t ld_bs = check_planes(a_bs, K / 128, M, "gemm_mx: a_bs");
  TORCH_CHECK(sw.is_cuda() && sw.scalar_type() == at::kFloat && sw.numel() == N && sw.is_contiguous(),
              "gemm_mx: sw f32 [N]");
  const int64_t NO = glu ? N / 2 : N;
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.glu = (int)glu;
  lumen::MxArgs mx{};
  void* cp = nullptr;
  int64_t ldc = 0;
  if (out.has_value() && out->defined()) {
    check_bf16_rows(*out, "out");
    TORCH_CHECK(out->size(0) >= M && out->size(1) >= NO, "gemm_mx: out [M, N (or N/2 with glu)] bf16");
    cp = out->data_ptr();
    ldc = out->stride(0);
  } else {
    TORCH_CHECK(q8.has_value() && q8->defined() && !(residual.has_value() && residual->defined()),
                "gemm_mx: out may only be omitted with q8 (and no residual)");
    mx.skip_c = 1;
  }
  ep.act = (int)act;
  TORCH_CHECK(!(glu && act), "gemm_mx: act with glu");
  if (row_aff.has_value() && row_aff->defined()) {
    TORCH_CHECK(!glu && !(bias.has_value() && bias->defined()) && col_aff.has_value() && col_aff->defined(),
                "gemm_mx: LN fold (row_aff) takes col_aff, no bias / glu");
    TORCH_CHECK(row_aff->is_cuda() && row_aff->scalar_type() == at::kFloat && row_aff->is_contiguous() &&
                row_aff->numel() >= 2 * M, "gemm_mx: row_aff fp32 [M, 2]");
    TORCH_CHECK(col_aff->is_cuda() && col_aff->scalar_type() == at::kFloat && col_aff->is_contiguous() &&
                col_aff->numel() == 2 * N, "gemm_mx: col_aff fp32 [2, N]");
    ep.row_aff = row_aff->data_ptr<float>();
    ep.col_aff = col_aff->data_ptr<float>();
  }
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N && bias->is_contiguous() &&
                (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16), "gemm_mx: bias");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(!glu, "gemm_mx: residual with glu");
    check_bf16_rows(*residual, "residual");
    ep.residual = bf(*residual);
    ep.ldr = residual->stride(0);
  }
  if (ssq_in.has_value() && ssq_in->defined()) {
    check_f32_rows(*ssq_in, M, K / 128, "gemm_mx: ssq_in");
    TORCH_CHECK(ssq_in->size(1) == K / 128 && ssq_in->is_contiguous(), "gemm_mx: ssq_in [M, K/128] contiguous");
    mx.ssq_in = ssq_in->data_ptr<float>();
    mx.ssq_in_tiles = (int)(K / 128);
    mx.norm_eps = (float)norm_eps;
  }
  if (q8.has_value() && q8->defined()) {
    check_f8_rows(*q8, "gemm_mx: q8");
    TORCH_CHECK(q8->size(0) >= M && q8->size(1) == NO, "gemm_mx: q8 [M, out columns]");
    TORCH_CHECK(qs.has_value() && qs->defined() && NO % 128 == 0, "gemm_mx: q8 needs qs (output width % 128)");
    mx.ldqs = check_planes(*qs, NO / 128, M, "gemm_mx: qs");
    mx.q8 = reinterpret_cast<uint8_t*>(q8->data_ptr());
    mx.ldq = q8->stride(0);
    mx.qs = qs->data_ptr<uint8_t>();
  }
  if (ssq_out.has_value() && ssq_out->defined()) {
    TORCH_CHECK(!glu && cp != nullptr, "gemm_mx: ssq_out needs the bf16 output");
    check_f32_rows(*ssq_out, M, N / 128, "gemm_mx: ssq_out");
    TORCH_CHECK(ssq_out->size(1) == N / 128 && ssq_out->is_contiguous(), "gemm_mx: ssq_out [M, N/128] contiguous");
    mx.ssq_out = ssq_out->data_ptr<float>();
    mx.ssq_out_tiles = (int)(N / 128);
  }
  const at::DeviceGuard guard(a8.device());
  LM_CHECK_HIP(lumen::gemm_mx(reinterpret_cast<const uint8_t*>(a8.data_ptr()), a8.stride(0), a_bs.data_ptr<uint8_t>(),
                                 ld_bs, reinterpret_cast<const uint8_t*>(w8.data_ptr()), w8.stride(0),
                                 sw.data_ptr<float>(), cp, ldc, (int)M, (int)N, (int)K, ep, mx, cur_stream(),
                                 (int)variant));
}

// bf16 rows -> MX fp8 + E8M0 per 32 columns (+ per-(row, 128-column) sums of squares)
void quant_rows_mx(const at::Tensor& x, at::Tensor q8, at::Tensor qs, const c10::optional<at::Tensor>& ssq) {
  check_bf16_rows(x, "x");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 128 == 0 && x.stride(0) % 8 == 0, "quant_rows_mx: K % 128 == 0, 16-byte aligned rows");
  check_f8_rows(q8, "quant_rows_mx: q8");
  TORCH_CHECK(q8.size(0) >= M && q8.size(1) == K, "quant_rows_mx: q8 shape");
  const int64_t ldqs = check_planes(qs, K / 128, M, "quant_rows_mx: qs");
  float* sp = nullptr;
  int64_t lds = 0;
  if (ssq.has_value() && ssq->defined()) {
    check_f32_rows(*ssq, M, K / 128, "quant_rows_mx: ssq");
    sp = ssq->data_ptr<float>();
    lds = ssq->stride(0);
  }
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::quant_rows_mx(bf(x), x.stride(0), reinterpret_cast<uint8_t*>(q8.data_ptr()), q8.stride(0),
                                       qs.data_ptr<uint8_t>(), ldqs, sp, lds, (int)M, (int)K, cur_stream()));
}

// per-token fp8 quantisation of bf16 rows: out8 [M, K] e4m3fn, scale [M] = amax / 448
void quant_rows_fp8(const at::Tensor& x, at::Tensor out8, at::Tensor scale) {
  check_bf16_rows(x, "x");
  check_f8_rows(out8, "quant_rows_fp8: out8");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(out8.size(0) >= M && out8.size(1) == K && K % 8 == 0, "quant_rows_fp8: shapes");
  TORCH_CHECK(x.stride(0) % 8 == 0, "quant_rows_fp8: x rows must be 16-byte aligned");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= M && scale.is_contiguous(),
              "quant_rows_fp8: scale f32 [M]");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::quant_rows_fp8(bf(x), x.stride(0), reinterpret_cast<uint8_t*>(out8.data_ptr()), out8.stride(0),
                                        scale.data_ptr<float>(), (int)M, (int)K, cur_stream()));
}

// RMSNorm(x [+ add] -> resid_out) fused with per-token fp8 quantisation of the normed rows
void rms_norm_quant_fp8(const at::Tensor& x, const c10::optional<at::Tensor>& add,
                        const c10::optional<at::Tensor>& resid_out, const at::Tensor& gamma, double eps, at::Tensor out8,
                        at::Tensor scale) {
  check_bf16_rows(x, "x");
  check_f8_rows(out8, "rms_norm_quant_fp8: out8");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 8 == 0 && K <= 16384 && x.stride(0) % 8 == 0, "rms_norm_quant_fp8: K % 8 == 0, K <= 16384");
  TORCH_CHECK(out8.size(0) >= M && out8.size(1) == K, "rms_norm_quant_fp8: out8 shape");
  TORCH_CHECK(gamma.is_cuda() && gamma.scalar_type() == at::kBFloat16 && gamma.numel() == K && gamma.is_contiguous(),
              "rms_norm_quant_fp8: gamma bf16 [K]");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= M && scale.is_contiguous(),
              "rms_norm_quant_fp8: scale f32 [M]");
  const uint16_t* ap = nullptr;
  int64_t lda = 0;
  if (add.has_value() && add->defined()) {
    check_bf16_rows(*add, "add");
    TORCH_CHECK(add->size(0) >= M && add->size(1) == K && add->stride(0) % 8 == 0, "rms_norm_quant_fp8: add");
    ap = bf(*add);
    lda = add->stride(0);
  }
  uint16_t* rp = nullptr;
  int64_t ldr = 0;
  if (resid_out.has_value() && resid_out->defined()) {
    check_bf16_rows(*resid_out, "resid_out");
    TORCH_CHECK(resid_out->size(0) >= M && resid_out->size(1) == K && resid_out->stride(0) % 8 == 0,
                "rms_norm_quant_fp8: resid_out");
    rp = const_cast<uint16_t*>(bf(*resid_out));
    ldr = resid_out->stride(0);
  }
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::rms_norm_quant_fp8(bf(x), x.stride(0), ap, lda, rp, ldr, bf(gamma), (float)eps,
                                            reinterpret_cast<uint8_t*>(out8.data_ptr()), out8.stride(0),
                                            scale.data_ptr<float>(), (int)M, (int)K, cur_stream()));
}

// in-process A/B switch of a kernel variant (csrc/tuning.h); returns the previous value
int64_t set_tuning_op(int64_t flag, int64_t value) {
  const int prev = lumen::tuning((int)flag);
  lumen::set_tuning((int)flag, (int)value);
  return prev;
}

// profiling: route per-workgroup timestamps of the gemm / gemm_lnf ops into dbg [wg, 4] (empty: off)
void gemm_set_dbg(const at::Tensor& dbg) {
  TORCH_CHECK(dbg.is_cuda() && dbg.scalar_type() == at::kLong && dbg.is_contiguous(), "gemm_set_dbg: int64");
  g_gemm_dbg = dbg.numel() > 0 ? dbg.data_ptr<int64_t>() : nullptr;
}

// profiling: plain GEMM with per-workgroup timestamps (start, prologue, K-loop, epilogue) in dbg [wg, 4]
void gemm_probe(const at::Tensor& a, const at::Tensor& w, at::Tensor out, at::Tensor dbg, int64_t tile) {
  check_bf16_rows(a, "a");
  check_bf16_rows(w, "w");
  TORCH_CHECK(dbg.is_cuda() && dbg.scalar_type() == at::kLong && dbg.is_contiguous(), "gemm_probe: dbg int64");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  TORCH_CHECK(dbg.numel() >= ((M + 255) / 256) * ((N + 255) / 256) * 4, "gemm_probe: dbg too small");
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.dbg = dbg.data_ptr<int64_t>();
  const at::DeviceGuard guard(a.device());
  LM_CHECK_HIP(lumen::gemm_bf16(bf(a), a.stride(0), bf(w), w.stride(0), out.data_ptr(), out.stride(0),
                                   (int)M, (int)N, (int)K, ep, (int)tile, cur_stream()));
}

// ---------------------------------------------------------------- norms
void norm(const at::Tensor& x, const c10::optional<at::Tensor>& row_idx, const c10::optional<at::Tensor>& add,
          const c10::optional<at::Tensor>& resid_out, const at::Tensor& w, const c10::optional<at::Tensor>& b,
          at::Tensor out, double eps, int64_t mode) {
  check_bf16_rows(x, "x");
  const int64_t D = x.size(1);
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "norm: D must be a multiple of 8 and <= 8192");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() == D, "norm: weight");
  const int64_t rows = out.size(0);
  const int64_t* idx = nullptr;
  if (row_idx.has_value() && row_idx->defined()) {
    TORCH_CHECK(row_idx->scalar_type() == at::kLong && row_idx->numel() == rows, "norm: row_idx");
    idx = row_idx->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(x.size(0) >= rows, "norm: rows");
  }
  const uint16_t* addp = nullptr; int64_t add_stride = 0;
  if (add.has_value() && add->defined()) { check_bf16_rows(*add, "add"); addp = bf(*add); add_stride = add->stride(0); }
  uint16_t* rp = nullptr; int64_t r_stride = 0;
  if (resid_out.has_value() && resid_out->defined()) { check_bf16_rows(*resid_out, "resid_out"); rp = bfm(*resid_out); r_stride = resid_out->stride(0); }
  const uint16_t* bp = nullptr;
  if (b.has_value() && b->defined()) { TORCH_CHECK(b->scalar_type() == at::kBFloat16 && b->numel() == D); bp = bf(*b); }
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) == D, "norm: out");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::norm_rows(bf(x), x.stride(0), idx, addp, add_stride, rp, r_stride, bf(w), bp,
                                   out.data_ptr(), out.stride(0), out.scalar_type() == at::kFloat, (int)rows,
                                   (int)D, (float)eps, (int)mode, cur_stream()));
}

void l2norm_(at::Tensor x, double eps) {
  check_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 2, "l2norm_: f32 2-D contiguous");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::l2norm_f32(x.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (float)eps, cur_stream()));
}

void cls_fill(at::Tensor x, const at::Tensor& cls, const at::Tensor& pos, int64_t seq) {
  check_bf16_rows(x, "x");
  const int64_t D = x.size(1);
  TORCH_CHECK(x.size(0) % seq == 0, "cls_fill: rows % seq");
  TORCH_CHECK(cls.numel() == D && pos.size(-1) == D, "cls_fill: shapes");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::cls_fill(bfm(x), seq * x.stride(0), bf(cls), bf(pos), (int)(x.size(0) / seq), (int)D,
                                  cur_stream()));
}

void embed_gather(const at::Tensor& ids, const at::Tensor& table, const c10::optional<at::Tensor>& pos,
                  at::Tensor out, int64_t seq, int64_t id_offset) {
  check_gpu(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "embed_gather: ids int64");
  TORCH_CHECK(table.scalar_type() == at::kBFloat16 && table.is_contiguous(), "embed_gather: table");
  const int64_t D = table.size(1);
  TORCH_CHECK(out.is_contiguous() && out.numel() == ids.numel() * D, "embed_gather: out");
  const uint16_t* pp = nullptr;
  if (pos.has_value() && pos->defined()) { TORCH_CHECK(pos->is_contiguous() && pos->size(-1) == D); pp = bf(*pos); }
  const at::DeviceGuard guard(ids.device());
  LM_CHECK_HIP(lumen::embed_gather(ids.data_ptr<int64_t>(), bf(table), pp, (int)seq, bfm(out), (int)ids.numel(),
                                      (int)D, table.size(0), id_offset, cur_stream()));
}

// ---------------------------------------------------------------- attention
// q: [B, Sq, H, D], k/v: [B, Sk, Hkv, D], o: [B, Sq, H, D]  (any strides, unit inner)
void attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor o,
               const c10::optional<at::Tensor>& kv_len, double scale, bool causal) {
  for (auto* t : {&q, &k, &v}) {
    check_gpu(*t, "qkv");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 4 && t->stride(3) == 1, "attention: bf16 4-D");
  }
  TORCH_CHECK(o.scalar_type() == at::kBFloat16 && o.dim() == 4 && o.stride(3) == 1, "attention: out");
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3);
  const int64_t Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && v.size(1) == Sk && v.size(2) == Hkv, "attention: kv shape");
  TORCH_CHECK(H % Hkv == 0, "attention: H % Hkv");
  TORCH_CHECK(D == 32 || D == 64 || D == 128, "attention: head dim must be 32/64/128");
  lumen::AttnArgs a{};
  a.q = bf(q); a.k = bf(k); a.v = bf(v); a.o = bfm(o);
  a.q_sb = q.stride(0); a.q_ss = q.stride(1); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_ss = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_ss = v.stride(1); a.v_sh = v.stride(2);
  a.o_sb = o.stride(0); a.o_ss = o.stride(1); a.o_sh = o.stride(2);
  if (kv_len.has_value() && kv_len->defined()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == B, "attention: kv_len int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.Sq = (int)Sq; a.Sk = (int)Sk; a.H = (int)H; a.Hkv = (int)Hkv;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.causal = causal ? 1 : 0;
  const at::DeviceGuard guard(q.device());
  LM_CHECK_HIP(lumen::attn_fwd(a, (int)B, (int)D, cur_stream()));
}

// attention with an MX fp8 output (the W8A8 o-projection's operand): o8 e4m3fn [B, Sq, H*D] (or
// [Sq, H*D] when B == 1), os uint8 scale planes [B, H*D/128, Sq, 4] (or 3-D when B == 1); o (bf16
// [B, Sq, H, D]) optional.
void attention_mx(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const c10::optional<at::Tensor>& o,
                  at::Tensor o8, at::Tensor os, const c10::optional<at::Tensor>& kv_len, double scale, bool causal) {
  for (auto* t : {&q, &k, &v}) {
    check_gpu(*t, "qkv");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 4 && t->stride(3) == 1, "attention_mx: bf16 4-D");
  }
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3);
  const int64_t Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && v.size(1) == Sk && v.size(2) == Hkv && H % Hkv == 0,
              "attention_mx: kv shape");
  TORCH_CHECK(D == 64 || D == 128, "attention_mx: head dim 64 / 128");
  TORCH_CHECK(o8.is_cuda() && o8.scalar_type() == at::kFloat8_e4m3fn && o8.stride(-1) == 1 &&
              (o8.dim() == 3 || (o8.dim() == 2 && o8.size(0) >= B * Sq)) && o8.size(-1) >= H * D &&
              o8.size(-2) >= Sq && o8.stride(-2) % 4 == 0, "attention_mx: o8 e4m3fn [B, Sq, >= H*D] or [B*Sq, >= H*D]");
  TORCH_CHECK((H * D) % 128 == 0, "attention_mx: H*D % 128");
  TORCH_CHECK(os.is_cuda() && os.scalar_type() == at::kByte && (os.dim() == 3 || (os.dim() == 4)) &&
              os.size(-3) == H * D / 128 && os.size(-2) >= Sq && os.size(-1) == 4 && os.stride(-1) == 1 &&
              os.stride(-2) == 4 && os.stride(-3) % 4 == 0 && (os.dim() == 4 || os.size(-2) >= B * Sq) &&
              reinterpret_cast<uintptr_t>(os.data_ptr()) % 4 == 0,
              "attention_mx: os uint8 scale planes [(B,) H*D/128, >= Sq, 4]");
  lumen::AttnArgs a{};
  a.q = bf(q); a.k = bf(k); a.v = bf(v);
  a.q_sb = q.stride(0); a.q_ss = q.stride(1); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_ss = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_ss = v.stride(1); a.v_sh = v.stride(2);
  if (o.has_value() && o->defined()) {
    TORCH_CHECK(o->scalar_type() == at::kBFloat16 && o->dim() == 4 && o->stride(3) == 1, "attention_mx: out");
    a.o = bfm(*o);
    a.o_sb = o->stride(0); a.o_ss = o->stride(1); a.o_sh = o->stride(2);
  }
  a.o8 = reinterpret_cast<uint8_t*>(o8.data_ptr());
  a.os = os.data_ptr<uint8_t>();
  a.o8_sb = o8.dim() == 3 ? o8.stride(0) : Sq * o8.stride(0); a.o8_ss = o8.stride(-2);   // 2-D: rows b-major
  a.os_sb = os.dim() == 4 ? os.stride(0) : Sq * 4; a.os_ss = os.stride(-3);
  if (kv_len.has_value() && kv_len->defined()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == B, "attention_mx: kv_len int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.Sq = (int)Sq; a.Sk = (int)Sk; a.H = (int)H; a.Hkv = (int)Hkv;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.causal = causal ? 1 : 0;
  const at::DeviceGuard guard(q.device());
  LM_CHECK_HIP(lumen::attn_fwd(a, (int)B, (int)D, cur_stream()));
}

// ---------------------------------------------------------------- image prep
void image_prep2(const at::Tensor& src, const at::Tensor& geom, at::Tensor out, at::Tensor tmp, int64_t out_h,
                 int64_t out_w, int64_t filter, bool swap_rb, std::vector<double> mean, std::vector<double> std_,
                 double scale, double pad, int64_t layout, int64_t patch, int64_t kpad, int64_t max_ch,
                 int64_t max_dw) {
  check_gpu(src, "src");
  check_gpu(out, "out");
  TORCH_CHECK(src.scalar_type() == at::kByte, "image_prep: uint8 src");
  TORCH_CHECK(geom.is_cuda() && geom.scalar_type() == at::kLong && geom.dim() == 2 && geom.size(1) == 11 &&
                  geom.is_contiguous(), "image_prep: geom int64 [B, 11] on device");
  TORCH_CHECK(tmp.scalar_type() == at::kFloat && tmp.dim() == 4 && tmp.size(3) == 3 && tmp.is_contiguous(),
              "image_prep: tmp f32 [B, H, W, 3]");
  TORCH_CHECK(mean.size() == 3 && std_.size() == 3, "image_prep: mean/std");
  TORCH_CHECK(out.is_contiguous(), "image_prep: out contiguous");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "image_prep: out dtype");
  const int64_t B = geom.size(0);
  lumen::PrepArgs a{};
  a.src = src.data_ptr<uint8_t>();
  a.geom = reinterpret_cast<const lumen::ImgGeomRaw*>(geom.data_ptr<int64_t>());
  a.tmp = tmp.data_ptr<float>();
  a.tmp_h = (int)tmp.size(1); a.tmp_w = (int)tmp.size(2);
  TORCH_CHECK(tmp.size(0) >= B && a.tmp_h >= max_ch && a.tmp_w >= max_dw, "image_prep: tmp too small");
  a.out = out.data_ptr();
  a.out_bf16 = out.scalar_type() == at::kBFloat16;
  a.OH = (int)out_h; a.OW = (int)out_w;
  if (layout == 2) {
    TORCH_CHECK(patch > 0 && out_h % patch == 0 && out_w % patch == 0, "image_prep: patch grid");
    TORCH_CHECK(kpad >= 3 * patch * patch, "image_prep: kpad");
    TORCH_CHECK(out.numel() == B * (out_h / patch) * (out_w / patch) * kpad, "image_prep: patch out size");
  } else {
    TORCH_CHECK(out.numel() == B * (layout == 3 ? 8 : 3) * out_h * out_w, "image_prep: out size");
  }
  a.filter = (int)filter; a.swap_rb = swap_rb ? 1 : 0;
  for (int i = 0; i < 3; ++i) { a.mean[i] = (float)mean[i]; a.inv_std[i] = (float)(1.0 / std_[i]); }
  a.scale = (float)scale; a.pad = (float)pad;
  a.layout = (int)layout; a.patch = (int)patch; a.kpad = (int)kpad;
  const at::DeviceGuard guard(src.device());
  LM_CHECK_HIP(lumen::image_prep(a, (int)B, (int)max_ch, (int)max_dw, cur_stream()));
}

// ViT patch rows, PIL filters: the fused per-band kernel (csrc/image.hip prep_band_kernel); rcap / taps are
// the host's bounds over the batch (ops.image_prep)
void image_prep_band(const at::Tensor& src, const at::Tensor& geom, at::Tensor out, int64_t out_h, int64_t out_w,
                     int64_t filter, bool swap_rb, std::vector<double> mean, std::vector<double> std_, double scale,
                     double pad, int64_t patch, int64_t kpad, int64_t rcap, int64_t cwcap, int64_t taps) {
  check_gpu(src, "src");
  check_gpu(out, "out");
  TORCH_CHECK(src.scalar_type() == at::kByte, "image_prep_band: uint8 src");
  TORCH_CHECK(geom.is_cuda() && geom.scalar_type() == at::kLong && geom.dim() == 2 && geom.size(1) == 11 &&
                  geom.is_contiguous(), "image_prep_band: geom int64 [B, 11] on device");
  TORCH_CHECK(mean.size() == 3 && std_.size() == 3, "image_prep_band: mean/std");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kBFloat16, "image_prep_band: bf16 contiguous out");
  TORCH_CHECK(filter == 0 || filter == 1, "image_prep_band: PIL filters only");
  TORCH_CHECK(patch > 0 && out_h % patch == 0 && out_w % patch == 0 && kpad >= 3 * patch * patch && kpad % 8 == 0,
              "image_prep_band: patch grid / kpad");
  const int64_t B = geom.size(0);
  TORCH_CHECK(out.numel() == B * (out_h / patch) * (out_w / patch) * kpad, "image_prep_band: patch out size");
  lumen::PrepArgs a{};
  a.src = src.data_ptr<uint8_t>();
  a.geom = reinterpret_cast<const lumen::ImgGeomRaw*>(geom.data_ptr<int64_t>());
  a.out = out.data_ptr();
  a.out_bf16 = 1;
  a.OH = (int)out_h; a.OW = (int)out_w;
  a.filter = (int)filter; a.swap_rb = swap_rb ? 1 : 0;
  for (int i = 0; i < 3; ++i) { a.mean[i] = (float)mean[i]; a.inv_std[i] = (float)(1.0 / std_[i]); }
  a.scale = (float)scale; a.pad = (float)pad;
  a.layout = 2; a.patch = (int)patch; a.kpad = (int)kpad;
  const at::DeviceGuard guard(src.device());
  LM_CHECK_HIP(lumen::image_prep_band(a, (int)B, (int)rcap, (int)cwcap, (int)taps, cur_stream()));
}

// ---------------------------------------------------------------- top-k
void row_topk(const at::Tensor& scores, int64_t k, double scale, at::Tensor out_v, at::Tensor out_i,
              const c10::optional<at::Tensor>& out_lse, int64_t index_offset) {
  check_gpu(scores, "scores");
  TORCH_CHECK(scores.scalar_type() == at::kFloat && scores.dim() == 2 && scores.stride(1) == 1, "row_topk: f32 [B, N]");
  TORCH_CHECK(k >= 1 && k <= 64 && k <= scores.size(1), "row_topk: 1 <= k <= min(64, N)");
  const int64_t B = scores.size(0);
  TORCH_CHECK(out_v.scalar_type() == at::kFloat && out_v.is_contiguous() && out_v.numel() == B * k, "row_topk: out_v");
  TORCH_CHECK(out_i.scalar_type() == at::kInt && out_i.is_contiguous() && out_i.numel() == B * k, "row_topk: out_i");
  float* lse = nullptr;
  if (out_lse.has_value() && out_lse->defined()) {
    TORCH_CHECK(out_lse->scalar_type() == at::kFloat && out_lse->numel() == B, "row_topk: out_lse");
    lse = out_lse->data_ptr<float>();
  }
  const at::DeviceGuard guard(scores.device());
  const int nch = lumen::topk_chunks((int)scores.size(1));
  at::Tensor ws;
  if (nch > 1) ws = at::empty({B * nch * (2 * k + 2)}, scores.options());
  LM_CHECK_HIP(lumen::row_topk(scores.data_ptr<float>(), scores.stride(0), (int)B, (int)scores.size(1), (int)k,
                                  (float)scale, out_v.data_ptr<float>(), out_i.data_ptr<int>(), lse, (int)index_offset,
                                  nch > 1 ? ws.data_ptr<float>() : nullptr, cur_stream()));
}

// ---------------------------------------------------------------- convolution / CNN support (NHWC)
static int64_t pixel_stride(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, name, ": NHWC 4-D with unit channel stride");
  const int64_t ld = t.stride(2);
  TORCH_CHECK(t.stride(1) == t.size(2) * ld && t.stride(0) == t.size(1) * t.stride(1), name,
              ": pixels must be uniformly strided (channel-slice views allowed)");
  TORCH_CHECK(ld % 8 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0, name, ": 16-byte aligned pixels");
  return ld;
}

void conv2d(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
            const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& prelu, int64_t act,
            std::vector<int64_t> stride, std::vector<int64_t> padding, std::vector<int64_t> dilation, at::Tensor out,
            int64_t tile, int64_t post_act, const c10::optional<at::Tensor>& aff_scale,
            const c10::optional<at::Tensor>& aff_shift, const c10::optional<at::Tensor>& aff_out) {
  check_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv2d: bf16");
  const int64_t ldx = pixel_stride(x, "x");
  TORCH_CHECK(w.dim() == 4 && w.is_contiguous(), "conv2d: w [Cout, KH, KW, Cin] contiguous");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const int64_t Cout = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(w.size(3) == Cin && Cin % 8 == 0, "conv2d: Cin mismatch or not a multiple of 8");
  TORCH_CHECK(Cout % 16 == 0, "conv2d: Cout must be a multiple of 16");
  TORCH_CHECK(stride.size() == 2 && (padding.size() == 2 || padding.size() == 4) && dilation.size() == 2,
              "conv2d: 2-D params (padding [ph, pw] or ONNX-style [top, left, bottom, right])");
  // asymmetric padding: the kernels pad top / left explicitly; bottom / right follow from Ho / Wo
  // (taps past the input edge read zeros either way)
  const int64_t pb = padding.size() == 4 ? padding[2] : padding[0], pr = padding.size() == 4 ? padding[3] : padding[1];
  const int64_t Ho = (H + padding[0] + pb - dilation[0] * (KH - 1) - 1) / stride[0] + 1;
  const int64_t Wo = (W + padding[1] + pr - dilation[1] * (KW - 1) - 1) / stride[1] + 1;
  const int64_t ldo = pixel_stride(out, "out");
  TORCH_CHECK(out.size(0) == N && out.size(1) == Ho && out.size(2) == Wo && out.size(3) == Cout, "conv2d: out shape");
  lumen::GemmEpi ep{};
  ep.alpha = 1.f;
  ep.act = (int)act;
  ep.out_f32 = out.scalar_type() == at::kFloat;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() == Cout && bias->is_contiguous(), "conv2d: bias");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (residual.has_value() && residual->defined()) {
    ep.ldr = pixel_stride(*residual, "residual");
    ep.residual = bf(*residual);
  }
  if (prelu.has_value() && prelu->defined()) {
    TORCH_CHECK(prelu->scalar_type() == at::kBFloat16 && prelu->numel() == Cout, "conv2d: prelu");
    ep.prelu = bf(*prelu);
  }
  TORCH_CHECK(post_act == 0 || post_act == 3, "conv2d: post_act supports none / relu");
  ep.post_act = (int)post_act;
  if (aff_scale.has_value() && aff_scale->defined()) {
    // output affine (next layer's pre-conv BatchNorm): fp32 [Cout] scale / shift, bf16 output
    TORCH_CHECK(aff_shift.has_value() && aff_shift->defined(), "conv2d: aff_scale needs aff_shift");
    for (const at::Tensor* t : {&*aff_scale, &*aff_shift})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == Cout &&
                      (reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) == 0,
                  "conv2d: aff scale / shift fp32 [Cout] contiguous, 16-byte aligned");
    TORCH_CHECK(out.scalar_type() == at::kBFloat16, "conv2d: output affine needs a bf16 output");
    ep.aff_s = aff_scale->data_ptr<float>();
    ep.aff_t = aff_shift->data_ptr<float>();
    if (aff_out.has_value() && aff_out->defined()) {
      TORCH_CHECK(aff_out->scalar_type() == at::kBFloat16 && aff_out->size(0) == N && aff_out->size(1) == Ho &&
                      aff_out->size(2) == Wo && aff_out->size(3) == Cout, "conv2d: aff_out shape / dtype");
      ep.ld_aff = pixel_stride(*aff_out, "aff_out");
      ep.aff_out = reinterpret_cast<uint16_t*>(aff_out->data_ptr());
    }
  }
  lumen::ConvArgs a{};
  a.x = bf(x); a.w = bf(w); a.out = out.data_ptr(); a.ldx = ldx; a.ldo = ldo;
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.Cin = (int)Cin; a.Cout = (int)Cout; a.KH = (int)KH; a.KW = (int)KW;
  a.sh = (int)stride[0]; a.sw = (int)stride[1]; a.ph = (int)padding[0]; a.pw = (int)padding[1];
  a.dh = (int)dilation[0]; a.dw = (int)dilation[1]; a.Ho = (int)Ho; a.Wo = (int)Wo;
  ep.dbg = g_gemm_dbg;
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::conv2d_igemm(a, ep, (int)tile, cur_stream()));
}

void conv2d_dw(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act,
               std::vector<int64_t> stride, std::vector<int64_t> padding, std::vector<int64_t> dilation,
               at::Tensor out) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.dim() == 4 && x.scalar_type() == at::kBFloat16, "conv2d_dw: x NHWC contiguous");
  TORCH_CHECK(w.is_contiguous() && w.dim() == 3, "conv2d_dw: w [KH, KW, C]");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && w.size(2) == C, "conv2d_dw: C % 8 / mismatch");
  TORCH_CHECK(out.is_contiguous() && out.dim() == 4 && out.size(3) == C, "conv2d_dw: out");
  const void* bp = nullptr; int bf32 = 0;
  if (bias.has_value() && bias->defined()) { bp = bias->data_ptr(); bf32 = bias->scalar_type() == at::kFloat; }
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::conv2d_depthwise(bf(x), bf(w), bp, bf32, out.data_ptr(), (int)N, (int)H, (int)W, (int)C,
                                          (int)w.size(0), (int)w.size(1), (int)stride[0], (int)stride[1],
                                          (int)padding[0], (int)padding[1], (int)dilation[0], (int)dilation[1],
                                          (int)out.size(1), (int)out.size(2), (int)act,
                                          out.scalar_type() == at::kFloat, cur_stream()));
}

void channel_affine(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift, at::Tensor out,
                    int64_t act, const c10::optional<at::Tensor>& prelu) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.scalar_type() == at::kBFloat16, "channel_affine: x/out");
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && scale.numel() == C && shift.numel() == C && scale.scalar_type() == at::kFloat, "channel_affine: C");
  const uint16_t* pp = nullptr;
  if (prelu.has_value() && prelu->defined()) pp = bf(*prelu);
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::channel_affine(bf(x), scale.data_ptr<float>(), shift.data_ptr<float>(), bfm(out),
                                        x.numel() / C, (int)C, (int)act, pp, cur_stream()));
}

void pool2d(const at::Tensor& x, at::Tensor out, std::vector<int64_t> kernel, std::vector<int64_t> stride,
            std::vector<int64_t> padding, bool is_max) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.dim() == 4 && x.size(3) % 8 == 0, "pool2d: NHWC");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::pool2d(bf(x), bfm(out), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                                (int)kernel[0], (int)kernel[1], (int)stride[0], (int)stride[1], (int)padding[0],
                                (int)padding[1], (int)out.size(1), (int)out.size(2), is_max ? 1 : 0, cur_stream()));
}

void global_avgpool(const at::Tensor& x, at::Tensor out) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.dim() == 4 && out.scalar_type() == at::kFloat, "global_avgpool");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::global_avgpool(bf(x), out.data_ptr<float>(), (int)x.size(0), (int)(x.size(1) * x.size(2)),
                                        (int)x.size(3), cur_stream()));
}

void upsample_add(const at::Tensor& x, const c10::optional<at::Tensor>& add, at::Tensor out, int64_t factor) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.dim() == 4 && x.size(3) % 8 == 0, "upsample_add: x");
  const int64_t ldo = pixel_stride(out, "out");
  const uint16_t* ap = nullptr;
  if (add.has_value() && add->defined()) { TORCH_CHECK(add->is_contiguous()); ap = bf(*add); }
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::upsample_add(bf(x), ap, bfm(out), (int)x.size(0), (int)x.size(1), (int)x.size(2),
                                      (int)x.size(3), (int)factor, ldo, cur_stream()));
}

void channel_scale_(at::Tensor x, const at::Tensor& s) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.dim() == 4 && s.scalar_type() == at::kFloat, "channel_scale_");
  const at::DeviceGuard guard(x.device());
  LM_CHECK_HIP(lumen::channel_scale(bfm(x), s.data_ptr<float>(), (int)x.size(0), (int)(x.size(1) * x.size(2)),
                                       (int)x.size(3), cur_stream()));
}

void pixel_shuffle_up(const at::Tensor& y, at::Tensor out, int64_t factor) {
  check_gpu(y, "y");
  TORCH_CHECK(y.is_contiguous() && out.is_contiguous(), "pixel_shuffle_up");
  const int64_t C = out.size(3);
  const at::DeviceGuard guard(y.device());
  LM_CHECK_HIP(lumen::pixel_shuffle_up(bf(y), bfm(out), (int)y.size(0), (int)y.size(1), (int)y.size(2), (int)C,
                                          (int)factor, cur_stream()));
}

// DBNet head tail (csrc/conv.hip db_head_up): h [N, H4, W4, C] bf16 -> prob [N, 4*H4, 4*W4] fp32
void db_head_up(const at::Tensor& h, const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2p,
                const at::Tensor& b2, at::Tensor out) {
  check_gpu(h, "h");
  TORCH_CHECK(h.dim() == 4 && h.is_contiguous() && h.scalar_type() == at::kBFloat16, "db_head_up: h NHWC bf16");
  const int64_t N = h.size(0), H4 = h.size(1), W4 = h.size(2), C = h.size(3);
  TORCH_CHECK(C == 16 || C == 32, "db_head_up: C must be 16 or 32");
  TORCH_CHECK(w1.is_contiguous() && w1.scalar_type() == at::kBFloat16 && w1.size(0) == 4 * C && w1.size(1) == C,
              "db_head_up: w1 [4C, C] bf16");
  TORCH_CHECK(b1.is_contiguous() && b1.scalar_type() == at::kFloat && b1.numel() == 4 * C, "db_head_up: b1 [4C] fp32");
  TORCH_CHECK(w2p.is_contiguous() && w2p.scalar_type() == at::kBFloat16 && w2p.numel() == 4 * 64 * 8,
              "db_head_up: w2p [4, 64, 8] bf16");
  TORCH_CHECK(b2.is_contiguous() && b2.scalar_type() == at::kFloat && b2.numel() >= 4, "db_head_up: b2 [4] fp32");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kFloat && out.dim() == 3 && out.size(0) == N &&
              out.size(1) == 4 * H4 && out.size(2) == 4 * W4, "db_head_up: out [N, 4*H4, 4*W4] fp32");
  for (const at::Tensor* t : {&w1, &b1, &w2p, &b2, (const at::Tensor*)&out})
    TORCH_CHECK(t->device() == h.device(), "db_head_up: device");
  const at::DeviceGuard guard(h.device());
  LM_CHECK_HIP(lumen::db_head_up(bf(h), bf(w1), b1.data_ptr<float>(), bf(w2p), b2.data_ptr<float>(),
                                 out.data_ptr<float>(), (int)N, (int)H4, (int)W4, (int)C, cur_stream()));
}

}  // namespace

TORCH_LIBRARY(lumen, m) {
  m.def("gemm(Tensor a, Tensor w, Tensor? bias, Tensor? residual, Tensor? table, int table_period, "
        "int table_offset, int act, float alpha, Tensor(o!) out, int out_group, int out_group_stride, "
        "int out_row_offset, int tile, Tensor? prelu=None, int glu=0) -> ()");
  m.def("norm(Tensor x, Tensor? row_idx, Tensor? add, Tensor(r!)? resid_out, Tensor w, Tensor? b, "
        "Tensor(o!) out, float eps, int mode) -> ()");
  m.def("l2norm_(Tensor(a!) x, float eps) -> ()");
  m.def("gemm_lnf(Tensor a, Tensor w, Tensor col_aff, Tensor row_aff, int act, Tensor(o!) out, int tile) -> ()");
  m.def("ln_row_stats(Tensor x, Tensor(o!) out, float eps, Tensor(q!)? q8=None, Tensor(s!)? qs=None) -> ()");
  m.def("gemm_probe(Tensor a, Tensor w, Tensor(o!) out, Tensor(d!) dbg, int tile) -> ()");
  m.def("gemm_set_dbg(Tensor dbg) -> ()");
  m.def("set_tuning(int flag, int value) -> int", &set_tuning_op);
  m.def("gemm_w8(Tensor a, Tensor w8, Tensor scale, Tensor? bias, Tensor? residual, int act, Tensor(o!) out, "
        "int glu) -> ()");
  m.def("gemm_dec(Tensor a, Tensor w, Tensor? scale, Tensor? bias, Tensor? residual, Tensor(o!) out, int glu, "
        "int norm, float eps, Tensor? ssq_in, Tensor(s!)? ssq_out) -> ()");
  m.def("gemm_f8(Tensor a8, Tensor sa, Tensor w8, Tensor sw, Tensor? bias, Tensor? residual, Tensor(o!) out, "
        "int glu, int splits=-1, int variant=0) -> ()");
  m.def("quant_rows_fp8(Tensor x, Tensor(o!) out8, Tensor(s!) scale) -> ()");
  m.def("gemm_mx(Tensor a8, Tensor a_bs, Tensor w8, Tensor sw, Tensor? bias, Tensor? residual, Tensor(o!)? out, "
        "int glu, Tensor? ssq_in, float norm_eps, Tensor(q!)? q8, Tensor(s!)? qs, Tensor(t!)? ssq_out, int variant, "
        "int act=0, Tensor? row_aff=None, Tensor? col_aff=None) -> ()");
  m.def("quant_rows_mx(Tensor x, Tensor(q!) q8, Tensor(s!) qs, Tensor(t!)? ssq) -> ()");
  m.def("rms_norm_quant_fp8(Tensor x, Tensor? add, Tensor(r!)? resid_out, Tensor gamma, float eps, Tensor(o!) out8, "
        "Tensor(s!) scale) -> ()");
  m.def("cls_fill(Tensor(a!) x, Tensor cls, Tensor pos, int seq) -> ()");
  m.def("embed_gather(Tensor ids, Tensor table, Tensor? pos, Tensor(o!) out, int seq, int id_offset) -> ()");
  m.def("attention(Tensor q, Tensor k, Tensor v, Tensor(o!) o, Tensor? kv_len, float scale, bool causal) -> ()");
  m.def("attention_mx(Tensor q, Tensor k, Tensor v, Tensor(o!)? o, Tensor(q8!) o8, Tensor(s!) os, Tensor? kv_len, "
        "float scale, bool causal) -> ()");
  m.def("image_prep(Tensor src, Tensor geom, Tensor(o!) out, Tensor(t!) tmp, int out_h, int out_w, int filter, "
        "bool swap_rb, float[] mean, float[] std, float scale, float pad, int layout, int patch, int kpad, "
        "int max_ch, int max_dw) -> ()");
  m.def("image_prep_band(Tensor src, Tensor geom, Tensor(o!) out, int out_h, int out_w, int filter, bool swap_rb, "
        "float[] mean, float[] std, float scale, float pad, int patch, int kpad, int rcap, int cwcap, int taps) -> ()");
  m.def("row_topk(Tensor scores, int k, float scale, Tensor(v!) out_v, Tensor(i!) out_i, Tensor(l!)? out_lse, "
        "int index_offset) -> ()");
  m.def("conv2d(Tensor x, Tensor w, Tensor? bias, Tensor? residual, Tensor? prelu, int act, int[] stride, "
        "int[] padding, int[] dilation, Tensor(o!) out, int tile, int post_act=0, Tensor? aff_scale=None, "
        "Tensor? aff_shift=None, Tensor(b!)? aff_out=None) -> ()");
  m.def("conv2d_dw(Tensor x, Tensor w, Tensor? bias, int act, int[] stride, int[] padding, int[] dilation, "
        "Tensor(o!) out) -> ()");
  m.def("channel_affine(Tensor x, Tensor scale, Tensor shift, Tensor(o!) out, int act, Tensor? prelu) -> ()");
  m.def("pool2d(Tensor x, Tensor(o!) out, int[] kernel, int[] stride, int[] padding, bool is_max) -> ()");
  m.def("global_avgpool(Tensor x, Tensor(o!) out) -> ()");
  m.def("upsample_add(Tensor x, Tensor? add, Tensor(o!) out, int factor) -> ()");
  m.def("channel_scale_(Tensor(a!) x, Tensor s) -> ()");
  m.def("pixel_shuffle_up(Tensor y, Tensor(o!) out, int factor) -> ()");
  m.def("db_head_up(Tensor h, Tensor w1, Tensor b1, Tensor w2p, Tensor b2, Tensor(o!) out) -> ()");
}

TORCH_LIBRARY_IMPL(lumen, CUDA, m) {
  m.impl("gemm", &gemm);
  m.impl("norm", &norm);
  m.impl("l2norm_", &l2norm_);
  m.impl("gemm_lnf", &gemm_lnf);
  m.impl("ln_row_stats", &ln_row_stats);
  m.impl("gemm_probe", &gemm_probe);
  m.impl("gemm_set_dbg", &gemm_set_dbg);
  m.impl("gemm_w8", &gemm_w8);
  m.impl("gemm_f8", &gemm_f8);
  m.impl("gemm_dec", &gemm_dec);
  m.impl("quant_rows_fp8", &quant_rows_fp8);
  m.impl("gemm_mx", &gemm_mx);
  m.impl("quant_rows_mx", &quant_rows_mx);
  m.impl("rms_norm_quant_fp8", &rms_norm_quant_fp8);
  m.impl("cls_fill", &cls_fill);
  m.impl("embed_gather", &embed_gather);
  m.impl("attention", &attention);
  m.impl("attention_mx", &attention_mx);
  m.impl("image_prep", &image_prep2);
  m.impl("image_prep_band", &image_prep_band);
  m.impl("row_topk", &row_topk);
  m.impl("conv2d", &conv2d);
  m.impl("conv2d_dw", &conv2d_dw);
  m.impl("channel_affine", &channel_affine);
  m.impl("pool2d", &pool2d);
  m.impl("global_avgpool", &global_avgpool);
  m.impl("upsample_add", &upsample_add);
  m.impl("channel_scale_", &channel_scale_);
  m.impl("pixel_shuffle_up", &pixel_shuffle_up);
  m.impl("db_head_up", &db_head_up);
}
