// torch.ops.lumen.* registration of the decoder-LLM kernels (llm.hip): fused RoPE +
// paged KV-cache write, paged flash-decoding attention, repetition penalty.
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include "llm.h"

namespace lumen {
uint32_t* splitk_counters(const at::Tensor& like, int64_t tiles);   // ops.cpp
}

namespace {

int64_t* g_decode_dbg = nullptr;   // profiling only (decode_set_dbg)

#define CHECK_HIP3(expr)                                                                   \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "lumen HIP error: ", hipGetErrorString(_e), " @ ", #expr); \
  } while (0)

inline hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }
inline uint16_t* bfp(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

// bf16 or float8_e4m3fn caches (both the same dtype); returns 1 for fp8
int check_cache(const at::Tensor& kc, const at::Tensor& vc, int64_t Hkv, int64_t D) {
  const bool f8 = kc.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(kc.is_cuda() && (kc.scalar_type() == at::kBFloat16 || f8) && kc.is_contiguous() && kc.dim() == 4,
              "k_cache: bf16 / float8_e4m3fn [NB, Hkv, 64, D]");
  TORCH_CHECK(vc.is_cuda() && vc.scalar_type() == kc.scalar_type() && vc.is_contiguous() && vc.dim() == 4,
              "v_cache: same dtype as k_cache, [NB, Hkv, D, 64]");
  TORCH_CHECK(kc.size(1) == Hkv && kc.size(2) == lumen::KV_BLOCK && kc.size(3) == D, "k_cache shape");
  TORCH_CHECK(vc.size(0) == kc.size(0) && vc.size(1) == Hkv && vc.size(2) == D && vc.size(3) == lumen::KV_BLOCK,
              "v_cache shape");
  return f8 ? 1 : 0;
}

// qkv [T, >= (H + 2 Hkv) D] bf16 (rotated in place); pos int32 [T]; cos_sin f32 [P, D/2, 2];
// slots int64 [T] (optional): writes rotated k / v into the paged cache.
void rope_kv(at::Tensor qkv, const at::Tensor& pos, const at::Tensor& cos_sin, const c10::optional<at::Tensor>& slots,
             at::Tensor k_cache, at::Tensor v_cache, int64_t H, int64_t Hkv, int64_t D) {
  TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 2 && qkv.stride(1) == 1, "qkv");
  TORCH_CHECK(qkv.size(1) >= (H + 2 * Hkv) * D, "qkv: too few columns");
  TORCH_CHECK(D % 2 == 0 && D <= 256, "rope: head dim");
  const int64_t T = qkv.size(0);
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kInt && pos.numel() == T && pos.is_contiguous(), "pos int32 [T]");
  TORCH_CHECK(cos_sin.is_cuda() && cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
              cos_sin.dim() == 3 && cos_sin.size(1) == D / 2 && cos_sin.size(2) == 2, "cos_sin f32 [P, D/2, 2]");
  lumen::RopeKVArgs a{};
  a.qkv = bfp(qkv); a.ld = qkv.stride(0);
  a.pos = pos.data_ptr<int>(); a.cos_sin = cos_sin.data_ptr<float>();
  if (slots.has_value() && slots->defined()) {
    TORCH_CHECK(slots->is_cuda() && slots->scalar_type() == at::kLong && slots->numel() == T && slots->is_contiguous(),
                "slots int64 [T]");
    a.kv_fp8 = check_cache(k_cache, v_cache, Hkv, D);
    a.slots = slots->data_ptr<int64_t>();
    a.k_cache = reinterpret_cast<uint16_t*>(k_cache.data_ptr()); a.v_cache = reinterpret_cast<uint16_t*>(v_cache.data_ptr());
  }
  a.T = (int)T; a.H = (int)H; a.Hkv = (int)Hkv; a.D = (int)D;
  const at::DeviceGuard g(qkv.device());
  CHECK_HIP3(lumen::rope_kv(a, cur()));
}

// q [B, >= H D] rows (bf16); block_table int32 [B, max_blocks]; ctx_len int32 [B]; out [B, >= H D] rows.
void paged_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                  const at::Tensor& block_table, const at::Tensor& ctx_len, at::Tensor out, int64_t H, int64_t Hkv,
                  double scale, int64_t nsplit, int64_t blocks_per_split, const c10::optional<at::Tensor>& part_o,
                  const c10::optional<at::Tensor>& part_ml, const c10::optional<at::Tensor>& pos,
                  const c10::optional<at::Tensor>& cos_sin, const c10::optional<at::Tensor>& slots,
                  const c10::optional<at::Tensor>& pf0, const c10::optional<at::Tensor>& pf1) {
  const int64_t D = k_cache.size(3);
  const int kv_fp8 = check_cache(k_cache, v_cache, Hkv, D);
  TORCH_CHECK(D == 32 || D == 64 || D == 128, "paged_decode: head dim 32, 64 or 128");
  TORCH_CHECK(H % Hkv == 0 && H / Hkv <= 16, "paged_decode: at most 16 query heads per kv head");
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == at::kBFloat16 && q.dim() == 2 && q.stride(1) == 1 && q.size(1) >= H * D &&
              q.stride(0) % 8 == 0, "paged_decode: q rows");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.dim() == 2 && out.stride(1) == 1 &&
              out.size(1) >= H * D, "paged_decode: out rows");
  const int64_t B = q.size(0);
  TORCH_CHECK(out.size(0) == B, "paged_decode: out batch");
  TORCH_CHECK(block_table.is_cuda() && block_table.scalar_type() == at::kInt && block_table.dim() == 2 &&
              block_table.size(0) == B && block_table.stride(1) == 1, "block_table int32 [B, max_blocks]");
  TORCH_CHECK(ctx_len.is_cuda() && ctx_len.scalar_type() == at::kInt && ctx_len.numel() == B && ctx_len.is_contiguous(),
              "ctx_len int32 [B]");
  // the kernel widens the splits to cover each sequence's own context (blocks per split =
  // max(blocks_per_split, ceil(blocks / nsplit))), so any split count covers the table
  TORCH_CHECK(nsplit >= 1 && blocks_per_split >= 1, "paged_decode: nsplit / blocks_per_split");
  lumen::DecodeArgs a{};
  a.q = bfp(q); a.q_sb = q.stride(0);
  a.k_cache = reinterpret_cast<const uint16_t*>(k_cache.data_ptr());
  a.v_cache = reinterpret_cast<const uint16_t*>(v_cache.data_ptr());
  a.kv_fp8 = kv_fp8;
  a.block_table = block_table.data_ptr<int>(); a.bt_stride = (int)block_table.stride(0);
  a.ctx_len = ctx_len.data_ptr<int>();
  a.o = bfp(out); a.o_sb = out.stride(0);
  a.H = (int)H; a.Hkv = (int)Hkv; a.nsplit = (int)nsplit; a.blocks_per_split = (int)blocks_per_split;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  if (nsplit > 1) {
    TORCH_CHECK(part_o.has_value() && part_ml.has_value(), "paged_decode: split workspace required");
    TORCH_CHECK(part_o->scalar_type() == at::kFloat && part_o->is_contiguous() && part_o->numel() >= B * H * nsplit * D,
                "part_o");
    TORCH_CHECK(part_ml->scalar_type() == at::kFloat && part_ml->is_contiguous() && part_ml->numel() >= B * H * nsplit * 2,
                "part_ml");
    a.part_o = part_o->data_ptr<float>(); a.part_ml = part_ml->data_ptr<float>();
    TORCH_CHECK(nsplit <= 32, "paged_decode: at most 32 context splits");
    a.split_cnt = lumen::splitk_counters(q, B * Hkv);
  }
  if (pos.has_value() && pos->defined()) {   // fused RoPE + current-token cache write
    TORCH_CHECK(D == 64 || D == 128, "paged_decode: fused rope needs head dim 64 or 128");
    TORCH_CHECK(q.size(1) >= (H + 2 * Hkv) * D, "paged_decode: fused rope needs the packed qkv rows");
    TORCH_CHECK(pos->is_cuda() && pos->scalar_type() == at::kInt && pos->numel() == B && pos->is_contiguous(),
                "pos int32 [B]");
    TORCH_CHECK(cos_sin.has_value() && cos_sin->is_cuda() && cos_sin->scalar_type() == at::kFloat &&
                cos_sin->is_contiguous() && cos_sin->size(-1) == 2 && cos_sin->size(-2) * 2 == D, "cos_sin f32 [P, D/2, 2]");
    TORCH_CHECK(slots.has_value() && slots->is_cuda() && slots->scalar_type() == at::kLong && slots->numel() == B &&
                slots->is_contiguous(), "slots int64 [B]");
    a.pos = pos->data_ptr<int>();
    a.cos_sin = cos_sin->data_ptr<float>();
    a.slots = slots->data_ptr<int64_t>();
    a.k_cache_w = reinterpret_cast<uint16_t*>(k_cache.data_ptr());
    a.v_cache_w = reinterpret_cast<uint16_t*>(v_cache.data_ptr());
  }
  const c10::optional<at::Tensor>* pfs[2] = {&pf0, &pf1};
  for (int r = 0; r < 2; ++r) {
    const auto& t = *pfs[r];
    if (t.has_value() && t->defined()) {
      TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->device() == q.device(), "paged_decode: prefetch tensor");
      a.pf[r] = reinterpret_cast<const uint8_t*>(t->data_ptr());
      a.pf_bytes[r] = t->numel() * t->element_size();
    }
  }
  if (B == 0) return;
  a.dbg = g_decode_dbg;
  const at::DeviceGuard g(q.device());
  CHECK_HIP3(lumen::paged_decode(a, (int)B, (int)D, cur()));
}

// profiling: per-workgroup timestamps of paged_decode into dbg [B, Hkv, nsplit, 8] int64 (empty: off)
void decode_set_dbg(const at::Tensor& dbg) {
  TORCH_CHECK(dbg.is_cuda() && dbg.scalar_type() == at::kLong && dbg.is_contiguous(), "decode_set_dbg: int64");
  g_decode_dbg = dbg.numel() > 0 ? dbg.data_ptr<int64_t>() : nullptr;
}

void rep_penalty_(at::Tensor logits, const at::Tensor& ids, const at::Tensor& penalty) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kFloat && logits.dim() == 2 && logits.stride(1) == 1,
              "rep_penalty: logits f32 [B, V]");
  const int64_t B = logits.size(0);
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kInt && ids.is_contiguous() && ids.dim() == 2 && ids.size(0) == B,
              "rep_penalty: ids int32 [B, n]");
  TORCH_CHECK(penalty.is_cuda() && penalty.scalar_type() == at::kFloat && penalty.numel() == B, "penalty f32 [B]");
  const at::DeviceGuard g(logits.device());
  CHECK_HIP3(lumen::rep_penalty(logits.data_ptr<float>(), logits.stride(0), ids.data_ptr<int>(), (int)ids.size(1),
                                penalty.data_ptr<float>(), (int)B, (int)logits.size(1), cur()));
}

// int32 CPU values -> int64 device tensor through the kernel arguments (llm.hip:upload_i64)
void upload_small(const at::Tensor& src, at::Tensor out) {
  TORCH_CHECK(!src.is_cuda() && src.scalar_type() == at::kInt && src.is_contiguous(), "upload_small: src int32 CPU");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() && out.numel() == src.numel(),
              "upload_small: out int64 like src");
  TORCH_CHECK(src.numel() <= lumen::kUploadMax, "upload_small: at most ", lumen::kUploadMax, " values");
  lumen::UploadArgs a;
  memcpy(a.v, src.data_ptr<int32_t>(), (size_t)src.numel() * sizeof(int32_t));
  const at::DeviceGuard g(out.device());
  CHECK_HIP3(lumen::upload_i64(a, out.data_ptr<int64_t>(), (int)src.numel(), cur()));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(lumen, m) {
  m.def("upload_small(Tensor src, Tensor(o!) out) -> ()");
  m.def("rope_kv(Tensor(a!) qkv, Tensor pos, Tensor cos_sin, Tensor? slots, Tensor(k!) k_cache, Tensor(v!) v_cache, "
        "int H, int Hkv, int D) -> ()");
  m.def("paged_decode(Tensor q, Tensor(k!) k_cache, Tensor(v!) v_cache, Tensor block_table, Tensor ctx_len, "
        "Tensor(o!) out, int H, int Hkv, float scale, int nsplit, int blocks_per_split, Tensor(p!)? part_o=None, "
        "Tensor(m!)? part_ml=None, Tensor? pos=None, Tensor? cos_sin=None, Tensor? slots=None, Tensor? pf0=None, "
        "Tensor? pf1=None) -> ()");
  m.def("rep_penalty_(Tensor(a!) logits, Tensor ids, Tensor penalty) -> ()");
  m.def("decode_set_dbg(Tensor dbg) -> ()");
}

TORCH_LIBRARY_IMPL(lumen, CUDA, m) {
  m.impl("rope_kv", &rope_kv);
  m.impl("paged_decode", &paged_decode);
  m.impl("rep_penalty_", &rep_penalty_);
  m.impl("upload_small", &upload_small);
  m.impl("decode_set_dbg", &decode_set_dbg);
}
