// Decoder-LLM kernels (llm.hip) shared with their torch bindings (ops_llm.cpp).
//
// Paged KV cache layout (block = 64 tokens of one sequence):
//   k_cache [num_blocks, Hkv, 64, D]   token-major rows: the S^T = K Q^T MFMA A-operand
//                                      reads 16-byte pieces of K rows directly from HBM
//   v_cache [num_blocks, Hkv, D, 64]   transposed (d-major): the O^T = V^T P^T A-operand
//                                      needs 8 consecutive tokens of one d -> one 16-byte load
// Either bf16 or OCP e4m3fn (LUMEN_KV_DTYPE=fp8: half the bytes per token; 8-byte loads widened
// to bf16 fragments in registers, unit scale, values saturated to +-448 on write).
// so the decode kernel streams both straight from global memory into MFMA
// fragments with no LDS staging and no transposing reads.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lumen {

constexpr int KV_BLOCK = 64;

struct RopeKVArgs {
  uint16_t* qkv;          // [T, ld] bf16: q heads | k heads | v heads (rotated in place)
  int64_t ld;
  const int* pos;         // [T] positions
  const float* cos_sin;   // [max_pos, D/2, 2] (cos, sin)
  const int64_t* slots;   // [T] cache slot = block * 64 + offset, < 0 = do not cache; null = no cache write
  uint16_t* k_cache;
  uint16_t* v_cache;
  int T, H, Hkv, D;
  int kv_fp8;             // caches hold OCP e4m3fn bytes (unit scale, saturated) instead of bf16
};
hipError_t rope_kv(const RopeKVArgs& a, hipStream_t stream);

struct DecodeArgs {
  const uint16_t* q;      // [B, q_sb] rows; head h at h * D
  int64_t q_sb;
  const uint16_t* k_cache;
  const uint16_t* v_cache;
  const int* block_table; // [B, bt_stride]
  int bt_stride;
  const int* ctx_len;     // [B] tokens in cache (including the current one)
  uint16_t* o;            // [B, o_sb] rows; head h at h * D
  int64_t o_sb;
  float* part_o;          // [B, H, nsplit, D]   (nsplit > 1)
  float* part_ml;         // [B, H, nsplit, 2]
  int H, Hkv, nsplit, blocks_per_split;
  float scale_log2;
  // fused RoPE + cache write (decode, D = 64 / 128): q comes unrotated from the QKV projection
  // and is rotated in registers; the split owning the sequence's last block rotates the current
  // token's k and writes k / v to slots[b] before its attention loop reads that block
  const int* pos;         // [B] positions (null = q / cache already prepared by rope_kv)
  const float* cos_sin;   // [max_pos, D/2, 2]
  const int64_t* slots;   // [B]
  uint16_t* k_cache_w;    // writable views of the caches
  uint16_t* v_cache_w;
  int kv_fp8;             // caches hold e4m3fn bytes: widened to bf16 on load (cvt_scalef32_pk_bf16_fp8)
  uint32_t* split_cnt;    // [B, Hkv] zeroed tickets of the in-launch split combine (nsplit > 1; nsplit <= 32)
  // Weight prefetch into the Infinity Cache: workgroups beyond the attention grid (grid.z >= B)
  // read these bytes with default-policy loads and drop them, so the GEMV that runs next (the
  // o projection) streams its weights from the 256 MiB MALL instead of HBM while the attention
  // itself occupies only a few dozen CUs.  null / 0 = none.
  const uint8_t* pf[2];
  int64_t pf_bytes[2];
  // profiling only (tools/decode_attn_timeline.py): per-workgroup s_memrealtime stamps [B, Hkv, nsplit, 8]
  int64_t* dbg;
};
hipError_t paged_decode(const DecodeArgs& a, int B, int D, hipStream_t stream);

hipError_t rep_penalty(float* logits, int64_t ld, const int* ids, int maxn, const float* penalty, int B, int V,
                       hipStream_t stream);

// <= kUploadMax int32 values -> int64 device array, carried in the kernel arguments
constexpr int kUploadMax = 896;
struct UploadArgs {
  int32_t v[kUploadMax];
};
hipError_t upload_i64(const UploadArgs& a, int64_t* out, int n, hipStream_t stream);

}  // namespace lumen
