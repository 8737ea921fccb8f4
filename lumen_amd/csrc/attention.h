// Fused attention forward (attention.hip) shared with its torch binding (ops.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lumen {

struct AttnArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o;
  int64_t q_sb, q_ss, q_sh;   // strides (elements) batch / seq / head
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t o_sb, o_ss, o_sh;
  const int* kv_len;          // optional per-batch valid key count
  // optional MX fp8 copy of O (attn_fwd_kernel only; the W8A8 o-projection's A operand): e4m3fn
  // [b, s, h*D] with one E8M0 byte per 32 d (os [b, s, h*D/32]); o may then be null (no bf16 O)
  uint8_t* o8; uint8_t* os;
  int64_t o8_sb, o8_ss, os_sb, os_ss;
  int Sq, Sk, H, Hkv;
  float scale_log2;           // softmax_scale * log2(e)
  int causal;                 // query i attends keys j <= i + (Sk - Sq)
};

hipError_t attn_fwd(const AttnArgs& a, int B, int D, hipStream_t stream);

}  // namespace lumen
