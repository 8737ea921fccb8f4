// IPC one-shot / two-shot all-reduce (comm.hip) shared with its torch bindings (ops_comm.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lumen {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 128;
constexpr int64_t AR_CTL_BYTES = 32768;
constexpr int AR_SPIN_LIMIT = 2000000;   // ~1-4 s of polling before a peer is declared missing

// control block at the start of every rank's buffer
struct ArCtl {
  uint32_t flag[2][AR_MAX_BLOCKS][AR_MAX_RANKS];   // flag[parity][block][src rank], written by the peers
  uint32_t flag2[2][AR_MAX_BLOCKS][AR_MAX_RANKS];  // two-shot phase 2 (reduced slices published)
  uint32_t epoch;                                   // this rank's call counter (ONE for every block of
                                                    // every call: all blocks agree on the parity)
  uint32_t done;                                    // blocks of the current call that finished
  uint32_t err;                                     // set when a peer never arrived
};
static_assert(sizeof(ArCtl) <= AR_CTL_BYTES, "control block too large");

// base[r] = rank r's uncached IPC buffer as mapped in THIS process (base[rank] = own buffer)
struct ArPeers {
  char* base[AR_MAX_RANKS];
};

hipError_t custom_all_reduce(const void* in, void* out, const ArPeers& peers, int rank, int world, int64_t bytes,
                             int is_bf16, int64_t cap_bytes, hipStream_t stream);
// two-shot (reduce-scatter + all-gather over the same mapped buffers): each rank reads 2 (n-1)/n of
// the message instead of (n-1) x -- the bandwidth form for prefill-sized messages
hipError_t custom_all_reduce_2shot(const void* in, void* out, const ArPeers& peers, int rank, int world,
                                   int64_t bytes, int is_bf16, int64_t cap_bytes, hipStream_t stream);

}  // namespace lumen
