// Scratch buffers for split-K slabs and persistent-kernel partials, one per (device, stream, tag).
//
// Work on one stream runs in order, so a buffer private to a stream can be reused by every
// launch on it without any further synchronisation; two streams (the 2-stream micro-batched
// towers, two services in one hub process) never share one.  Growth happens outside stream
// capture only: the old buffer is freed after a hipStreamSynchronize of its stream, unless a
// captured graph has recorded its address ("pinned"), in which case it is kept alive for the
// life of the process -- a later eager call that needs more bytes on a reused stream handle
// must not free memory a graph replays into.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace lumen {

enum WorkspaceTag : int { WS_F8_SPLIT = 0, WS_PP_TAIL = 1, WS_SK_SLAB = 2, WS_SK_CNT = 3, WS_CLS_PART = 4 };

// zero: a fresh allocation is zero-filled on the stream (arrival counters)
inline void* stream_workspace(size_t bytes, hipStream_t stream, int tag, size_t min_bytes, bool zero = false) {
  struct Slot {
    void* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
  };
  static std::mutex mu;
  static std::map<std::tuple<int, hipStream_t, int>, Slot> cache;
  static std::vector<void*> kept;   // pinned buffers outgrown on their stream
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess) return nullptr;
  const bool capturing = st != hipStreamCaptureStatusNone;
  std::lock_guard<std::mutex> lk(mu);
  Slot& s = cache[std::make_tuple(dev, stream, tag)];
  if (s.cap >= bytes) {
    if (capturing) s.pinned = true;
    return s.p;
  }
  if (capturing) return nullptr;   // nothing is allocated during capture: callers fall back
  if (s.p != nullptr) {
    if (s.pinned) {
      kept.push_back(s.p);
    } else {
      (void)hipStreamSynchronize(stream);   // the stream's earlier users of the old buffer are done
      (void)hipFree(s.p);
    }
  }
  s = Slot{};
  void* p = nullptr;
  const size_t want = bytes < min_bytes ? min_bytes : bytes;
  if (hipMalloc(&p, want) != hipSuccess) return nullptr;
  if (zero && hipMemsetAsync(p, 0, want, stream) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  s.p = p;
  s.cap = want;
  return p;
}

}  // namespace lumen
