// Paged-KV block manager (host runtime, C ABI for ctypes).
//
// The VLM engine keeps every sequence's KV in 64-token blocks of one large
// per-layer pool on the GPU (layouts in ../llm.h).  This manager owns the
// block free list, per-sequence block tables and reference counts (prefix
// sharing between sequences forked from a common prompt); the Python engine
// asks it for capacity before each step and copies the tables it returns
// into the device block-table tensor.  Thread-safe (one mutex): the engine
// thread allocates while request threads may query stats.
#include <algorithm>
#include <cstdint>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kBlock = 64;

struct Seq {
  std::vector<int> blocks;
  int tokens = 0;
};

struct Manager {
  explicit Manager(int n) : ref(n, 0) {
    free.reserve(n);
    for (int i = n - 1; i >= 0; --i) free.push_back(i);
  }
  std::mutex mu;
  std::vector<int> free;
  std::vector<int> ref;
  std::unordered_map<int64_t, Seq> seqs;

  int take() {
    const int b = free.back();
    free.pop_back();
    ref[b] = 1;
    return b;
  }
  void drop(int b) {
    if (--ref[b] == 0) free.push_back(b);
  }
};

}  // namespace

extern "C" {

void* lumen_kv_create(int num_blocks) { return num_blocks > 0 ? new Manager(num_blocks) : nullptr; }

void lumen_kv_destroy(void* h) { delete static_cast<Manager*>(h); }

int lumen_kv_free_blocks(void* h) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  return (int)m->free.size();
}

int lumen_kv_num_seqs(void* h) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  return (int)m->seqs.size();
}

// Grow sequence `seq` to hold `n_tokens` tokens.  Returns the number of blocks the
// sequence now owns, or -1 (and changes nothing) when the pool cannot supply them.
int lumen_kv_reserve(void* h, int64_t seq, int n_tokens) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  Seq& s = m->seqs[seq];
  const int need = (n_tokens + kBlock - 1) / kBlock - (int)s.blocks.size();
  if (need > (int)m->free.size()) {
    if (s.blocks.empty()) m->seqs.erase(seq);
    return -1;
  }
  for (int i = 0; i < need; ++i) s.blocks.push_back(m->take());
  s.tokens = std::max(s.tokens, n_tokens);
  return (int)s.blocks.size();
}

// Would reserving n_tokens for `seq` succeed?  (admission control)
int lumen_kv_can_reserve(void* h, int64_t seq, int n_tokens) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->seqs.find(seq);
  const int have = it == m->seqs.end() ? 0 : (int)it->second.blocks.size();
  return (n_tokens + kBlock - 1) / kBlock - have <= (int)m->free.size();
}

// Copy up to `max` block ids of `seq` into `out`; returns the block count (-1: unknown seq).
int lumen_kv_table(void* h, int64_t seq, int* out, int max) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->seqs.find(seq);
  if (it == m->seqs.end()) return -1;
  const auto& b = it->second.blocks;
  const int n = std::min<int>((int)b.size(), max);
  std::copy(b.begin(), b.begin() + n, out);
  return (int)b.size();
}

// Share the full blocks of `src` with a new sequence `dst` (prefix caching).  The
// partially filled last block is NOT shared: the caller re-computes / copies it.
// Returns the number of tokens covered by the shared blocks, or -1.
int lumen_kv_fork(void* h, int64_t src, int64_t dst) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->seqs.find(src);
  if (it == m->seqs.end() || m->seqs.count(dst)) return -1;
  const int full = it->second.tokens / kBlock;
  Seq d;
  for (int i = 0; i < full; ++i) {
    const int b = it->second.blocks[i];
    ++m->ref[b];
    d.blocks.push_back(b);
  }
  d.tokens = full * kBlock;
  m->seqs[dst] = d;
  return d.tokens;
}

int lumen_kv_release(void* h, int64_t seq) {
  auto* m = static_cast<Manager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->seqs.find(seq);
  if (it == m->seqs.end()) return -1;
  for (int b : it->second.blocks) m->drop(b);
  m->seqs.erase(it);
  return 0;
}

}  // extern "C"
