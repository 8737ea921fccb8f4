// Cross-process request channel between serving front ends and a GPU engine process
// (host runtime, C ABI for ctypes).
//
// The reference serves every request inside one gRPC process on a 10-thread pool, batch 1
// (src/lumen/server.py:232-235).  Here K front-end processes (gRPC accept, chunk reassembly,
// JPEG decode, tokenisation -- all CPU work that Python's one interpreter lock would serialise)
// feed ONE engine process per GPU, which merges their requests into device batches.  A channel
// is one shared memory region (memfd, mapped by every process at its own address):
//
//   Header | submission ring | free ring | Slot[nslots] | payload[nslots][slot_bytes]
//                                                       | result[nslots][result_bytes]
//
// * a front end takes a FREE slot from the free ring, writes the request payload (a decoded
//   image, token ids, ...) and its descriptor into the slot, and pushes the slot id onto the
//   submission ring (state QUEUED);
// * the engine pops up to max_n queued slots -- blocking on a futex while the ring is empty,
//   then lingering up to linger_us for more so concurrent requests form one batch -- marks them
//   RUNNING, runs the batch, writes each result into the slot's result area and completes it
//   (DONE / ERROR), waking the one front-end thread that waits on that slot's state word;
// * the front end copies the result out and releases the slot.
//
// Rings are bounded MPMC queues (per-cell sequence numbers); every blocking wait is a shared
// (not process-private) futex on a word of the region with a timeout, so a dead peer costs a
// timeout, never a hang.  The engine writes a heartbeat; a restarted engine bumps the
// generation and fails the slots its predecessor left RUNNING.
//
// Streaming requests (VLM token streams): while a slot is RUNNING the engine may APPEND partial
// records ([u32 length][bytes], 8-byte aligned) to the slot's result area (lumen_ch_partial); the
// front end waits on the slot's pseq futex word (bumped by every append and by completion) and
// hands each record on as it lands (lumen_ch_wait_partial).  The final result then goes after the
// log (Slot::roff), so nothing the front end has not read yet is overwritten.  An append to a slot
// its front end abandoned returns -2: the engine stops generating for it.
//
// A front end that stops waiting (timeout) ABANDONS its slot instead of leaking it: a slot that
// is still queued is marked ABANDONED_Q and the engine frees it when it pops it; one that is
// running is marked ABANDONED_R and the engine frees it at completion (or a restarted engine
// frees it); one that already finished is freed by the front end on the spot.  Every hand-over
// is a compare-and-swap on the state word, so exactly one side returns the slot to the free ring.
#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <new>

namespace {

constexpr uint32_t kMagic = 0x4c4d4348;   // "LMCH"
constexpr uint32_t kVersion = 2;

enum State : uint32_t { FREE = 0, FILLING = 1, QUEUED = 2, RUNNING = 3, DONE = 4, ERROR = 5,
                       ABANDONED_Q = 6, ABANDONED_R = 7 };

struct alignas(64) Cell {
  std::atomic<uint64_t> seq;
  uint32_t val;
};

struct alignas(64) Ring {
  uint32_t cap;   // power of two
  uint32_t mask;
  alignas(64) std::atomic<uint64_t> head;   // next enqueue position
  alignas(64) std::atomic<uint64_t> tail;   // next dequeue position
};

struct alignas(64) Header {
  uint32_t magic, version, nslots, cap;
  uint64_t slot_bytes, result_bytes;
  uint64_t sq_cells_off, free_cells_off, slots_off, payload_off, result_off, total;
  alignas(64) std::atomic<uint64_t> heartbeat_ns;
  std::atomic<uint32_t> engine_gen;
  std::atomic<uint32_t> engine_pid;
  alignas(64) std::atomic<uint32_t> sq_futex;     // bumped on every submission
  alignas(64) std::atomic<uint32_t> free_futex;   // bumped on every release
  alignas(64) std::atomic<int32_t> depth;         // queued + running (load balancing)
  alignas(64) Ring sq;
  alignas(64) Ring fq;
};

// Per-slot descriptor (mirrored by lumen_amd/parallel/shm_channel.py:_SlotDesc)
struct alignas(64) Slot {
  std::atomic<uint32_t> state;   // futex word
  uint32_t kind;                 // request kind (channel-specific code)
  uint32_t dtype;                // payload element type code
  uint32_t ndim;
  uint32_t shape[4];
  uint64_t nbytes;               // payload bytes
  uint32_t rdtype;               // result element type code
  uint32_t rndim;
  uint32_t rshape[4];
  uint64_t rbytes;               // result bytes
  uint32_t status;               // 0 ok; else an error (message text in the result area)
  uint32_t gen;                  // engine generation that ran it
  uint64_t tag;                  // submitter tag (pid << 32 | sequence), diagnostics
  char meta[128];                // small per-request options (UTF-8 JSON), NUL-terminated
  std::atomic<uint32_t> pseq;    // futex word: bumped by every partial append and by completion
  uint32_t pflags;               // reserved
  std::atomic<uint64_t> plen;    // bytes of partial records in the result area
  uint64_t roff;                 // offset of the final result in the result area (after the log)
};

inline uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// shared futexes: the region is mapped at different addresses in different processes
inline long futex_wait(std::atomic<uint32_t>* w, uint32_t expected, int64_t timeout_ns) {
  timespec ts;
  ts.tv_sec = (time_t)(timeout_ns / 1000000000ll);
  ts.tv_nsec = (long)(timeout_ns % 1000000000ll);
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expected, &ts, nullptr, 0);
}

inline void futex_wake(std::atomic<uint32_t>* w, int n) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, n, nullptr, nullptr, 0);
}

inline Header* H(void* base) { return static_cast<Header*>(base); }
inline Cell* cells(void* base, uint64_t off) { return reinterpret_cast<Cell*>(static_cast<char*>(base) + off); }
inline Slot* slots(void* base) { return reinterpret_cast<Slot*>(static_cast<char*>(base) + H(base)->slots_off); }

inline uint64_t align64(uint64_t x) { return (x + 63) & ~uint64_t(63); }

bool ring_push(Ring& r, Cell* c, uint32_t v) {
  uint64_t pos = r.head.load(std::memory_order_relaxed);
  for (;;) {
    Cell& cell = c[pos & r.mask];
    const uint64_t seq = cell.seq.load(std::memory_order_acquire);
    const int64_t dif = (int64_t)seq - (int64_t)pos;
    if (dif == 0) {
      if (r.head.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        cell.val = v;
        cell.seq.store(pos + 1, std::memory_order_release);
        return true;
      }
    } else if (dif < 0) {
      return false;   // full
    } else {
      pos = r.head.load(std::memory_order_relaxed);
    }
  }
}

bool ring_pop(Ring& r, Cell* c, uint32_t* v) {
  uint64_t pos = r.tail.load(std::memory_order_relaxed);
  for (;;) {
    Cell& cell = c[pos & r.mask];
    const uint64_t seq = cell.seq.load(std::memory_order_acquire);
    const int64_t dif = (int64_t)seq - (int64_t)(pos + 1);
    if (dif == 0) {
      if (r.tail.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        *v = cell.val;
        cell.seq.store(pos + r.mask + 1, std::memory_order_release);
        return true;
      }
    } else if (dif < 0) {
      return false;   // empty
    } else {
      pos = r.tail.load(std::memory_order_relaxed);
    }
  }
}

void ring_init(Ring& r, Cell* c, uint32_t cap) {
  r.cap = cap;
  r.mask = cap - 1;
  r.head.store(0);
  r.tail.store(0);
  for (uint32_t i = 0; i < cap; ++i) c[i].seq.store(i);
}

uint32_t pow2_at_least(uint32_t n) {
  uint32_t c = 1;
  while (c < n) c <<= 1;
  return c;
}

struct Layout {
  uint32_t cap;
  uint64_t sq_cells, free_cells, slots, payload, result, total;
};

Layout layout(int nslots, uint64_t slot_bytes, uint64_t result_bytes) {
  Layout L{};
  L.cap = pow2_at_least((uint32_t)nslots);
  uint64_t off = align64(sizeof(Header));
  L.sq_cells = off;
  off = align64(off + (uint64_t)L.cap * sizeof(Cell));
  L.free_cells = off;
  off = align64(off + (uint64_t)L.cap * sizeof(Cell));
  L.slots = off;
  off = align64(off + (uint64_t)nslots * sizeof(Slot));
  off = (off + 4095) & ~uint64_t(4095);   // payload slots page aligned (H2D straight from them)
  L.payload = off;
  off += (uint64_t)nslots * ((slot_bytes + 4095) & ~uint64_t(4095));
  L.result = off;
  off += (uint64_t)nslots * align64(result_bytes);
  L.total = (off + 4095) & ~uint64_t(4095);
  return L;
}

}  // namespace

extern "C" {

uint64_t lumen_ch_region_bytes(int nslots, uint64_t slot_bytes, uint64_t result_bytes) {
  if (nslots <= 0) return 0;
  return layout(nslots, slot_bytes, result_bytes).total;
}

// Format a zero-filled region of lumen_ch_region_bytes() bytes (the creating process, once).
int lumen_ch_init(void* base, int nslots, uint64_t slot_bytes, uint64_t result_bytes) {
  if (base == nullptr || nslots <= 0 || slot_bytes == 0) return -1;
  const Layout L = layout(nslots, slot_bytes, result_bytes);
  Header* h = H(base);
  new (h) Header();
  h->nslots = (uint32_t)nslots;
  h->cap = L.cap;
  h->slot_bytes = (slot_bytes + 4095) & ~uint64_t(4095);
  h->result_bytes = align64(result_bytes);
  h->sq_cells_off = L.sq_cells;
  h->free_cells_off = L.free_cells;
  h->slots_off = L.slots;
  h->payload_off = L.payload;
  h->result_off = L.result;
  h->total = L.total;
  h->heartbeat_ns.store(0);
  h->engine_gen.store(0);
  h->engine_pid.store(0);
  h->sq_futex.store(0);
  h->free_futex.store(0);
  h->depth.store(0);
  ring_init(h->sq, cells(base, L.sq_cells), L.cap);
  ring_init(h->fq, cells(base, L.free_cells), L.cap);
  Slot* s = slots(base);
  for (int i = 0; i < nslots; ++i) {
    new (&s[i]) Slot();
    s[i].state.store(FREE);
    ring_push(h->fq, cells(base, L.free_cells), (uint32_t)i);
  }
  std::atomic_thread_fence(std::memory_order_release);
  h->version = kVersion;
  h->magic = kMagic;
  return 0;
}

int lumen_ch_check(void* base) {
  return base != nullptr && H(base)->magic == kMagic && H(base)->version == kVersion ? 0 : -1;
}

int lumen_ch_nslots(void* base) { return (int)H(base)->nslots; }
uint64_t lumen_ch_slot_bytes(void* base) { return H(base)->slot_bytes; }
uint64_t lumen_ch_result_bytes(void* base) { return H(base)->result_bytes; }
uint64_t lumen_ch_total_bytes(void* base) { return H(base)->total; }
uint64_t lumen_ch_slot_desc_off(void* base, int i) { return H(base)->slots_off + (uint64_t)i * sizeof(Slot); }
uint64_t lumen_ch_payload_off(void* base, int i) { return H(base)->payload_off + (uint64_t)i * H(base)->slot_bytes; }
uint64_t lumen_ch_result_off(void* base, int i) { return H(base)->result_off + (uint64_t)i * H(base)->result_bytes; }
int lumen_ch_slot_desc_size() { return (int)sizeof(Slot); }
int lumen_ch_slot_state(void* base, int i) { return (int)slots(base)[i].state.load(std::memory_order_acquire); }
int lumen_ch_depth(void* base) { return H(base)->depth.load(std::memory_order_relaxed); }

// A FREE slot (state FILLING) or -1 after timeout_ms (every slot in use).
int lumen_ch_acquire(void* base, int timeout_ms) {
  Header* h = H(base);
  Cell* fc = cells(base, h->free_cells_off);
  const uint64_t deadline = now_ns() + (uint64_t)(timeout_ms < 0 ? 0 : timeout_ms) * 1000000ull;
  for (;;) {
    const uint32_t seen = h->free_futex.load(std::memory_order_acquire);
    uint32_t v;
    if (ring_pop(h->fq, fc, &v)) {
      Slot& s = slots(base)[v];
      s.status = 0;
      s.rbytes = 0;
      s.rndim = 0;
      s.meta[0] = 0;
      s.plen.store(0, std::memory_order_relaxed);
      s.roff = 0;
      s.state.store(FILLING, std::memory_order_release);
      return (int)v;
    }
    const uint64_t t = now_ns();
    if (t >= deadline) return -1;
    futex_wait(&h->free_futex, seen, (int64_t)(deadline - t));
  }
}

// Publish a filled slot to the engine.
int lumen_ch_submit(void* base, int slot, uint64_t tag) {
  Header* h = H(base);
  Slot& s = slots(base)[slot];
  s.tag = tag;
  h->depth.fetch_add(1, std::memory_order_relaxed);
  s.state.store(QUEUED, std::memory_order_release);
  if (!ring_push(h->sq, cells(base, h->sq_cells_off), (uint32_t)slot)) {   // cannot happen: cap >= nslots
    h->depth.fetch_sub(1, std::memory_order_relaxed);
    s.state.store(FILLING, std::memory_order_release);
    return -1;
  }
  h->sq_futex.fetch_add(1, std::memory_order_release);
  futex_wake(&h->sq_futex, 1);
  return 0;
}

// Wait until the slot is DONE / ERROR; returns the state, or -1 after timeout_ms.
int lumen_ch_wait(void* base, int slot, int timeout_ms) {
  Slot& s = slots(base)[slot];
  const uint64_t deadline = now_ns() + (uint64_t)(timeout_ms < 0 ? 0 : timeout_ms) * 1000000ull;
  for (;;) {
    const uint32_t st = s.state.load(std::memory_order_acquire);
    if (st == DONE || st == ERROR) return (int)st;
    const uint64_t t = now_ns();
    if (t >= deadline) return -1;
    futex_wait(&s.state, st, (int64_t)(deadline - t));
  }
}

// Return a slot to the free ring (after the result was copied out, or to abandon a FILLING slot).
void lumen_ch_release(void* base, int slot) {
  Header* h = H(base);
  slots(base)[slot].state.store(FREE, std::memory_order_release);
  ring_push(h->fq, cells(base, h->free_cells_off), (uint32_t)slot);
  h->free_futex.fetch_add(1, std::memory_order_release);
  futex_wake(&h->free_futex, 1);
}

// Engine: pop up to max_n queued slots into out (state RUNNING).  Blocks up to wait_ms for the
// first; after it, keeps collecting for up to linger_us (batch formation window).  Returns the
// count (0 on timeout).
int lumen_ch_pop_batch(void* base, int* out, int max_n, int wait_ms, int linger_us) {
  Header* h = H(base);
  Cell* sc = cells(base, h->sq_cells_off);
  Slot* sl = slots(base);
  const uint32_t gen = h->engine_gen.load(std::memory_order_relaxed);
  int n = 0;
  const uint64_t t0 = now_ns();
  const uint64_t first_deadline = t0 + (uint64_t)(wait_ms < 0 ? 0 : wait_ms) * 1000000ull;
  uint64_t linger_deadline = 0;
  while (n < max_n) {
    const uint32_t seen = h->sq_futex.load(std::memory_order_acquire);
    uint32_t v;
    if (ring_pop(h->sq, sc, &v)) {
      uint32_t st = QUEUED;
      if (!sl[v].state.compare_exchange_strong(st, RUNNING, std::memory_order_acq_rel)) {
        // ABANDONED_Q: its front end gave up while it was queued; free it here
        h->depth.fetch_sub(1, std::memory_order_relaxed);
        lumen_ch_release(base, (int)v);
        continue;
      }
      sl[v].gen = gen;
      out[n++] = (int)v;
      if (n == 1) linger_deadline = now_ns() + (uint64_t)(linger_us < 0 ? 0 : linger_us) * 1000ull;
      continue;
    }
    const uint64_t t = now_ns();
    const uint64_t dl = n == 0 ? first_deadline : linger_deadline;
    if (t >= dl) break;
    futex_wait(&h->sq_futex, seen, (int64_t)(dl - t));
  }
  return n;
}

// Engine: finish a RUNNING slot (status 0 -> DONE, else ERROR) and wake its waiter.
void lumen_ch_complete(void* base, int slot, int status) {
  Header* h = H(base);
  Slot& s = slots(base)[slot];
  s.status = (uint32_t)status;
  uint32_t st = RUNNING;
  const bool handed = s.state.compare_exchange_strong(st, status == 0 ? DONE : ERROR, std::memory_order_acq_rel);
  h->depth.fetch_sub(1, std::memory_order_relaxed);
  if (handed) {
    futex_wake(&s.state, INT_MAX);
    s.pseq.fetch_add(1, std::memory_order_release);   // a streaming waiter sleeps on pseq
    futex_wake(&s.pseq, INT_MAX);
  } else if (st == ABANDONED_R) {
    lumen_ch_release(base, slot);   // nobody waits for it any more
  }
}

// Engine: append one partial record to a RUNNING slot.  0 ok, -1 no room left in the result
// area (the record is dropped: the final result must carry everything), -2 the slot is no longer
// RUNNING (abandoned by its front end, or failed by a restart): stop producing for it.
int lumen_ch_partial(void* base, int slot, const void* data, uint64_t n) {
  Header* h = H(base);
  Slot& s = slots(base)[slot];
  if (s.state.load(std::memory_order_acquire) != RUNNING) return -2;
  const uint64_t at = s.plen.load(std::memory_order_relaxed);
  const uint64_t rec = (4 + n + 7) & ~uint64_t(7);
  if (n > 0xffffffffull || at + rec > h->result_bytes) return -1;
  char* dst = static_cast<char*>(base) + lumen_ch_result_off(base, slot) + at;
  const uint32_t len = (uint32_t)n;
  std::memcpy(dst, &len, 4);
  if (n) std::memcpy(dst + 4, data, n);
  s.plen.store(at + rec, std::memory_order_release);
  s.pseq.fetch_add(1, std::memory_order_release);
  futex_wake(&s.pseq, INT_MAX);
  return 0;
}

uint64_t lumen_ch_plen(void* base, int slot) {
  return slots(base)[slot].plen.load(std::memory_order_acquire);
}

// Front end of a streaming slot: wait until it has partial bytes past seen_plen (returns RUNNING)
// or is DONE / ERROR (returns that state); -1 after timeout_ms.
int lumen_ch_wait_partial(void* base, int slot, uint64_t seen_plen, int timeout_ms) {
  Slot& s = slots(base)[slot];
  const uint64_t deadline = now_ns() + (uint64_t)(timeout_ms < 0 ? 0 : timeout_ms) * 1000000ull;
  for (;;) {
    const uint32_t seq = s.pseq.load(std::memory_order_acquire);
    if (s.plen.load(std::memory_order_acquire) > seen_plen) return RUNNING;
    const uint32_t st = s.state.load(std::memory_order_acquire);
    if (st == DONE || st == ERROR) return (int)st;
    const uint64_t t = now_ns();
    if (t >= deadline) return -1;
    futex_wait(&s.pseq, seq, (int64_t)(deadline - t));
  }
}

// Front end: give up on a submitted slot (after a wait timeout).  Returns 1 when the slot was
// already finished and is freed here, 0 when the engine will free it (queued / running).
int lumen_ch_abandon(void* base, int slot) {
  Slot& s = slots(base)[slot];
  for (;;) {
    uint32_t st = s.state.load(std::memory_order_acquire);
    if (st == DONE || st == ERROR) {
      lumen_ch_release(base, slot);
      return 1;
    }
    const uint32_t to = st == QUEUED ? ABANDONED_Q : st == RUNNING ? ABANDONED_R : 0;
    if (to == 0) return -1;   // FREE / FILLING / already abandoned: not a submitted slot
    if (s.state.compare_exchange_weak(st, to, std::memory_order_acq_rel)) return 0;
  }
}

void lumen_ch_heartbeat(void* base, uint32_t pid) {
  H(base)->engine_pid.store(pid, std::memory_order_relaxed);
  H(base)->heartbeat_ns.store(now_ns(), std::memory_order_release);
}

// ns since the last heartbeat (UINT64_MAX: never)
uint64_t lumen_ch_heartbeat_age_ns(void* base) {
  const uint64_t hb = H(base)->heartbeat_ns.load(std::memory_order_acquire);
  if (hb == 0) return UINT64_MAX;
  const uint64_t t = now_ns();
  return t > hb ? t - hb : 0;
}

// A (re)started engine: new generation; slots a previous engine left RUNNING fail (their
// waiters see ERROR with the message below); QUEUED ones stay queued for the new engine.
int lumen_ch_engine_start(void* base, uint32_t pid) {
  Header* h = H(base);
  h->engine_gen.fetch_add(1, std::memory_order_acq_rel);
  int failed = 0;
  Slot* sl = slots(base);
  for (uint32_t i = 0; i < h->nslots; ++i) {
    uint32_t ab = ABANDONED_R;   // abandoned while the dead engine ran it: nobody else frees it
    if (sl[i].state.compare_exchange_strong(ab, FREE, std::memory_order_acq_rel)) {
      h->depth.fetch_sub(1, std::memory_order_relaxed);
      lumen_ch_release(base, (int)i);
      continue;
    }
    uint32_t st = RUNNING;
    if (sl[i].state.load(std::memory_order_acquire) == RUNNING) {
      const char text[] = "engine restarted while this request was running";
      // after any partial records a streaming front end may still be reading
      uint64_t at = (sl[i].plen.load(std::memory_order_acquire) + 63) & ~uint64_t(63);
      if (at + sizeof(text) > h->result_bytes) at = 0;
      char* msg = static_cast<char*>(base) + lumen_ch_result_off(base, (int)i) + at;
      std::memcpy(msg, text, sizeof(text));
      sl[i].rbytes = sizeof(text) - 1;
      sl[i].status = 1;
      sl[i].roff = at;
      if (sl[i].state.compare_exchange_strong(st, ERROR, std::memory_order_acq_rel)) {
        h->depth.fetch_sub(1, std::memory_order_relaxed);
        futex_wake(&sl[i].state, INT_MAX);
        sl[i].pseq.fetch_add(1, std::memory_order_release);
        futex_wake(&sl[i].pseq, INT_MAX);
        ++failed;
      }
    }
  }
  lumen_ch_heartbeat(base, pid);
  return failed;
}

}  // extern "C"
