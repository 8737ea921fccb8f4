// Tensor-parallel step bus: one writer (TP rank 0, the engine) -> N readers (the follower ranks
// on the same node), in host shared memory (host runtime, C ABI for ctypes).
//
// Every engine step the leader tells the followers what to replay: a decode step descriptor
// (token ids, positions, cache slots, context lengths, block table, ~100 bytes at batch 1) or a
// pickled control message.  Sending that through a device collective costs each follower a
// broadcast plus a device->host copy of the buffer before it can even pick the graph to replay;
// through this bus a follower's host sees the descriptor a few hundred nanoseconds after the
// leader wrote it and launches its step while the leader launches its own.
//
// Layout of the region (POSIX shm, mapped by every rank at its own address):
//
//   BusHeader | slot[nslots] = { uint64 length | payload[slot_bytes] }
//
// The writer fills slot (head % nslots) and publishes it with a release store of head + 1 (and
// a futex wake for readers that went to sleep); reader r copies slot (tail[r] % nslots) once
// head > tail[r] and advances its own tail.  The writer never overwrites a slot a reader has
// not consumed: it waits while head - min(tail) == nslots.  Waits spin briefly (a decode step is
// ~1-3 ms, so a reader normally catches the next message in the spin) and then sleep on a
// shared futex with a timeout: a dead peer costs a timeout, never a hang.
#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstdint>
#include <cstring>
#include <new>

namespace {

constexpr uint32_t kBusMagic = 0x4c4d4253;   // "LMBS"
constexpr int kMaxReaders = 16;

struct alignas(64) Tail {
  std::atomic<uint64_t> v;
};

struct alignas(64) BusHeader {
  uint32_t magic, nslots, nreaders, writer_pid;
  uint64_t slot_bytes, total;
  alignas(64) std::atomic<uint64_t> head;        // messages published
  alignas(64) std::atomic<uint32_t> head_word;   // futex word: low 32 bits of head
  std::atomic<uint32_t> closed;
  alignas(64) std::atomic<uint32_t> tail_word;   // futex word bumped whenever a reader advances
  Tail tail[kMaxReaders];                        // messages consumed, per reader
};

inline uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

inline long futex_wait(std::atomic<uint32_t>* w, uint32_t expected, int64_t timeout_ns) {
  timespec ts{(time_t)(timeout_ns / 1000000000ll), (long)(timeout_ns % 1000000000ll)};
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expected, &ts, nullptr, 0);
}

inline void futex_wake(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

inline void cpu_relax() { __builtin_ia32_pause(); }

inline BusHeader* B(void* base) { return static_cast<BusHeader*>(base); }

inline uint64_t hdr_bytes() { return (sizeof(BusHeader) + 63) & ~uint64_t(63); }

inline char* slot(void* base, uint64_t i) {
  BusHeader* h = B(base);
  return static_cast<char*>(base) + hdr_bytes() + (i % h->nslots) * (8 + h->slot_bytes);
}

uint64_t min_tail(BusHeader* h) {
  uint64_t m = UINT64_MAX;
  for (uint32_t r = 0; r < h->nreaders; ++r) {
    const uint64_t t = h->tail[r].v.load(std::memory_order_acquire);
    m = t < m ? t : m;
  }
  return h->nreaders ? m : h->head.load(std::memory_order_relaxed);
}

void* map_fd(int fd, uint64_t bytes) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  return p == MAP_FAILED ? nullptr : p;
}

}  // namespace

extern "C" {

uint64_t lumen_bus_region_bytes(int nslots, uint64_t slot_bytes) {
  return hdr_bytes() + (uint64_t)nslots * (8 + ((slot_bytes + 63) & ~uint64_t(63)));
}

// Writer: create + initialise the named region (fails if the name exists).  Returns the mapping.
void* lumen_bus_create(const char* name, int nslots, uint64_t slot_bytes, int nreaders) {
  if (nslots < 2 || nreaders < 0 || nreaders > kMaxReaders || slot_bytes == 0) return nullptr;
  slot_bytes = (slot_bytes + 63) & ~uint64_t(63);
  const uint64_t total = lumen_bus_region_bytes(nslots, slot_bytes);
  const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return nullptr;
  if (ftruncate(fd, (off_t)total) != 0) {
    close(fd);
    shm_unlink(name);
    return nullptr;
  }
  void* base = map_fd(fd, total);
  close(fd);
  if (!base) {
    shm_unlink(name);
    return nullptr;
  }
  std::memset(base, 0, hdr_bytes());
  BusHeader* h = new (base) BusHeader();
  h->nslots = (uint32_t)nslots;
  h->nreaders = (uint32_t)nreaders;
  h->writer_pid = (uint32_t)getpid();
  h->slot_bytes = slot_bytes;
  h->total = total;
  h->head.store(0, std::memory_order_relaxed);
  for (int r = 0; r < kMaxReaders; ++r) h->tail[r].v.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  reinterpret_cast<std::atomic<uint32_t>*>(&h->magic)->store(kBusMagic, std::memory_order_release);
  return base;
}

// Reader: map an existing region by name.
void* lumen_bus_open(const char* name) {
  const int fd = shm_open(name, O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || (uint64_t)st.st_size < hdr_bytes()) {
    close(fd);
    return nullptr;
  }
  void* base = map_fd(fd, (uint64_t)st.st_size);
  close(fd);
  if (!base) return nullptr;
  if (reinterpret_cast<std::atomic<uint32_t>*>(&B(base)->magic)->load(std::memory_order_acquire) != kBusMagic) {
    munmap(base, (size_t)st.st_size);
    return nullptr;
  }
  return base;
}

int lumen_bus_unlink(const char* name) { return shm_unlink(name); }

void lumen_bus_unmap(void* base) {
  if (base) munmap(base, (size_t)B(base)->total);
}

uint64_t lumen_bus_slot_bytes(void* base) { return B(base)->slot_bytes; }
uint32_t lumen_bus_writer_pid(void* base) { return B(base)->writer_pid; }
uint64_t lumen_bus_head(void* base) { return B(base)->head.load(std::memory_order_acquire); }

// Writer: publish n bytes.  0 = ok, -1 = timed out waiting for a slow reader, -2 = too big / closed.
int lumen_bus_publish(void* base, const void* data, uint64_t n, int timeout_ms) {
  BusHeader* h = B(base);
  if (n > h->slot_bytes || h->closed.load(std::memory_order_relaxed)) return -2;
  const uint64_t hd = h->head.load(std::memory_order_relaxed);
  const uint64_t t0 = now_ns();
  const uint64_t limit = (uint64_t)timeout_ms * 1000000ull;
  while (hd - min_tail(h) >= h->nslots) {          // the slot about to be reused is still unread
    const uint32_t w = h->tail_word.load(std::memory_order_acquire);
    if (hd - min_tail(h) < h->nslots) break;
    const uint64_t el = now_ns() - t0;
    if (el >= limit) return -1;
    futex_wait(&h->tail_word, w, (int64_t)(limit - el < 1000000ull ? limit - el : 1000000ull));
  }
  char* s = slot(base, hd);
  std::memcpy(s + 8, data, n);
  *reinterpret_cast<uint64_t*>(s) = n;
  h->head.store(hd + 1, std::memory_order_release);
  h->head_word.store((uint32_t)(hd + 1), std::memory_order_release);
  futex_wake(&h->head_word);
  return 0;
}

// Reader r: copy the next message into out (cap bytes).  Returns its length, -1 on timeout,
// -2 if the bus was closed, -3 if out is too small (the message stays unread).
// spin_us: busy-wait this long before sleeping on the futex.
int64_t lumen_bus_next(void* base, int reader, void* out, uint64_t cap, int timeout_ms, int spin_us) {
  BusHeader* h = B(base);
  if (reader < 0 || reader >= (int)h->nreaders) return -2;
  const uint64_t tl = h->tail[reader].v.load(std::memory_order_relaxed);
  const uint64_t t0 = now_ns();
  const uint64_t spin = (uint64_t)spin_us * 1000ull;
  const uint64_t limit = (uint64_t)timeout_ms * 1000000ull;
  for (;;) {
    if (h->head.load(std::memory_order_acquire) > tl) break;
    if (h->closed.load(std::memory_order_relaxed)) return -2;
    const uint64_t el = now_ns() - t0;
    if (el < spin) {
      for (int i = 0; i < 64; ++i) cpu_relax();
      continue;
    }
    if (el >= limit) return -1;
    const uint32_t w = h->head_word.load(std::memory_order_acquire);
    if (h->head.load(std::memory_order_acquire) > tl) break;
    futex_wait(&h->head_word, w, (int64_t)(limit - el < 1000000ull ? limit - el : 1000000ull));
  }
  const char* s = slot(base, tl);
  const uint64_t n = *reinterpret_cast<const uint64_t*>(s);
  if (n > cap) return -3;
  std::memcpy(out, s + 8, n);
  h->tail[reader].v.store(tl + 1, std::memory_order_release);
  h->tail_word.fetch_add(1, std::memory_order_acq_rel);
  futex_wake(&h->tail_word);
  return (int64_t)n;
}

void lumen_bus_close(void* base) {
  BusHeader* h = B(base);
  h->closed.store(1, std::memory_order_release);
  h->head_word.fetch_add(1, std::memory_order_acq_rel);
  futex_wake(&h->head_word);
  h->tail_word.fetch_add(1, std::memory_order_acq_rel);
  futex_wake(&h->tail_word);
}

}  // extern "C"
