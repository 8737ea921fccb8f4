// Parallel baseline-JPEG entropy decoder (host runtime, C ABI for ctypes).
//
// Replaces the single-threaded libjpeg-turbo decode (via Pillow) that the reference runs per
// request (packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:661-665,
// packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:478).  On a high-entropy photo
// most of libjpeg's time is the Huffman decode (a 687 KiB noise JPEG: 80 % of its decode time
// even at 1/8 DCT scale), which is sequential by construction.  Here it is split over the
// cores; the dequantise + IDCT + chroma upsampling + colour conversion run on the GPU
// (csrc/jpeg.hip) from the coefficient planes this file produces.
//
// Without restart markers the bitstream has no known symbol boundaries, so every chunk of
// the (unstuffed) entropy-coded segment is first decoded SPECULATIVELY from its first bit,
// guessing "start of an MCU", recording every block boundary (bit position, block phase
// inside the MCU) it passes.  Huffman codes self-synchronise: an exact decode entering the
// chunk (from the previous chunk's exact end) soon lands on one of those recorded
// boundaries, and from there the speculative blocks are the true ones.  The sequential
// fix-up pass therefore only re-decodes the few blocks before that meeting point; a chunk
// that never synchronises is simply decoded exactly (correct, just serial).  With restart
// markers (DRI) the restart intervals are decoded independently.
//
// Coefficients land de-zigzagged, not dequantised, in per-component planes
// [blocks_h][blocks_w][64] int16 (padded to whole MCUs), DC already integrated.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <array>
#include <thread>
#include <vector>

#include "../jpeg_huff.h"
#include "../jpeg_huff_core.h"

namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int kFast = 10;   // lookahead bits of the fast tables

struct Huff {
  uint16_t fast[1 << kFast];   // (length << 8) | symbol for codes of <= kFast bits, 0 = slow path
  // AC only: code AND its extra bits within the lookahead -> the coefficient in one step:
  // (value << 16) | (run << 12) | (total length << 4) | 1, 0 = not in the lookahead
  int32_t fast_ac[1 << kFast];
  int32_t maxcode[18];
  int32_t valptr[17];
  int32_t mincode[17];
  uint8_t vals[256];
  bool present = false;
};

struct Comp {
  int id, h, v, tq, td, ta;
  int bw, bh;   // blocks per row / column (whole MCUs)
};

struct Jpeg {
  int width = 0, height = 0, ncomp = 0, hmax = 1, vmax = 1, restart = 0;
  int mcux = 0, mcuy = 0;
  bool progressive = false, supported = true;
  Comp comp[4];
  uint16_t qt[4][64];   // natural order
  Huff dc[4], ac[4];
  int scan_ncomp = 0, scan_comp[4];
  size_t ecs_begin = 0, ecs_end = 0;   // entropy-coded segment in the input
};

// false when the code counts oversubscribe the code space (more length-l codes than 2^l minus
// those taken by shorter codes), the check libjpeg's jdhuff makes: such a table would index
// past the fast tables below.
bool build_huff(Huff& h, const uint8_t* counts, const uint8_t* vals, int nvals) {
  {
    int64_t c = 0;
    for (int l = 1; l <= 16; ++l) {
      c += counts[l - 1];
      if (c > ((int64_t)1 << l)) return false;
      c <<= 1;
    }
  }
  memset(h.fast, 0, sizeof(h.fast));
  memcpy(h.vals, vals, nvals);
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    h.valptr[l] = k;
    h.mincode[l] = code;
    code += counts[l - 1];
    k += counts[l - 1];
    h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
    code <<= 1;
  }
  h.maxcode[17] = 0x7fffffff;
  // fast tables
  memset(h.fast_ac, 0, sizeof(h.fast_ac));
  code = 0;
  k = 0;
  for (int l = 1; l <= kFast; ++l) {
    for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
      const int shift = kFast - l;
      const int rs = vals[k], run = rs >> 4, sz = rs & 15;
      for (int j = 0; j < (1 << shift); ++j) {
        const int idx = (code << shift) | j;
        if (idx >= (1 << kFast)) return false;
        h.fast[idx] = (uint16_t)((l << 8) | rs);
        if (sz != 0 && l + sz <= kFast) {
          const int extra = (j >> (shift - sz)) & ((1 << sz) - 1);
          const int v = extra < (1 << (sz - 1)) ? extra - (1 << sz) + 1 : extra;
          h.fast_ac[idx] = (int32_t)((uint32_t)(v & 0xFFFF) << 16) | (run << 12) | ((l + sz) << 4) | 1;
        }
      }
    }
    code <<= 1;
  }
  h.present = true;
  return true;
}

inline int read16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// 0 ok, 1 unsupported, -1 malformed
int parse(const uint8_t* d, size_t n, Jpeg& J) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return -1;
  size_t i = 2;
  bool sof = false;
  while (i + 4 <= n) {
    if (d[i] != 0xFF) return -1;
    int m = d[i + 1];
    if (m == 0xFF) { ++i; continue; }
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) { i += 2; continue; }
    const int L = read16(d + i + 2);
    if (i + 2 + (size_t)L > n || L < 2) return -1;
    const uint8_t* s = d + i + 4;
    const int sl = L - 2;
    if (m == 0xC0 || m == 0xC1) {          // baseline / extended sequential Huffman
      if (sl < 6) return -1;
      if (s[0] != 8) return 1;             // 12-bit
      J.height = read16(s + 1);
      J.width = read16(s + 3);
      J.ncomp = s[5];
      if (J.ncomp != 1 && J.ncomp != 3) return 1;
      if (sl < 6 + 3 * J.ncomp || J.width <= 0 || J.height <= 0) return -1;
      for (int c = 0; c < J.ncomp; ++c) {
        J.comp[c].id = s[6 + 3 * c];
        J.comp[c].h = s[7 + 3 * c] >> 4;
        J.comp[c].v = s[7 + 3 * c] & 15;
        J.comp[c].tq = s[8 + 3 * c] & 3;
        if (J.comp[c].h < 1 || J.comp[c].h > 2 || J.comp[c].v < 1 || J.comp[c].v > 2) return 1;
        J.hmax = std::max(J.hmax, J.comp[c].h);
        J.vmax = std::max(J.vmax, J.comp[c].v);
      }
      sof = true;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return 1;                            // progressive / lossless / arithmetic
    } else if (m == 0xC4) {                // DHT
      int o = 0;
      while (o + 17 <= sl) {
        const int tc = s[o] >> 4, th = s[o] & 15;
        if (th > 3 || tc > 1) return -1;
        int tot = 0;
        for (int l = 0; l < 16; ++l) tot += s[o + 1 + l];
        if (tot > 256 || o + 17 + tot > sl) return -1;
        if (!build_huff(tc == 0 ? J.dc[th] : J.ac[th], s + o + 1, s + o + 17, tot)) return -1;
        o += 17 + tot;
      }
    } else if (m == 0xDB) {                // DQT
      int o = 0;
      while (o < sl) {
        const int pq = s[o] >> 4, tq = s[o] & 15;
        if (tq > 3) return -1;
        if (pq == 0) {
          if (o + 65 > sl) return -1;
          for (int k = 0; k < 64; ++k) J.qt[tq][kZigzag[k]] = s[o + 1 + k];
          o += 65;
        } else {
          if (o + 129 > sl) return -1;
          for (int k = 0; k < 64; ++k) J.qt[tq][kZigzag[k]] = (uint16_t)read16(s + o + 1 + 2 * k);
          o += 129;
        }
      }
    } else if (m == 0xDD) {                // DRI
      if (sl < 2) return -1;
      J.restart = read16(s);
    } else if (m == 0xDA) {                // SOS: the one scan of a sequential image
      if (!sof) return -1;
      J.scan_ncomp = s[0];
      if (J.scan_ncomp != J.ncomp) return 1;   // multi-scan sequential files: not handled here
      for (int k = 0; k < J.scan_ncomp; ++k) {
        const int cid = s[1 + 2 * k];
        int ci = -1;
        for (int c = 0; c < J.ncomp; ++c)
          if (J.comp[c].id == cid) ci = c;
        if (ci < 0) return -1;
        J.scan_comp[k] = ci;
        J.comp[ci].td = s[2 + 2 * k] >> 4;
        J.comp[ci].ta = s[2 + 2 * k] & 15;
        if (J.comp[ci].td > 3 || J.comp[ci].ta > 3 || !J.dc[J.comp[ci].td].present || !J.ac[J.comp[ci].ta].present)
          return -1;
      }
      J.ecs_begin = i + 2 + L;
      // the segment runs to the first marker that is not a stuffed 0xFF00 or an RSTn
      size_t e = J.ecs_begin;
      while (e + 1 < n) {
        if (d[e] == 0xFF && d[e + 1] != 0x00 && !(d[e + 1] >= 0xD0 && d[e + 1] <= 0xD7)) break;
        ++e;
      }
      J.ecs_end = e;
      break;
    }
    i += 2 + L;
  }
  if (!sof || J.ecs_end <= J.ecs_begin) return -1;
  if (J.ncomp == 1) {   // a single-component scan is not interleaved: 8x8 MCUs
    J.comp[0].h = J.comp[0].v = J.hmax = J.vmax = 1;
  }
  J.mcux = (J.width + 8 * J.hmax - 1) / (8 * J.hmax);
  J.mcuy = (J.height + 8 * J.vmax - 1) / (8 * J.vmax);
  for (int c = 0; c < J.ncomp; ++c) {
    J.comp[c].bw = J.mcux * J.comp[c].h;
    J.comp[c].bh = J.mcuy * J.comp[c].v;
  }
  return 0;
}

// ---------------------------------------------------------------------------- bitstream
struct Stream {
  std::vector<uint8_t> bytes;      // unstuffed, + kPad zero bytes (one block's worst-case read)
  std::vector<size_t> seg_bits;    // restart-interval starts (bit offsets), seg_bits[0] = 0
  size_t nbits = 0;
};

constexpr size_t kPad = 512;

void unstuff(const uint8_t* d, size_t b, size_t e, Stream& S) {
  S.bytes.resize(e - b + kPad);
  uint8_t* out = S.bytes.data();
  size_t o = 0;
  S.seg_bits.push_back(0);
  size_t i = b;
  while (i < e) {
    const uint8_t* ff = static_cast<const uint8_t*>(memchr(d + i, 0xFF, e - i));
    const size_t run = ff ? (size_t)(ff - (d + i)) : e - i;
    memcpy(out + o, d + i, run);
    o += run;
    i += run;
    if (i >= e) break;
    // d[i] == 0xFF
    if (i + 1 < e && d[i + 1] == 0x00) {
      out[o++] = 0xFF;
      i += 2;
    } else if (i + 1 < e && d[i + 1] >= 0xD0 && d[i + 1] <= 0xD7) {
      S.seg_bits.push_back(o * 8);
      i += 2;
    } else {
      out[o++] = 0xFF;
      ++i;
    }
  }
  S.nbits = o * 8;
  S.bytes.resize(o + kPad);
  memset(S.bytes.data() + o, 0, kPad);
}

inline uint64_t peek64(const uint8_t* p, size_t pos) {
  uint64_t w;
  memcpy(&w, p + (pos >> 3), 8);
  w = __builtin_bswap64(w);
  return w << (pos & 7);
}

inline int decode_slow(const Huff& h, uint64_t w, size_t& pos) {
  for (int l = kFast + 1; l <= 16; ++l) {
    const int code = (int)(w >> (64 - l));
    if (code <= h.maxcode[l]) {
      pos += l;
      return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
  }
  return -1;
}

inline int decode_sym(const Huff& h, const uint8_t* p, size_t& pos) {
  const uint64_t w = peek64(p, pos);
  const uint16_t f = h.fast[w >> (64 - kFast)];
  if (f) {
    pos += f >> 8;
    return f & 0xFF;
  }
  return decode_slow(h, w, pos);
}

inline int extend(uint32_t v, int s) { return v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v; }

inline uint32_t getbits(const uint8_t* p, size_t& pos, int s) {
  const uint32_t v = (uint32_t)(peek64(p, pos) >> (64 - s));
  pos += s;
  return v;
}

// one block (DC diff in out[0]); false on an invalid code or a coefficient run past 63
inline bool decode_block(const uint8_t* p, size_t& pos, const Huff& dc, const Huff& ac, int16_t* out) {
  memset(out, 0, 64 * sizeof(int16_t));
  int s = decode_sym(dc, p, pos);
  if (s < 0 || s > 11) return false;
  out[0] = (int16_t)(s ? extend(getbits(p, pos, s), s) : 0);
  for (int k = 1; k < 64;) {
    const uint64_t w = peek64(p, pos);
    const int32_t fa = ac.fast_ac[w >> (64 - kFast)];
    if (fa) {   // code + extra bits in the lookahead
      k += (fa >> 12) & 15;
      if (k > 63) return false;
      out[kZigzag[k]] = (int16_t)(fa >> 16);
      pos += (fa >> 4) & 31;
      ++k;
      continue;
    }
    const uint16_t f = ac.fast[w >> (64 - kFast)];
    int rs;
    if (f) {
      pos += f >> 8;
      rs = f & 0xFF;
    } else {
      rs = decode_slow(ac, w, pos);
    }
    if (rs < 0) return false;
    const int r = rs >> 4, sz = rs & 15;
    if (sz == 0) {
      if (r != 15) break;   // EOB
      k += 16;
      continue;
    }
    k += r;
    if (k > 63) return false;
    out[kZigzag[k]] = (int16_t)extend(getbits(p, pos, sz), sz);
    ++k;
  }
  return true;
}

// ---------------------------------------------------------------------------- thread pool
class Pool {
 public:
  explicit Pool(int n) { grow(n); }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() {
    std::lock_guard<std::mutex> g(mu_);
    return (int)th_.size();
  }
  // more worker threads (never fewer: another request may be inside parallel_for)
  void grow(int n) {
    std::lock_guard<std::mutex> g(mu_);
    while ((int)th_.size() < n) th_.emplace_back([this] { run(); });
  }
  // f(i) for i in [0, n), the calling thread helping; returns when all are done.  Concurrent
  // callers (several request threads) take turns.  The job state is shared-owned: a worker that
  // picked the job up late finds every index taken and leaves without touching f or this frame.
  void parallel_for(int n, const std::function<void(int)>& f) {
    std::lock_guard<std::mutex> turn(run_mu_);
    auto job = std::make_shared<Job>();
    job->n = n;
    job->f = &f;
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    work(*job);
    while (job->done.load() < n) std::this_thread::yield();
    std::lock_guard<std::mutex> g(mu_);
    job_.reset();
  }

 private:
  struct Job {
    std::atomic<int> next{0}, done{0};
    int n = 0;
    const std::function<void(int)>* f = nullptr;
  };
  static void work(Job& j) {
    for (int i; (i = j.next.fetch_add(1)) < j.n;) {
      (*j.f)(i);
      j.done.fetch_add(1);
    }
  }
  void run() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (gen_ != seen && job_); });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      work(*job);
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_mu_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

std::mutex g_pool_mu;
Pool* g_pool = nullptr;

// created with the first caller's thread count and grown when a later caller wants more
Pool& pool(int want) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  if (g_pool == nullptr) g_pool = new Pool(std::max(0, want - 1));
  else g_pool->grow(want - 1);
  return *g_pool;
}

// ---------------------------------------------------------------------------- decode
struct Layout {
  int bpm = 1;                 // blocks per MCU
  int pcomp[10], ph[10], pv[10];
  size_t plane_off[4];         // element offset of each component plane in the coefficient buffer
};

Layout make_layout(const Jpeg& J) {
  Layout L;
  int k = 0;
  for (int s = 0; s < J.scan_ncomp; ++s) {
    const int c = J.scan_comp[s];
    for (int v = 0; v < J.comp[c].v; ++v)
      for (int h = 0; h < J.comp[c].h; ++h) {
        L.pcomp[k] = c;
        L.ph[k] = h;
        L.pv[k] = v;
        ++k;
      }
  }
  L.bpm = k;
  size_t off = 0;
  for (int c = 0; c < J.ncomp; ++c) {
    L.plane_off[c] = off;
    off += (size_t)J.comp[c].bw * J.comp[c].bh * 64;
  }
  return L;
}

// decode-order block index -> its coefficient block in the planes
inline int16_t* block_ptr(const Jpeg& J, const Layout& L, int16_t* coefs, int64_t b) {
  const int64_t mcu = b / L.bpm;
  const int ph = (int)(b % L.bpm);
  const int c = L.pcomp[ph];
  const int my = (int)(mcu / J.mcux), mx = (int)(mcu % J.mcux);
  const int row = my * J.comp[c].v + L.pv[ph], col = mx * J.comp[c].h + L.ph[ph];
  return coefs + L.plane_off[c] + ((size_t)row * J.comp[c].bw + col) * 64;
}

struct Boundary {
  size_t pos;
  int phase;
  int nb;   // blocks decoded (into the chunk's buffer) before this boundary
};

struct Chunk {
  size_t start, end;
  std::vector<int16_t> blk;      // speculative blocks, 64 each
  std::vector<Boundary> marks;   // block boundaries passed
  Boundary fin{};                // first boundary at / after `end` (or where decoding stopped)
  // fix-up results
  std::vector<int16_t> pre;      // exact blocks decoded before the meeting point
  int take_from = 0, take_to = 0;   // speculative blocks [take_from, take_to) are exact
  int count = 0;                 // exact blocks this chunk contributes
  // continuation precomputed in parallel: decoding from the PREVIOUS chunk's fin state into this
  // chunk until it meets one of this chunk's marks (what the sequential fix-up would do when the
  // previous chunk ended on the exact path -- the common case)
  std::vector<int16_t> cpre;
  bool csynced = false, cfail = false;
  size_t cm = 0, cpos = 0;
  int cphase = 0;
};

void speculate(const Jpeg& J, const Layout& L, const uint8_t* p, Chunk& C, int64_t max_blocks) {
  size_t pos = C.start;
  int phase = 0;
  int16_t tmp[64];
  C.blk.reserve(((C.end - C.start) / 16 + 16) * 64);
  while (pos < C.end) {
    C.marks.push_back({pos, phase, (int)(C.blk.size() / 64)});
    if ((int64_t)(C.blk.size() / 64) >= max_blocks) break;
    const Comp& cp = J.comp[L.pcomp[phase]];
    const size_t p0 = pos;
    if (!decode_block(p, pos, J.dc[cp.td], J.ac[cp.ta], tmp)) {
      pos = p0 + 1;   // garbage: slide one bit, guess an MCU start again
      phase = 0;
      continue;
    }
    C.blk.insert(C.blk.end(), tmp, tmp + 64);
    phase = phase + 1 == L.bpm ? 0 : phase + 1;
  }
  C.fin = {pos, phase, (int)(C.blk.size() / 64)};
}

}  // namespace

extern "C" {

// info: [w, h, ncomp, hmax, vmax, restart, mcux, mcuy, (h, v, bw, bh, tq) x ncomp]
// returns 0 ok, 1 unsupported (progressive / arithmetic / 12-bit / CMYK / multi-scan), -1 malformed
int lumen_jpeg_info(const uint8_t* data, uint64_t len, int* info) {
  Jpeg J;
  const int r = parse(data, (size_t)len, J);
  if (r != 0) return r;
  info[0] = J.width; info[1] = J.height; info[2] = J.ncomp; info[3] = J.hmax; info[4] = J.vmax;
  info[5] = J.restart; info[6] = J.mcux; info[7] = J.mcuy;
  for (int c = 0; c < J.ncomp; ++c) {
    info[8 + 5 * c] = J.comp[c].h; info[9 + 5 * c] = J.comp[c].v; info[10 + 5 * c] = J.comp[c].bw;
    info[11 + 5 * c] = J.comp[c].bh; info[12 + 5 * c] = J.comp[c].tq;
  }
  return 0;
}

// Entropy-decode into coefs (sum over components of bw * bh * 64 int16, zero-filled by the caller
// is not required) and the components' quantisation tables qt [ncomp][64] (natural order).
// nthreads <= 1: sequential.  stats (nullable) [chunks, resynced, serial_blocks, total_blocks].
// Returns 0 ok, 1 unsupported, -1 malformed / truncated.
int lumen_jpeg_decode_coefs(const uint8_t* data, uint64_t len, int nthreads, int16_t* coefs, uint16_t* qt,
                            int64_t* stats) {
  Jpeg J;
  const int r = parse(data, (size_t)len, J);
  if (r != 0) return r;
  const Layout L = make_layout(J);
  for (int c = 0; c < J.ncomp; ++c) memcpy(qt + 64 * c, J.qt[J.comp[c].tq], 64 * sizeof(uint16_t));
  Stream S;
  unstuff(data, J.ecs_begin, J.ecs_end, S);
  const uint8_t* p = S.bytes.data();
  const int64_t total = (int64_t)J.mcux * J.mcuy * L.bpm;
  int64_t st[4] = {0, 0, 0, total};
  std::vector<int16_t> dcdiff;   // decode order DC differences are integrated at the end

  if (J.restart > 0 && S.seg_bits.size() > 1) {
    // restart intervals: independent segments, DC predictors reset at each
    const int nseg = (int)S.seg_bits.size();
    const int64_t per = (int64_t)J.restart * L.bpm;
    // a stream with fewer restart intervals than the frame needs would leave blocks unwritten
    // (stale coefficients of an earlier request in a reused staging buffer): reject it
    if ((int64_t)nseg * per < total) return -1;
    std::atomic<int> bad{0};
    auto seg = [&](int s) {
      size_t pos = S.seg_bits[s];
      int64_t b0 = (int64_t)s * per, b1 = std::min(total, b0 + per);
      int pred[4] = {0, 0, 0, 0};
      for (int64_t b = b0; b < b1; ++b) {
        const int ph = (int)(b % L.bpm);
        const Comp& cp = J.comp[L.pcomp[ph]];
        int16_t* out = block_ptr(J, L, coefs, b);
        if (pos > S.nbits || !decode_block(p, pos, J.dc[cp.td], J.ac[cp.ta], out)) { bad.store(1); return; }
        pred[L.pcomp[ph]] += out[0];
        out[0] = (int16_t)pred[L.pcomp[ph]];
      }
    };
    if (nthreads > 1) pool(nthreads).parallel_for(nseg, seg);
    else for (int s = 0; s < nseg; ++s) seg(s);
    st[0] = nseg;
    if (stats) memcpy(stats, st, sizeof(st));
    return bad.load() ? -1 : 0;
  }

  // no restart markers: speculative chunks + sequential fix-up + parallel placement
  const size_t nbits = S.nbits;
  int nch = nthreads > 1 ? std::min<int64_t>(4 * nthreads, (int64_t)(nbits / 4096) + 1) : 1;
  nch = std::max(nch, 1);
  std::vector<Chunk> ch(nch);
  for (int i = 0; i < nch; ++i) {
    ch[i].start = nbits * i / nch;
    ch[i].end = nbits * (i + 1) / nch;
  }
  auto spec = [&](int i) { speculate(J, L, p, ch[i], total); };
  if (nch > 1) pool(nthreads).parallel_for(nch, spec);
  else spec(0);
  // pass 2 (parallel): chunk i - 1's fin state continued into chunk i until it meets a mark there.
  // The sequential fix-up below then only stitches (it measured ~600 serially decoded blocks on a
  // 1024 x 768 noise JPEG with 64 chunks, the part that kept 16 threads no faster than 4).
  auto cont = [&](int i) {
    if (i == 0) return;
    Chunk& C = ch[i];
    const Chunk& P = ch[i - 1];
    size_t cpos = P.fin.pos, m = 0;
    int cphase = P.fin.phase;
    int16_t t64[64];
    for (;;) {
      while (m < C.marks.size() && C.marks[m].pos < cpos) ++m;
      if (m < C.marks.size() && C.marks[m].pos == cpos && C.marks[m].phase == cphase) { C.csynced = true; break; }
      if (cpos >= C.end || (int64_t)(C.cpre.size() / 64) >= total) break;
      const Comp& cp = J.comp[L.pcomp[cphase]];
      if (!decode_block(p, cpos, J.dc[cp.td], J.ac[cp.ta], t64)) { C.cfail = true; break; }
      C.cpre.insert(C.cpre.end(), t64, t64 + 64);
      cphase = cphase + 1 == L.bpm ? 0 : cphase + 1;
    }
    C.cm = m;
    C.cpos = cpos;
    C.cphase = cphase;
  };
  if (nch > 1) pool(nthreads).parallel_for(nch, cont);
  // chunk 0 started at the true start: exact as it stands
  ch[0].take_from = 0;
  ch[0].take_to = ch[0].fin.nb;
  ch[0].count = ch[0].fin.nb;
  size_t pos = ch[0].fin.pos;
  int phase = ch[0].fin.phase;
  int64_t done = ch[0].count;
  int16_t tmp[64];
  for (int i = 1; i < nch && done < total; ++i) {
    Chunk& C = ch[i];
    const Chunk& Pv = ch[i - 1];
    if (pos == Pv.fin.pos && phase == Pv.fin.phase && !C.cfail) {
      // entering exactly where the precomputed continuation started: take it
      const int64_t npre = (int64_t)(C.cpre.size() / 64);
      const int64_t k = std::min<int64_t>(npre, total - done);
      C.pre.assign(C.cpre.begin(), C.cpre.begin() + 64 * k);
      done += k;
      st[2] += k;
      if (k == npre && C.csynced && done < total) {
        ++st[1];
        C.take_from = C.marks[C.cm].nb;
        C.take_to = C.fin.nb;
        const int64_t room = total - done;
        if (C.take_to - C.take_from > room) C.take_to = C.take_from + (int)room;
        done += C.take_to - C.take_from;
        pos = C.fin.pos;
        phase = C.fin.phase;
      } else {
        pos = C.cpos;
        phase = C.cphase;
      }
      C.count = (int)(C.pre.size() / 64) + (C.take_to - C.take_from);
      continue;
    }
    size_t m = 0;   // first mark at / after pos
    while (m < C.marks.size() && C.marks[m].pos < pos) ++m;
    bool synced = false;
    for (;;) {
      while (m < C.marks.size() && C.marks[m].pos < pos) ++m;
      if (m < C.marks.size() && C.marks[m].pos == pos && C.marks[m].phase == phase) { synced = true; break; }
      if (pos >= C.end || done >= total) break;
      const Comp& cp = J.comp[L.pcomp[phase]];
      if (!decode_block(p, pos, J.dc[cp.td], J.ac[cp.ta], tmp)) return -1;   // the exact decode failed
      C.pre.insert(C.pre.end(), tmp, tmp + 64);
      ++done;
      phase = phase + 1 == L.bpm ? 0 : phase + 1;
      ++st[2];
    }
    if (synced) {
      ++st[1];
      C.take_from = C.marks[m].nb;
      C.take_to = C.fin.nb;
      const int64_t room = total - done;
      if (C.take_to - C.take_from > room) C.take_to = C.take_from + (int)room;
      done += C.take_to - C.take_from;
      pos = C.fin.pos;
      phase = C.fin.phase;
    }
    C.count = (int)(C.pre.size() / 64) + (C.take_to - C.take_from);
  }
  // blocks past the last chunk (should not happen: the last chunk ends at the stream's end)
  std::vector<int16_t> tail;
  while (done < total) {
    if (pos >= nbits) return -1;
    const Comp& cp = J.comp[L.pcomp[phase]];
    if (!decode_block(p, pos, J.dc[cp.td], J.ac[cp.ta], tmp)) return -1;
    tail.insert(tail.end(), tmp, tmp + 64);
    ++done;
    phase = phase + 1 == L.bpm ? 0 : phase + 1;
    ++st[2];
  }
  // placement with chunk-local DC integration (parallel), the chunks' DC offsets (sequential, one
  // add per chunk and component), then the offsets applied (parallel).  The former sequential DC
  // pass over every block ran cache-cold after a parallel placement: ~180 of ~520 us on the GPU
  // box at 8 threads (profiles/r6_jpeg_host_phases_v1.txt).
  std::vector<int64_t> base(nch + 1, 0);
  for (int i = 0; i < nch; ++i) base[i + 1] = base[i] + ch[i].count;
  const int64_t tail0 = base[nch];
  std::vector<std::array<int, 4>> dsum(nch + 1, std::array<int, 4>{0, 0, 0, 0});
  auto place = [&](int i) {
    const Chunk& C = ch[i];
    int64_t b = base[i];
    int acc[4] = {0, 0, 0, 0};
    auto put = [&](const int16_t* src) {
      const int c = L.pcomp[b % L.bpm];
      int16_t* out = block_ptr(J, L, coefs, b);
      memcpy(out, src, 128);
      acc[c] += out[0];
      out[0] = (int16_t)acc[c];
      ++b;
    };
    const int npre = (int)(C.pre.size() / 64);
    for (int k = 0; k < npre; ++k) put(&C.pre[64 * k]);
    for (int k = C.take_from; k < C.take_to; ++k) put(&C.blk[64 * (size_t)k]);
    for (int c = 0; c < 4; ++c) dsum[i][c] = acc[c];
  };
  if (nch > 1) pool(nthreads).parallel_for(nch, place);
  else place(0);
  // DC offset entering chunk i = the sum of every earlier chunk's DC differences (int wrap-around as
  // in the sequential form: the final int16 store keeps the low 16 bits either way)
  std::vector<std::array<int, 4>> off(nch + 1, std::array<int, 4>{0, 0, 0, 0});
  for (int i = 0; i < nch; ++i)
    for (int c = 0; c < 4; ++c) off[i + 1][c] = off[i][c] + dsum[i][c];
  auto shift = [&](int i) {
    const std::array<int, 4>& o = off[i];
    if (o[0] == 0 && o[1] == 0 && o[2] == 0 && o[3] == 0) return;
    for (int64_t b = base[i]; b < base[i + 1]; ++b) {
      int16_t* out = block_ptr(J, L, coefs, b);
      out[0] = (int16_t)(out[0] + o[L.pcomp[b % L.bpm]]);
    }
  };
  if (nch > 1) pool(nthreads).parallel_for(nch, shift);
  int pred[4];
  for (int c = 0; c < 4; ++c) pred[c] = off[nch][c];
  for (size_t k = 0; k < tail.size() / 64; ++k) {
    const int64_t b = tail0 + (int64_t)k;
    const int c = L.pcomp[b % L.bpm];
    int16_t* out = block_ptr(J, L, coefs, b);
    memcpy(out, &tail[64 * k], 128);
    pred[c] += out[0];
    out[0] = (int16_t)pred[c];
  }
  st[0] = nch;
  if (stats) memcpy(stats, st, sizeof(st));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------- GPU entropy decode
// The preparation the GPU decoder (csrc/jpeg_huff.hip) needs from the host: header parse, the
// Huffman tables (same fast tables as above), byte unstuffing and the restart-interval starts,
// written as one descriptor + stream into the caller's (pinned) upload buffer.  O(bytes) memchr /
// memcpy work: ~20 us for a 1024 x 768 photo against ~1.5-3 ms for the entropy decode itself.
namespace {

void copy_dc(lumen::JHuffDc& d, const Huff& h) {
  memcpy(d.fast, h.fast, sizeof(d.fast));
  memcpy(d.maxcode, h.maxcode, sizeof(d.maxcode));
  memcpy(d.valptr, h.valptr, sizeof(d.valptr));
  memcpy(d.mincode, h.mincode, sizeof(d.mincode));
  memcpy(d.vals, h.vals, sizeof(d.vals));
}

void copy_ac(lumen::JHuffAc& d, const Huff& h) {
  memcpy(d.fast, h.fast, sizeof(d.fast));
  memcpy(d.fast_ac, h.fast_ac, sizeof(d.fast_ac));
  memcpy(d.maxcode, h.maxcode, sizeof(d.maxcode));
  memcpy(d.valptr, h.valptr, sizeof(d.valptr));
  memcpy(d.mincode, h.mincode, sizeof(d.mincode));
  memcpy(d.vals, h.vals, sizeof(d.vals));
}

}  // namespace

extern "C" {

int lumen_jpeg_desc_bytes() { return (int)sizeof(lumen::JHuffDesc); }

// Descriptor + stream of one baseline JPEG into out[0, cap) (out 16-byte aligned), its quantisation
// tables into qt [ncomp][64] (natural order), split for <= max_lanes decoding lanes (the GPU
// spreads them over max_lanes / 256 workgroups).  *need = bytes the entry takes.  Returns 0 ok,
// 1 unsupported, -1 malformed, 2 cap too small (nothing usable written; retry with *need).
int lumen_jpeg_prepare_gpu(const uint8_t* data, uint64_t len, uint8_t* out, int64_t cap, uint16_t* qt,
                           int64_t* need, int max_lanes) {
  Jpeg J;
  const int r = parse(data, (size_t)len, J);
  if (r != 0) return r;
  const Layout L = make_layout(J);
  const int64_t total = (int64_t)J.mcux * J.mcuy * L.bpm;
  const size_t ecs = J.ecs_end - J.ecs_begin;
  if (ecs >= ((size_t)1 << 25) || total >= ((int64_t)1 << 31)) return 1;   // 28-bit bit offsets on the GPU
  const int64_t dsz = (int64_t)((sizeof(lumen::JHuffDesc) + 255) & ~(size_t)255);
  const int64_t stream_cap = (int64_t)((ecs + 64 + 3) & ~(size_t)3);
  *need = dsz + stream_cap;
  if (*need > cap) return 2;
  for (int c = 0; c < J.ncomp; ++c) memcpy(qt + 64 * c, J.qt[J.comp[c].tq], 64 * sizeof(uint16_t));
  auto* Dd = reinterpret_cast<lumen::JHuffDesc*>(out);
  memset(Dd, 0, sizeof(*Dd));
  lumen::JHuffHead* D = &Dd->h;
  // unstuff straight into the upload buffer (as unstuff() above)
  uint8_t* st = out + dsz;
  std::vector<int32_t> segs{0};
  size_t o = 0, i = J.ecs_begin;
  const size_t e = J.ecs_end;
  while (i < e) {
    const uint8_t* ff = static_cast<const uint8_t*>(memchr(data + i, 0xFF, e - i));
    const size_t run = ff ? (size_t)(ff - (data + i)) : e - i;
    memcpy(st + o, data + i, run);
    o += run;
    i += run;
    if (i >= e) break;
    if (i + 1 < e && data[i + 1] == 0x00) {
      st[o++] = 0xFF;
      i += 2;
    } else if (i + 1 < e && data[i + 1] >= 0xD0 && data[i + 1] <= 0xD7) {
      segs.push_back((int32_t)(o * 8));
      i += 2;
    } else {
      st[o++] = 0xFF;
      ++i;
    }
  }
  const size_t words = (o + 64 + 3) / 4;
  memset(st + o, 0, words * 4 - o);
  // 32-bit words, big-endian within each word: the GPU byte-swaps on load
  D->nbits = (int32_t)(o * 8);
  D->nwords = (int32_t)words;
  D->total = (int32_t)total;
  D->bpm = L.bpm;
  D->ncomp = J.ncomp;
  D->mcux = J.mcux;
  D->stream_off = (int32_t)dsz;
  if (J.restart > 0 && segs.size() > 1) {
    const int64_t per = (int64_t)J.restart * L.bpm;
    const int nseg = (int)segs.size();
    if ((int64_t)nseg * per < total) return -1;   // fewer intervals than the frame needs
    const int64_t seg_off = dsz + (int64_t)words * 4;
    *need = seg_off + 4 * (int64_t)nseg;
    if (*need > cap) return 2;
    memcpy(out + seg_off, segs.data(), 4 * (size_t)nseg);
    D->restart_blocks = (int32_t)per;
    D->nseg = nseg;
    D->seg_off = (int32_t)seg_off;
  } else {
    *need = dsz + (int64_t)words * 4;
  }
  // synchronising decode: <= max_lanes subsequences of >= 128 bits
  const int64_t nb = std::max<int64_t>(D->nbits, 1);
  const int64_t lanes = std::min<int64_t>(std::max(max_lanes, lumen::kJHuffWgLanes), lumen::kJHuffMaxLanes);
  int64_t sub = std::max<int64_t>(128, (nb + lanes - 1) / lanes);
  sub = (sub + 31) & ~(int64_t)31;
  D->sub_bits = (int32_t)sub;
  D->nsub = (int32_t)((nb + sub - 1) / sub);
  // tables: one slot per distinct (class, id) the scan uses
  int dmap[4] = {-1, -1, -1, -1}, amap[4] = {-1, -1, -1, -1};
  for (int k = 0; k < L.bpm; ++k) {
    const Comp& cp = J.comp[L.pcomp[k]];
    if (dmap[cp.td] < 0) {
      dmap[cp.td] = D->ndc++;
      copy_dc(Dd->dc[dmap[cp.td]], J.dc[cp.td]);
    }
    if (amap[cp.ta] < 0) {
      amap[cp.ta] = D->nac++;
      copy_ac(Dd->ac[amap[cp.ta]], J.ac[cp.ta]);
    }
    D->pcomp[k] = L.pcomp[k];
    D->px[k] = L.ph[k];
    D->py[k] = L.pv[k];
    D->pdc[k] = dmap[cp.td];
    D->pac[k] = amap[cp.ta];
  }
  for (int c = 0; c < J.ncomp; ++c) {
    D->bw[c] = J.comp[c].bw;
    D->hh[c] = J.comp[c].h;
    D->vv[c] = J.comp[c].v;
    D->plane_off[c] = (int64_t)L.plane_off[c];
  }
  return 0;
}

// The GPU decoder's schedule run sequentially on the host (csrc/jpeg_huff.hip:jpeg_huff_kernel,
// lane by lane, round by round, the same per-lane code from jpeg_huff_core.h): the CPU-side
// oracle of the kernel's synchronisation / prefix-sum / placement logic.  Same blob, coefficient
// and err ([2n]: malformed flag, rounds) conventions as the kernel.
// stats (nullable) [4]: round-0 slides and blocks summed over the lanes, the most slides of a lane,
// the lanes
int lumen_jpeg_gpu_emulate(const uint8_t* blob, int n, int16_t* coefs, int32_t* err, int64_t* stats) {
  uint8_t zz[64];
  for (int k = 0; k < 64; ++k) zz[k] = (uint8_t)kZigzag[k];
  for (int img = 0; img < n; ++img) {
    const lumen::JHuffJob job = reinterpret_cast<const lumen::JHuffJob*>(blob)[img];
    const uint8_t* dp = blob + job.desc_off;
    const auto* D = reinterpret_cast<const lumen::JHuffDesc*>(dp);
    const lumen::JHuffHead& H = D->h;
    const lumen::jh::SrcMem w{reinterpret_cast<const uint32_t*>(dp + H.stream_off), (uint32_t)H.nwords};
    int16_t* co = coefs + job.coef_off;
    memset(co, 0, (size_t)H.total * 64 * sizeof(int16_t));   // as the kernel's launcher
    int bad = 0, rounds = 0;
    if (H.restart_blocks > 0) {
      const int32_t* segs = reinterpret_cast<const int32_t*>(dp + H.seg_off);
      for (int sg = 0; sg < H.nseg; ++sg)
        if (!lumen::jh::write_interval(H, D->dc, D->ac, w, segs, sg, co, zz)) bad = 1;
      err[2 * img] = bad;
      err[2 * img + 1] = 0;
      continue;
    }
    const int nsub = H.nsub;
    const uint32_t sub = (uint32_t)H.sub_bits;
    constexpr int kCap = 16;   // jpeg_huff.hip kMarkCap
    std::vector<uint32_t> epos(nsub);
    std::vector<int> eph(nsub, 0), dirty(nsub, 0);
    std::vector<lumen::jh::Span> sp(nsub), s0(nsub);
    std::vector<lumen::jh::Mark> marks((size_t)nsub * kCap);
    std::vector<uint32_t> keys((size_t)nsub * kCap);
    for (int i = 0; i < nsub; ++i) epos[i] = (uint32_t)i * sub;
    bool chg = false;
    for (int i = 0; i < nsub; ++i) {   // round 0: guesses, recording marks
      s0[i] = lumen::jh::run_span<lumen::jh::kRecord>(H, D->dc, D->ac, w, (uint32_t)i * sub, 0, (uint32_t)(i + 1) * sub,
                                                      zz, &keys[(size_t)i * kCap], 1, &marks[(size_t)i * kCap], kCap);
      sp[i] = s0[i];
      if (stats) {
        stats[0] += s0[i].slides;
        stats[1] += s0[i].n;
        stats[2] = std::max<int64_t>(stats[2], s0[i].slides);
        stats[3] += 1;
      }
    }
    for (int i = 0; i + 1 < nsub; ++i)
      if (sp[i].pos != epos[i + 1] || sp[i].phase != eph[i + 1]) {
        epos[i + 1] = sp[i].pos;
        eph[i + 1] = sp[i].phase;
        dirty[i + 1] = 1;
        chg = true;
      }
    rounds = 1;
    for (int r = 1; chg && r <= nsub + 1; ++r) {
      const std::vector<uint32_t> p0 = epos;
      const std::vector<int> ph0 = eph, d0 = dirty;
      std::fill(dirty.begin(), dirty.end(), 0);
      chg = false;
      for (int i = 0; i < nsub; ++i) {
        if (!d0[i]) continue;
        const uint32_t end = (uint32_t)(i + 1) * sub;
        sp[i] = i + 1 < nsub ? lumen::jh::run_span<lumen::jh::kSync>(H, D->dc, D->ac, w, p0[i], ph0[i], end, zz,
                                                                     &keys[(size_t)i * kCap], 1,
                                                                     &marks[(size_t)i * kCap], 0, &s0[i])
                             : lumen::jh::run_span<lumen::jh::kPlain>(H, D->dc, D->ac, w, p0[i], ph0[i], end, zz);
        if (i + 1 < nsub && (sp[i].pos != epos[i + 1] || sp[i].phase != eph[i + 1])) {
          epos[i + 1] = sp[i].pos;
          eph[i + 1] = sp[i].phase;
          dirty[i + 1] = 1;
          chg = true;
        }
      }
      rounds = r + 1;
    }
    int64_t base = 0, a0 = 0, a1 = 0, a2 = 0;
    for (int i = 0; i < nsub; ++i) {
      if (sp[i].good < sp[i].n && base + sp[i].good < H.total) bad = 1;
      if (i == nsub - 1 && base + sp[i].n < H.total) bad = 1;
      if (base < H.total &&
          !lumen::jh::write_span(H, D->dc, D->ac, w, epos[i], eph[i], (uint32_t)(i + 1) * sub, base, (int)a0, (int)a1,
                                 (int)a2, co, zz))
        bad = 1;
      base += sp[i].n;
      a0 += sp[i].d0;
      a1 += sp[i].d1;
      a2 += sp[i].d2;
    }
    err[2 * img] = bad;
    err[2 * img + 1] = rounds;
  }
  return 0;
}

}  // extern "C"
