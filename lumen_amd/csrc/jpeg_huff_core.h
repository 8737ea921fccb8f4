// Per-lane pieces of the GPU baseline-JPEG entropy decoder, shared by the kernel
// (csrc/jpeg_huff.hip) and its sequential host emulation (csrc/host/jpeg_decode.cpp:
// lumen_jpeg_gpu_emulate, the CPU test oracle of the kernel's schedule).  Plain C++ plus the
// host/device qualifier, so the g++-built host library compiles the same code.
//
// Decoding model (lane i of an image owns subsequence i = bits [i*SUB, (i+1)*SUB)):
//   entry state of lane i = (bit position, block phase inside the MCU) of the first block
//   boundary at / after i*SUB on the TRUE decode path.  Lane 0's is (0, 0).  Every lane decodes
//   whole blocks from its current entry until it passes its subsequence end; that exit is lane
//   i+1's next entry.  Starting from guesses (i*SUB, 0) the entries converge: an exact entry gives
//   an exact exit, and a lane whose guess-decode has re-synchronised with the true block
//   boundaries (Huffman codes self-synchronise) produces the same exit from the exact entry,
//   so the iteration stops once no exit changes -- usually after a few rounds.  Then block counts
//   and per-component DC-difference sums are prefix-summed and every lane re-decodes its span
//   writing de-zigzagged coefficients with the DC integrated (the host decoder's output layout).
// Restart-interval JPEGs need none of that: each interval is independent.
#pragma once
#include <cstdint>
#include <cstring>

#include "jpeg_huff.h"

#ifdef __HIPCC__
#define JH_FN __host__ __device__ __forceinline__
#else
#define JH_FN inline
#endif

namespace lumen {
namespace jh {

// Where the stream words come from: global memory (SrcMem: w[0, nw), zero past the end) or a
// window of them staged in LDS (SrcLds: words [w0, w0 + wn), zero elsewhere -- the kernel stages
// every word its lanes can reach: a span ends at most one block past its end).
struct SrcMem {
  const uint32_t* w;
  uint32_t nw;
  JH_FN uint32_t load(uint32_t i) const { return i < nw ? __builtin_bswap32(w[i]) : 0u; }
};

struct SrcLds {
  const uint32_t* lw;
  uint32_t w0, wn;
  JH_FN uint32_t load(uint32_t i) const {
    const uint32_t j = i - w0;
    return j < wn ? __builtin_bswap32(lw[j]) : 0u;
  }
};

template <class S>
struct Bits {
  S s;
  uint32_t pos;
  uint32_t ci;    // word index of cur's high half
  uint64_t cur;   // words ci, ci + 1 (big-endian bit order)
};

template <class S>
JH_FN void bits_init(Bits<S>& b, const S& src, uint32_t pos) {
  b.s = src;
  b.pos = pos;
  b.ci = pos >> 5;
  b.cur = ((uint64_t)src.load(b.ci) << 32) | src.load(b.ci + 1);
}

// the next 32 bits at pos, MSB first
template <class S>
JH_FN uint32_t peek(Bits<S>& b) {
  const uint32_t i = b.pos >> 5;
  if (i != b.ci) {
    b.cur = i == b.ci + 1 ? (b.cur << 32) | b.s.load(i + 1) : ((uint64_t)b.s.load(i) << 32) | b.s.load(i + 1);
    b.ci = i;
  }
  return (uint32_t)((b.cur << (b.pos & 31)) >> 32);
}

JH_FN int extend(uint32_t v, int s) { return v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v; }

// codes longer than the lookahead: (symbol, length) or symbol -1
template <class T>
JH_FN int slow_sym(const T& t, uint32_t x, int& len) {
  for (int l = kJHuffFast + 1; l <= 16; ++l) {
    const int code = (int)(x >> (32 - l));
    if (code <= t.maxcode[l]) {
      len = l;
      return t.vals[(t.valptr[l] + code - t.mincode[l]) & 255];
    }
  }
  return -1;
}

struct Span {
  uint32_t pos;      // exit: first block boundary at / after the subsequence end
  int32_t phase;
  int32_t n;         // blocks decoded
  int32_t good;      // blocks decoded before the first invalid code (n when none)
  int32_t slides;    // invalid codes met (each slid one bit)
  int32_t nmk;       // marks recorded (MARKS mode)
  int32_t d0, d1, d2;   // DC-difference sums per component
};

// A point of a decode path: the state at the start of a block (after `n` blocks, `slides` invalid
// codes and the DC sums so far).  Two decodes that reach the same (pos, phase) continue
// identically, so a re-decode that meets a mark of an earlier decode can take that decode's
// remaining result instead of decoding on.  The (pos << 4 | phase) keys are kept apart from the
// rest (the kernel holds the keys in LDS, the totals in global memory).
struct Mark {
  int32_t n, slides;
  int32_t d0, d1, d2, pad_[3];
};

JH_FN uint32_t mark_key(uint32_t pos, int phase) { return (pos << 4) | (uint32_t)phase; }

// a[c] += v for a component index c (selects, not a runtime-indexed array: that would live in
// scratch on the GPU)
JH_FN void add3(int32_t& a0, int32_t& a1, int32_t& a2, int c, int v) {
  a0 += c == 0 ? v : 0;
  a1 += c == 1 ? v : 0;
  a2 += c == 2 ? v : 0;
}

JH_FN int pick3(int a0, int a1, int a2, int c) { return c == 0 ? a0 : (c == 1 ? a1 : a2); }

// element offset of decode-order block blk in the image's coefficient planes
JH_FN int64_t block_off(const JHuffHead& H, int64_t blk) {
  const int64_t mcu = blk / H.bpm;
  const int p = (int)(blk - mcu * H.bpm);
  const int c = H.pcomp[p];
  const int64_t my = mcu / H.mcux, mx = mcu - my * H.mcux;
  const int64_t row = my * H.vv[c] + H.py[p], col = mx * H.hh[c] + H.px[p];
  return H.plane_off[c] + (row * H.bw[c] + col) * 64;
}

enum SpanMode { kPlain = 0, kRecord = 1, kSync = 2, kWrite = 3 };

// The symbol-at-a-time decoder every lane runs.  One loop iteration decodes ONE Huffman symbol
// (a DC difference or an AC run/level, with its extra bits) whatever the lane's position in its
// block: lanes of a wave stay in lock-step (the block-at-a-time form nests a coefficient loop in
// a block loop, and a wave then runs the longest lane's block at every step).
//
// Path points are block starts.  Decoding stops at the first one at / after `end` (or the stream's
// end, or block blk_end in kWrite).  An invalid code (a guessed entry that is not a true block
// boundary) slides one bit and guesses an MCU start again, as the host decoder's speculative pass
// does; in kWrite it is an error (returns r.good = -2).
//   kRecord: the first `cap` path points are stored: keys mkey[j * kstride], totals mk[j]
//   kSync:   at each path point the keys of an earlier decode (prev, its nmk marks) are checked;
//            on a meeting the result is completed from prev's totals without decoding further
//   kWrite:  blocks blk.. are written (coefficients into pre-zeroed planes, DC integrated from
//            the predictors p0..p2)
template <int MODE, class S>
JH_FN Span run_span(const JHuffHead& H, const JHuffDc* dc, const JHuffAc* ac, const S& w, uint32_t pos,
                    int phase, uint32_t end, const uint8_t* zz, uint32_t* mkey = nullptr, int kstride = 1,
                    Mark* mk = nullptr, int cap = 0, const Span* prev = nullptr, int64_t blk = 0,
                    int64_t blk_end = 0, int p0 = 0, int p1 = 0, int p2 = 0, int16_t* coefs = nullptr) {
  Bits<S> b;
  bits_init(b, w, pos);
  Span r{pos, phase, 0, -1, 0, 0, 0, 0, 0};
  const uint32_t nbits = (uint32_t)H.nbits;
  // >= 2 bits per block, 1 per slide; <= 64 symbols per block
  const int guard = MODE == kWrite ? 0x7fffffff : 64 * (2 * H.sub_bits + 64);
  int m = 0;
  const int nmk = MODE == kSync ? prev->nmk : 0;
  uint32_t key_m = MODE == kSync && nmk > 0 ? mkey[0] : 0xFFFFFFFFu;
  int k = 0;                    // next coefficient of the current block (0: its DC)
  uint32_t bstart = pos;        // start of the current block
  int diff = 0;                 // the block's DC difference
  int comp = H.pcomp[phase];
  const JHuffDc* tdc = &dc[H.pdc[phase]];
  const JHuffAc* tac = &ac[H.pac[phase]];
  int16_t* out = nullptr;
  for (int it = 0; it < guard; ++it) {
    if (k == 0) {   // a path point
      if (b.pos >= end || b.pos >= nbits) break;
      if (MODE == kWrite && blk >= blk_end) break;
      if (MODE == kRecord && r.nmk < cap) {
        mkey[r.nmk * kstride] = mark_key(b.pos, phase);
        Mark& mm = mk[r.nmk++];
        mm.n = r.n;
        mm.slides = r.slides;
        mm.d0 = r.d0;
        mm.d1 = r.d1;
        mm.d2 = r.d2;
      }
      if (MODE == kSync) {
        while (m < nmk && (key_m >> 4) < b.pos) {
          ++m;
          key_m = m < nmk ? mkey[m * kstride] : 0xFFFFFFFFu;
        }
        if (m < nmk && key_m == mark_key(b.pos, phase)) {
          const Mark q = mk[m];
          // the first invalid code of the taken suffix (at its start when it came before the mark
          // and a later one exists: conservative, only malformed streams have any on the exact path)
          if (r.good < 0 && prev->slides > q.slides) r.good = r.n + (prev->good >= q.n ? prev->good - q.n : 0);
          r.n += prev->n - q.n;
          r.slides += prev->slides - q.slides;
          r.d0 += prev->d0 - q.d0;
          r.d1 += prev->d1 - q.d1;
          r.d2 += prev->d2 - q.d2;
          if (r.good < 0) r.good = r.n;
          r.pos = prev->pos;
          r.phase = prev->phase;
          r.nmk = prev->nmk;
          return r;
        }
      }
      if (MODE == kWrite) out = coefs + block_off(H, blk);
      bstart = b.pos;
    }
    const uint32_t x = peek(b);
    const uint32_t idx = x >> (32 - kJHuffFast);
    bool bad = false, done = false;
    if (k == 0) {                                   // DC: size category + its extra bits
      const uint16_t f = tdc->fast[idx];
      int len = f >> 8, s = f & 0xFF;
      if (!f) s = slow_sym(*tdc, x, len);
      bad = s < 0 || s > 11;
      if (!bad) {
        diff = s ? extend((x << len) >> (32 - s), s) : 0;
        b.pos += len + s;
        k = 1;
      }
    } else {
      const int32_t fa = tac->fast_ac[idx];
      if (fa) {                                     // code + extra bits inside the lookahead
        k += (fa >> 12) & 15;
        bad = k > 63;
        if (!bad) {
          if (MODE == kWrite) out[zz[k]] = (int16_t)(fa >> 16);
          b.pos += (fa >> 4) & 31;
          ++k;
          done = k >= 64;
        }
      } else {
        const uint16_t f = tac->fast[idx];
        int len = f >> 8, rs = f & 0xFF;
        if (!f) rs = slow_sym(*tac, x, len);
        bad = rs < 0;
        if (!bad) {
          const int run = rs >> 4, sz = rs & 15;
          if (sz == 0) {
            b.pos += len;
            if (run != 15) {
              done = true;                          // EOB
            } else {
              k += 16;                              // ZRL
              done = k >= 64;
            }
          } else {
            k += run;
            bad = k > 63;
            if (!bad) {
              if (MODE == kWrite) out[zz[k]] = (int16_t)extend((x << len) >> (32 - sz), sz);
              b.pos += len + sz;
              ++k;
              done = k >= 64;
            }
          }
        }
      }
    }
    if (bad) {
      if (MODE == kWrite) {
        r.good = -2;
        break;
      }
      if (r.good < 0) r.good = r.n;
      ++r.slides;
      b.pos = bstart + 1;
      phase = 0;
      k = 0;
    } else if (done) {                              // block complete
      ++r.n;
      add3(r.d0, r.d1, r.d2, comp, diff);
      if (MODE == kWrite) {
        add3(p0, p1, p2, comp, diff);
        out[0] = (int16_t)pick3(p0, p1, p2, comp);
        ++blk;
      }
      phase = phase + 1 == H.bpm ? 0 : phase + 1;
      k = 0;
    } else {
      continue;
    }
    comp = H.pcomp[phase];
    tdc = &dc[H.pdc[phase]];
    tac = &ac[H.pac[phase]];
  }
  if (r.good == -1) r.good = r.n;
  r.pos = b.pos;
  r.phase = phase;
  if (MODE == kSync) r.nmk = prev->nmk;
  return r;
}

// the exact decode of blocks [blk, total) from an exact (pos, phase) until the position passes
// `end`, DC predictors starting at (p0, p1, p2), into pre-zeroed planes; false on an invalid code
template <class S>
JH_FN bool write_span(const JHuffHead& H, const JHuffDc* dc, const JHuffAc* ac, const S& w, uint32_t pos,
                      int phase, uint32_t end, int64_t blk, int p0, int p1, int p2, int16_t* coefs,
                      const uint8_t* zz) {
  const Span r = run_span<kWrite>(H, dc, ac, w, pos, phase, end, zz, nullptr, 1, nullptr, 0, nullptr, blk, H.total,
                                  p0, p1, p2, coefs);
  return r.good != -2;
}

// restart interval s: blocks [s * per, min(total, (s + 1) * per)) from the interval's start, into
// pre-zeroed planes; false on an invalid code or an interval overrunning the next one's start
template <class S>
JH_FN bool write_interval(const JHuffHead& H, const JHuffDc* dc, const JHuffAc* ac, const S& w,
                          const int32_t* segs, int s, int16_t* coefs, const uint8_t* zz) {
  const int64_t per = H.restart_blocks;
  const int64_t b0 = (int64_t)s * per;
  const int64_t b1 = b0 + per < H.total ? b0 + per : H.total;
  if (b0 >= b1) return true;
  const uint32_t end = s + 1 < H.nseg ? (uint32_t)segs[s + 1] : (uint32_t)H.nbits;
  const uint32_t start = (uint32_t)segs[s];
  const int phase = (int)(b0 % H.bpm);
  const Span r = run_span<kWrite>(H, dc, ac, w, start, phase, 0xFFFFFFFFu, zz, nullptr, 1, nullptr, 0, nullptr, b0, b1,
                                  0, 0, 0, coefs);
  return r.good != -2 && r.n == b1 - b0 && r.pos <= end;
}

}  // namespace jh
}  // namespace lumen
