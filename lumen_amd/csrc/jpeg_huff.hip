// Baseline-JPEG entropy decode on the GPU: one 1024-lane workgroup per image, every lane a
// serial Huffman decoder over its own <= 1/1024 of the bitstream, synchronised by iterating the
// lanes' entry states to the fixed point (the scheme and the per-lane code: jpeg_huff_core.h).
// Replaces the host entropy decode (csrc/host/jpeg_decode.cpp, ~1.5 ms for a 1024 x 768 photo on
// the request's critical path; the reference runs libjpeg via Pillow on one CPU thread,
// packages/lumen-vlm/src/lumen_vlm/backends/onnxrt_backend.py:661-665): the host only parses the
// header and unstuffs the bytes; the coefficient planes this kernel writes feed the existing
// IDCT / colour kernels (csrc/jpeg.hip) unchanged.
//
// An image's lanes (<= 4096) are spread over up to 16 workgroups of 256 (one wave per SIMD: the
// serial decode is issue-bound, so a lone image uses 16 CUs, not one), which meet at a global
// per-image barrier between rounds; a batch of images is one launch with the lane count per image
// chosen so that every workgroup is co-resident (images x workgroups <= CUs).  LDS: the descriptor
// with its Huffman tables (27 KB) + the workgroup's window of the stream.
#include "common.h"
#include "jpeg_huff_core.h"

namespace lumen {

__constant__ uint8_t kJpegZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                        12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                        35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                        58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int kWg = kJHuffWgLanes;      // 256 lanes = 4 waves = one wave per SIMD
constexpr int kMarkCap = 16;            // path points recorded per lane by the speculative round
constexpr int kExtraWords = 256;        // window words past a workgroup's last subsequence (8 Kbit)
constexpr int kMaxWindowWords = 24 * 1024;

// Global per-image state of the cross-workgroup rounds (zeroed before the launch).  An entry is
// (bit position << 4) | block phase in one word, so a lane never sees half of a neighbour's update.
struct HuffImgState {
  uint32_t bar;                          // barrier arrivals
  int32_t pad_[3];
  int32_t wsum[kJHuffMaxLanes / kWg][4]; // per-workgroup totals of the prefix sums
  int32_t chg[kJHuffMaxLanes + 4];       // round r changed an entry
  uint32_t entry[kJHuffMaxLanes];
};

__device__ __forceinline__ uint32_t ld_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_acq(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// barrier over the G workgroups of one image (all co-resident: the launcher keeps images x G <= CUs)
__device__ __forceinline__ void img_barrier(uint32_t* bar, int G, uint32_t& gen) {
  __threadfence();
  __syncthreads();
  ++gen;
  if (G > 1 && threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = gen * (uint32_t)G;
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t pack(uint32_t pos, int phase) { return (pos << 4) | (uint32_t)phase; }

// The lanes of one workgroup: round 0, the synchronisation rounds, the prefix sums and the write
// pass (see jpeg_huff_core.h for the scheme).
template <class Src>
__device__ __forceinline__ void huff_lanes(const JHuffDesc& sd, const Src& src, int16_t* co, HuffImgState* st,
                                           jh::Mark* marks, int lanes_stride, const uint8_t* zz, int32_t* s_err,
                                           int32_t (*wtot)[4], uint32_t* mkeys, int32_t* err, int64_t* tick) {
  const int tid = threadIdx.x, g = blockIdx.x, img = blockIdx.y;
  const bool tk = tick != nullptr && g == 0 && tid == 0;
  if (tk) tick[1] = wall_clock64();
  const JHuffHead& H = sd.h;
  const int nsub = H.nsub;
  const int G = (nsub + kWg - 1) / kWg;
  const uint32_t sub = (uint32_t)H.sub_bits;
  HuffImgState& S = *st;
  uint32_t gen = 0;
  const int L = g * kWg + tid;
  const bool lane = L < nsub;
  const uint32_t end = (uint32_t)(L + 1) * sub;
  jh::Mark* mk = marks + ((int64_t)img * lanes_stride + L) * kMarkCap;
  uint32_t* keys = mkeys + tid;                      // stride kWg: lanes on different banks
  // round 0: every lane decodes from its guess (L * sub, phase 0), recording its first path points
  jh::Span s0{0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t last_e = jh::mark_key((uint32_t)L * sub, 0), last_x = 0;
  if (lane) {
    s0 = jh::run_span<jh::kRecord>(H, sd.dc, sd.ac, src, (uint32_t)L * sub, 0, end, zz, keys, kWg, mk, kMarkCap);
    last_x = jh::mark_key(s0.pos, s0.phase);
    if (L + 1 < nsub) {
      st_rel(&S.entry[L + 1], last_x);
      if (last_x != jh::mark_key(end, 0)) st_rel(&S.chg[0], 1);
    }
  }
  if (L == 0) last_e = 0;
  jh::Span sp = s0;
  if (tk) tick[2] = wall_clock64();
  img_barrier(&S.bar, G, gen);
  if (tk) tick[3] = wall_clock64();
  // rounds to the fixed point: a lane whose entry changed re-decodes (stopping where it meets its
  // own round-0 path); after round r the first r + 1 entries are exact; a round without a change
  // ends it
  int rounds = 1;
  for (int r = 1; r <= nsub + 1 && ld_acq(&S.chg[r - 1]) != 0; ++r) {
    if (lane && L > 0) {
      const uint32_t e = ld_acq(&S.entry[L]);
      if (e != last_e) {
        last_e = e;
        sp = L + 1 < nsub
                 ? jh::run_span<jh::kSync>(H, sd.dc, sd.ac, src, e >> 4, (int)(e & 15), end, zz, keys, kWg, mk, 0, &s0)
                 : jh::run_span<jh::kPlain>(H, sd.dc, sd.ac, src, e >> 4, (int)(e & 15), end, zz);
        const uint32_t x = jh::mark_key(sp.pos, sp.phase);
        if (L + 1 < nsub && x != last_x) {
          last_x = x;
          st_rel(&S.entry[L + 1], x);
          st_rel(&S.chg[r], 1);
        }
      }
    }
    img_barrier(&S.bar, G, gen);
    if (tk && r < 100) tick[3 + r] = wall_clock64();
    rounds = r + 1;
  }

  // exclusive prefix sums of (blocks, DC-difference sums) over the lanes: in the wave, over the
  // waves of the workgroup, then over the workgroups
  const int wv = tid >> 6, ln = tid & 63;
  const int v0 = lane ? sp.n : 0, v1 = lane ? sp.d0 : 0, v2 = lane ? sp.d1 : 0, v3 = lane ? sp.d2 : 0;
  int i0 = v0, i1 = v1, i2 = v2, i3 = v3;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t0 = __shfl_up(i0, o, 64), t1 = __shfl_up(i1, o, 64), t2 = __shfl_up(i2, o, 64),
              t3 = __shfl_up(i3, o, 64);
    if (ln >= o) {
      i0 += t0;
      i1 += t1;
      i2 += t2;
      i3 += t3;
    }
  }
  if (ln == 63) {
    wtot[wv][0] = i0;
    wtot[wv][1] = i1;
    wtot[wv][2] = i2;
    wtot[wv][3] = i3;
  }
  __syncthreads();
  for (int k = 0; k < wv; ++k) {
    i0 += wtot[k][0];
    i1 += wtot[k][1];
    i2 += wtot[k][2];
    i3 += wtot[k][3];
  }
  if (G > 1) {
    if (tid == kWg - 1) {
      st_rel(&S.wsum[g][0], i0);
      st_rel(&S.wsum[g][1], i1);
      st_rel(&S.wsum[g][2], i2);
      st_rel(&S.wsum[g][3], i3);
    }
    img_barrier(&S.bar, G, gen);
    for (int k = 0; k < g; ++k) {
      i0 += ld_acq(&S.wsum[k][0]);
      i1 += ld_acq(&S.wsum[k][1]);
      i2 += ld_acq(&S.wsum[k][2]);
      i3 += ld_acq(&S.wsum[k][3]);
    }
  }
  const int base = i0 - v0;
  if (tk) tick[120] = wall_clock64();
  if (lane) {
    // an invalid code on the exact path before the frame's last block, or too few blocks
    bool bad = sp.good < sp.n && (int64_t)base + sp.good < H.total;
    if (L == nsub - 1 && (int64_t)base + sp.n < H.total) bad = true;
    if (base < H.total && !jh::write_span(H, sd.dc, sd.ac, src, last_e >> 4, (int)(last_e & 15), end, base, i1 - v1,
                                          i2 - v2, i3 - v3, co, zz))
      bad = true;
    if (bad) *s_err = 1;
  }
  __syncthreads();
  if (tid == 0) {
    if (*s_err) atomicOr(&err[2 * img], 1);
    if (g == 0) err[2 * img + 1] = rounds;
  }
  if (tk) tick[121] = wall_clock64();
}

// grid (workgroups per image, images).  err[2 * image] |= 1 when the stream is malformed /
// truncated (its coefficients are then unspecified; err zeroed before the launch),
// err[2 * image + 1] = rounds.  marks: lanes_stride * kMarkCap per image.
__global__ __launch_bounds__(kWg) void jpeg_huff_kernel(const uint8_t* __restrict__ blob, int16_t* __restrict__ coefs,
                                                        int32_t* __restrict__ err, HuffImgState* states,
                                                        jh::Mark* marks, int lanes_stride, int lds_words,
                                                        int64_t* ticks) {
  __shared__ JHuffDesc sd;
  __shared__ int32_t s_err;
  __shared__ int32_t wtot[kWg / 64][4];
  __shared__ uint8_t zz[64];
  __shared__ uint32_t mkeys[kMarkCap * kWg];
  extern __shared__ uint32_t lds_stream[];
  const int tid = threadIdx.x, g = blockIdx.x, img = blockIdx.y;
  int64_t* tick = ticks != nullptr ? ticks + (int64_t)img * 128 : nullptr;
  if (tick != nullptr && g == 0 && tid == 0) tick[0] = wall_clock64();
  const JHuffJob job = reinterpret_cast<const JHuffJob*>(blob)[img];
  const uint8_t* dp = blob + job.desc_off;
  {
    const uint4* src = reinterpret_cast<const uint4*>(dp);
    uint4* dst = reinterpret_cast<uint4*>(&sd);
    for (int i = tid; i < (int)(sizeof(JHuffDesc) / 16); i += kWg) dst[i] = src[i];
  }
  if (tid < 64) zz[tid] = kJpegZigzag[tid];
  if (tid == 0) s_err = 0;
  __syncthreads();
  const JHuffHead& H = sd.h;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(dp + H.stream_off);
  int16_t* co = coefs + job.coef_off;
  const bool restart = H.restart_blocks > 0;
  const int nsub = H.nsub;
  const int G = restart ? 1 : (nsub + kWg - 1) / kWg;
  if (g >= G) return;                               // uniform: this image needs fewer workgroups

  if (restart) {   // independent restart intervals, one workgroup
    const jh::SrcMem src{w, (uint32_t)H.nwords};
    const int32_t* segs = reinterpret_cast<const int32_t*>(dp + H.seg_off);
    bool ok = true;
    for (int s = tid; s < H.nseg; s += kWg) ok = ok && jh::write_interval(H, sd.dc, sd.ac, src, segs, s, co, zz);
    if (!ok) atomicOr(&err[2 * img], 1);
    if (tid == 0) err[2 * img + 1] = 0;
    return;
  }

  // this workgroup's window of the stream into LDS: every word its lanes can reach (a span ends at
  // most one block, < 2 Kbit, past its subsequence) when it fits, else global reads
  const uint32_t sub = (uint32_t)H.sub_bits;
  const uint32_t w0 = (uint32_t)(((uint64_t)g * kWg * sub) >> 5);
  const uint32_t need = w0 < (uint32_t)H.nwords ? min((uint32_t)H.nwords - w0, (uint32_t)(kWg * sub / 32 + kExtraWords)) : 0;
  if (need <= (uint32_t)lds_words) {
    for (uint32_t i = tid; i < need; i += kWg) lds_stream[i] = w[w0 + i];
    __syncthreads();
    huff_lanes(sd, jh::SrcLds{lds_stream, w0, need}, co, states + img, marks, lanes_stride, zz, &s_err, wtot, mkeys, err,
               tick);
  } else {
    huff_lanes(sd, jh::SrcMem{w, (uint32_t)H.nwords}, co, states + img, marks, lanes_stride, zz, &s_err, wtot, mkeys,
               err, tick);
  }
}

// bytes of the zeroed per-image state + marks scratch for n images of <= lanes lanes each
size_t jpeg_huff_scratch_bytes(int n, int lanes) {
  return (size_t)n * sizeof(HuffImgState) + (size_t)n * lanes * kMarkCap * sizeof(jh::Mark);
}
size_t jpeg_huff_state_bytes(int n) { return (size_t)n * sizeof(HuffImgState); }

// window: the largest per-workgroup stream window of the batch in words (0: no LDS staging)
hipError_t jpeg_huff_decode(const uint8_t* blob, int n, int max_wg, int16_t* coefs, int32_t* err, void* scratch,
                            int lanes, int window, int64_t* ticks, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int lds_words = window > 0 && window <= kMaxWindowWords ? ((window + 3) & ~3) : 0;
  const size_t dyn = (size_t)lds_words * 4;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)jpeg_huff_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       kMaxWindowWords * 4);
    if (e != hipSuccess) return e;
    attr = true;
  }
  auto* st = static_cast<HuffImgState*>(scratch);
  auto* mk = reinterpret_cast<jh::Mark*>(static_cast<uint8_t*>(scratch) + jpeg_huff_state_bytes(n));
  hipLaunchKernelGGL(jpeg_huff_kernel, dim3(max_wg, n), dim3(kWg), dyn, stream, blob, coefs, err, st, mk, lanes,
                     lds_words, ticks);
  return hipGetLastError();
}

}  // namespace lumen
