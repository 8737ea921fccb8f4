// GPU JPEG pixel reconstruction (jpeg.hip) shared with its torch binding (ops_post.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lumen {

struct JpegPlanes {
  const int16_t* coef;   // all planes, [bh][bw][64] each, natural order, not dequantised
  const uint16_t* qt;    // [ncomp][64]
  uint8_t* samp;         // component sample planes [bh * 8][bw * 8] each
  int64_t coef_off[3], samp_off[3];
  int bw[3], bh[3], h[3], v[3];
  int ncomp, hmax, vmax, width, height;
};

// One image of a batched reconstruction: its planes, its uint8 [height, width, 3] output and where
// its 8x8 blocks / pixels start in the batch's (4-block / 256-pixel padded) iteration spaces.
struct JpegBatchEntry {
  JpegPlanes P;
  uint8_t* out;
  int64_t blk0, pix0;
};

hipError_t jpeg_reconstruct(const JpegPlanes& P, uint8_t* out, hipStream_t stream);
// entries: device array of n entries (blk0 / pix0 ascending); total_blk / total_pix: padded totals
hipError_t jpeg_reconstruct_batch(const JpegBatchEntry* entries, int n, int64_t total_blk, int64_t total_pix,
                                  hipStream_t stream);

// GPU entropy decode (jpeg_huff.hip): blob = JHuffJob[n] + descriptors / streams (jpeg_huff.h);
// coefficient planes into coefs; err [2n] int32 zeroed (malformed flag, synchronisation rounds);
// scratch: jpeg_huff_scratch_bytes(n, lanes) zeroed; max_wg: the most workgroups an image needs
// (ceil(nsub / 256)); lanes: the most lanes of an image; window: the largest stream window (words);
// ticks (nullable): [n][128] wall-clock stamps of workgroup 0's phases (profiling)
hipError_t jpeg_huff_decode(const uint8_t* blob, int n, int max_wg, int16_t* coefs, int32_t* err, void* scratch,
                            int lanes, int window, int64_t* ticks, hipStream_t stream);
size_t jpeg_huff_scratch_bytes(int n, int lanes);

}  // namespace lumen
