// Descriptor of one baseline JPEG for the GPU entropy decoder (csrc/jpeg_huff.hip), written by
// the host preparation step (csrc/host/jpeg_decode.cpp: lumen_jpeg_prepare_gpu: header parse,
// Huffman table build, byte unstuffing) into a pinned upload blob.  Plain C++ (no HIP headers):
// the host library and the HIP kernels share this layout.
//
// Upload blob: JHuffJob[n] (padded to 256 bytes), then per image at job.desc_off (256-aligned):
//   JHuffDesc | unstuffed entropy-coded bytes as big-endian 32-bit words (zero padded) |
//   restart-interval starts (int32 bit offsets, restart JPEGs only)
#pragma once
#include <cstdint>

namespace lumen {

constexpr int kJHuffFast = 10;   // lookahead bits of the fast tables (as the host decoder's)
constexpr int kJHuffWgLanes = 256;     // lanes (threads) per workgroup: one wave per SIMD
constexpr int kJHuffMaxLanes = 4096;   // lanes per image (16 workgroups)

struct JHuffDc {
  uint16_t fast[1 << kJHuffFast];   // (length << 8) | symbol, 0 = longer code
  int32_t maxcode[18];
  int32_t valptr[17];
  int32_t mincode[17];
  uint8_t vals[256];
};

struct JHuffAc {
  uint16_t fast[1 << kJHuffFast];
  // code AND its extra bits within the lookahead: (value << 16) | (run << 12) | (length << 4) | 1
  int32_t fast_ac[1 << kJHuffFast];
  int32_t maxcode[18];
  int32_t valptr[17];
  int32_t mincode[17];
  uint8_t vals[256];
};

struct JHuffHead {
  int32_t nbits;          // entropy-coded bits (after unstuffing)
  int32_t nwords;         // 32-bit words of the stream including the zero padding
  int32_t total;          // blocks of the frame (whole MCUs)
  int32_t bpm;            // blocks per MCU
  int32_t ncomp;
  int32_t mcux;
  int32_t restart_blocks; // blocks per restart interval (0: no restart markers)
  int32_t nseg;           // restart intervals found in the stream
  int32_t sub_bits;       // bits per subsequence of the synchronising decode (no restarts)
  int32_t nsub;           // subsequences = lanes (<= kJHuffMaxLanes)
  int32_t ndc, nac;       // distinct tables used
  int32_t stream_off;     // bytes from the descriptor to the stream words
  int32_t seg_off;        // bytes from the descriptor to the restart starts
  // per block of the MCU: component, block column / row inside the MCU, table slots
  int32_t pcomp[10], px[10], py[10], pdc[10], pac[10];
  int32_t bw[3], hh[3], vv[3], pad_;
  int64_t plane_off[3];   // element offset of each component plane in the image's coefficients
};

struct JHuffDesc {
  JHuffHead h;
  JHuffDc dc[3];
  JHuffAc ac[3];
};

static_assert(sizeof(JHuffHead) % 16 == 0 && sizeof(JHuffDc) % 16 == 0 && sizeof(JHuffAc) % 16 == 0,
              "16-byte copies into LDS");

struct JHuffJob {
  int64_t desc_off;       // bytes from the blob start
  int64_t coef_off;       // int16 elements from the coefficient buffer start
};

}  // namespace lumen
