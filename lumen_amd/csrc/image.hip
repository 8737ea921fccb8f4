// Image preprocessing kernels (resize / pad / normalise / layout) for gfx950.
//
// A ragged batch of decoded uint8 HWC images (one flat buffer + per-image
// offset/height/width) is resampled straight into the tensor layout the next
// kernel wants: NCHW, NHWC, or ViT patch rows [B*P, Kpad] (im2col of the
// patch-embedding convolution, so the patch GEMM reads it as a plain A matrix).
//
// Two geometries cover every preprocessor of the reference:
//   canvas  : the image is first placed at (ox, oy) in a (cw x ch) canvas filled
//             with `pad` and the canvas is resized to the output
//             (VLM pad-to-square, packages/lumen-vlm/.../onnxrt_backend.py:661-719)
//   dst rect: the image is resized into (dw x dh) at (dx, dy) of the output and
//             the rest is `pad` (SCRFD letterbox, lumen-face onnxrt_backend.py:749-808;
//             OCR det resize, lumen-ocr onnxrt_backend.py:338-378)
// Filters: 0 = PIL BICUBIC (a=-0.5, antialiased on downscale; CLIP
// onnxrt_backend.py:410-431), 1 = PIL BILINEAR (antialiased), 2 = cv2
// INTER_LINEAR (half-pixel, no antialias), 3 = cv2 INTER_CUBIC (a=-0.75).
// Resampling is separable: pass 1 filters rows into an fp32 scratch, pass 2
// filters columns, normalises ((x/255 - mean)/std, or (x - mean)/std in 0..255
// units) and writes the layout.  ViT patch rows with the PIL filters take the fused
// per-band kernel instead (prep_band_kernel: uint8 row pass in LDS, no scratch round trip).
#include "common.h"

namespace lumen {

// 11 x int64 per image (host passes a [B, 11] int64 tensor)
struct ImgGeomRaw {
  int64_t ih, iw, off, cw, ch, ox, oy, dx, dy, dw, dh;
};
struct ImgGeom {
  int ih, iw;        // input image size
  int64_t off;       // byte offset of image in the flat buffer
  int cw, ch, ox, oy;  // source canvas: image at (ox, oy) inside (cw x ch)
  int dx, dy, dw, dh;  // destination rect inside the (OH x OW) output
};
__device__ __forceinline__ ImgGeom load_geom(const ImgGeomRaw* r) {
  ImgGeom g;
  g.ih = (int)r->ih; g.iw = (int)r->iw; g.off = r->off;
  g.cw = (int)r->cw; g.ch = (int)r->ch; g.ox = (int)r->ox; g.oy = (int)r->oy;
  g.dx = (int)r->dx; g.dy = (int)r->dy; g.dw = (int)r->dw; g.dh = (int)r->dh;
  return g;
}

struct PrepArgs {
  const uint8_t* src;
  const ImgGeomRaw* geom;   // device array [B]
  float* tmp;            // [B, max_ch, max_dw, 3]
  int tmp_h, tmp_w;      // scratch dims
  void* out;
  int OH, OW;
  int filter;
  int swap_rb;           // output channel order reversed (RGB <-> BGR)
  float mean[3], inv_std[3];
  float scale;           // 1/255 or 1
  float pad;             // raw pad value (0..255)
  int layout;            // 0 NCHW, 1 NHWC, 2 patches
  int patch;             // patch size for layout 2
  int kpad;              // padded K (row length) for layout 2
  int out_bf16;
};

__device__ __forceinline__ float cubic_w(float x, float a) {
  x = fabsf(x);
  if (x < 1.f) return ((a + 2.f) * x - (a + 3.f)) * x * x + 1.f;
  if (x < 2.f) return (((x - 5.f) * x + 8.f) * x - 4.f) * a;
  return 0.f;
}
__device__ __forceinline__ float filt(float x, int f) {
  if (f == 0) return cubic_w(x, -0.5f);
  if (f == 3) return cubic_w(x, -0.75f);
  x = fabsf(x);
  return x < 1.f ? 1.f - x : 0.f;
}
__device__ __forceinline__ float support(int f) { return (f == 0 || f == 3) ? 2.f : 1.f; }

// 1-D window for output index i of a (in_len -> out_len) resample
__device__ __forceinline__ void window(int i, int in_len, int out_len, int f, int& x0, int& x1,
                                       float& center, float& inv_ss) {
  const float scale = (float)in_len / (float)out_len;
  if (f >= 2) {  // cv2: no antialias, half-pixel centres, replicate border
    center = (i + 0.5f) * scale - 0.5f;
    const int r = (f == 3) ? 2 : 1;
    x0 = (int)floorf(center) - r + 1;
    x1 = x0 + 2 * r;
    inv_ss = 1.f;
    return;
  }
  const float ss = fmaxf(scale, 1.f);
  const float sup = support(f) * ss;
  center = (i + 0.5f) * scale;
  x0 = max((int)(center - sup + 0.5f), 0);
  x1 = min((int)(center + sup + 0.5f), in_len);
  inv_ss = 1.f / ss;
}

// canvas pixel fetch (raw 0..255), pad outside the image
__device__ __forceinline__ void canvas_px(const uint8_t* img, const ImgGeom& g, int x, int y, float pad, float* c) {
  const int ix = x - g.ox, iy = y - g.oy;
  if (ix < 0 || iy < 0 || ix >= g.iw || iy >= g.ih) { c[0] = c[1] = c[2] = pad; return; }
  const uint8_t* p = img + ((int64_t)iy * g.iw + ix) * 3;
  c[0] = p[0]; c[1] = p[1]; c[2] = p[2];
}

// pass 1: horizontal resample of every canvas row into tmp[b][y][x'][3], x' in [0, dw)
__global__ void prep_h_kernel(PrepArgs a) {
  const int b = blockIdx.z;
  const ImgGeom g = load_geom(a.geom + b);
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= g.dw || y >= g.ch) return;
  const uint8_t* img = a.src + g.off;
  int x0, x1; float center, inv_ss;
  window(x, g.cw, g.dw, a.filter, x0, x1, center, inv_ss);
  float acc[3] = {0.f, 0.f, 0.f}, ws = 0.f;
  for (int sx = x0; sx < x1; ++sx) {
    float w;
    int cx = sx;
    if (a.filter >= 2) { w = filt((float)sx - center, a.filter); cx = min(max(sx, 0), g.cw - 1); }
    else w = filt(((float)sx - center + 0.5f) * inv_ss, a.filter);
    float c[3];
    canvas_px(img, g, cx, y, a.pad, c);
    acc[0] += w * c[0]; acc[1] += w * c[1]; acc[2] += w * c[2];
    ws += w;
  }
  const float inv = ws != 0.f ? 1.f / ws : 0.f;
  float* t = a.tmp + (((int64_t)b * a.tmp_h + y) * a.tmp_w + x) * 3;
  if (a.filter < 2) {  // PIL rounds/clips to uint8 between the two passes
    for (int k = 0; k < 3; ++k) t[k] = fminf(fmaxf(rintf(acc[k] * inv), 0.f), 255.f);
  } else {
    t[0] = acc[0] * inv; t[1] = acc[1] * inv; t[2] = acc[2] * inv;
  }
}

// pass 2: vertical resample + normalise + layout
__global__ void prep_v_kernel(PrepArgs a) {
  const int b = blockIdx.z;
  const ImgGeom g = load_geom(a.geom + b);
  const int ox = blockIdx.x * blockDim.x + threadIdx.x;
  const int oy = blockIdx.y;
  if (ox >= a.OW || oy >= a.OH) return;
  float c[3];
  const int rx = ox - g.dx, ry = oy - g.dy;
  if (rx < 0 || ry < 0 || rx >= g.dw || ry >= g.dh) {
    c[0] = c[1] = c[2] = a.pad;
  } else {
    int y0, y1; float center, inv_ss;
    window(ry, g.ch, g.dh, a.filter, y0, y1, center, inv_ss);
    float acc[3] = {0.f, 0.f, 0.f}, ws = 0.f;
    for (int sy = y0; sy < y1; ++sy) {
      float w;
      int cy = sy;
      if (a.filter >= 2) { w = filt((float)sy - center, a.filter); cy = min(max(sy, 0), g.ch - 1); }
      else w = filt(((float)sy - center + 0.5f) * inv_ss, a.filter);
      const float* t = a.tmp + (((int64_t)b * a.tmp_h + cy) * a.tmp_w + rx) * 3;
      acc[0] += w * t[0]; acc[1] += w * t[1]; acc[2] += w * t[2];
      ws += w;
    }
    const float inv = ws != 0.f ? 1.f / ws : 0.f;
    // PIL / cv2 round and clip to uint8 after each resample pass
    for (int k = 0; k < 3; ++k) c[k] = fminf(fmaxf(rintf(acc[k] * inv), 0.f), 255.f);
  }
  float v[3];
  for (int k = 0; k < 3; ++k) {
    const int sk = a.swap_rb ? 2 - k : k;
    v[k] = (c[sk] * a.scale - a.mean[k]) * a.inv_std[k];
  }
  int64_t idx[3];
  if (a.layout == 0) {
    for (int k = 0; k < 3; ++k) idx[k] = (((int64_t)b * 3 + k) * a.OH + oy) * a.OW + ox;
  } else if (a.layout == 1) {
    for (int k = 0; k < 3; ++k) idx[k] = (((int64_t)b * a.OH + oy) * a.OW + ox) * 3 + k;
  } else if (a.layout == 3) {  // NHWC with channels padded to 8 (implicit-GEMM conv input, Cin % 8 == 0)
    const int64_t base = (((int64_t)b * a.OH + oy) * a.OW + ox) * 8;
    for (int k = 0; k < 3; ++k) idx[k] = base + k;
    if (a.out_bf16) {
      u32x4_t z = (u32x4_t){0u, 0u, 0u, 0u};
      *(u32x4_t*)((uint16_t*)a.out + base) = z;  // zero the pad lanes first (same thread writes 0..2 below)
    } else {
      for (int k = 3; k < 8; ++k) ((float*)a.out)[base + k] = 0.f;
    }
  } else {
    const int p = a.patch, gw = a.OW / p;
    const int64_t prow = (int64_t)b * (a.OH / p) * gw + (oy / p) * gw + (ox / p);
    for (int k = 0; k < 3; ++k) idx[k] = prow * a.kpad + k * p * p + (oy % p) * p + (ox % p);
  }
  if (a.out_bf16) {
    uint16_t* o = (uint16_t*)a.out;
    for (int k = 0; k < 3; ++k) o[idx[k]] = f2bf(v[k]);
  } else {
    float* o = (float*)a.out;
    for (int k = 0; k < 3; ++k) o[idx[k]] = v[k];
  }
}

// ---------------------------------------------------------------------------------------------
// Fused ViT prep for the PIL filters (0 / 1) into patch rows: one workgroup per (image, band of
// `patch` output rows), everything between the uint8 input and the bf16 patch rows stays in LDS.
//   0. tap weights per destination column (horizontal) and per band row (vertical), with the same
//      window / filt arithmetic as prep_h / prep_v;
//   1. the canvas pixels the band reads are staged once as packed RGBX words (a tap is then one
//      ds_read_b32 + v_cvt_f32_ubyte0..2 instead of three global byte loads; three ds_read_u8 of a
//      byte-packed stage measured slower); each thread owns one destination column, keeps its tap
//      weights in registers and filters every staged row, rounding and clipping to uint8 as PIL
//      does between its passes (exact to keep as bytes); the pad must then be integral (host);
//   2. each thread owns one output column: vertical pass + normalisation, bf16 into an LDS image
//      of the band's patch rows (K padding zeroed);
//   3. the band's patch rows are one contiguous run of gw * kpad bf16: 16-byte stores.
// Same weights and accumulation order as the two-pass kernels: bit-identical output, without their
// fp32 scratch round trip (b512 ViT-L/14: 352 MB) and the patch_pad launch.
// rcap: canvas rows per band; cwcap: staged canvas columns; TM >= taps per window (host bounds).
template <int K>
__device__ __forceinline__ float ubyte_f(uint32_t v) {   // byte K as float (v_cvt_f32_ubyteK)
  return (float)((v >> (8 * K)) & 0xffu);
}
__device__ __forceinline__ uint32_t pack_rgb(const float* c) {
  return (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16);
}

template <int TM>
__global__ void __launch_bounds__(256) prep_band_kernel(PrepArgs a, int rcap, int cwcap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const int b = blockIdx.y, band = blockIdx.x, tid = threadIdx.x;
  const ImgGeom g = load_geom(a.geom + b);
  const uint8_t* img = a.src + g.off;
  const int p = a.patch, gw = a.OW / p, OW = a.OW;
  const int oy0 = band * p;
  // LDS: [vertical tables][horizontal tables | staged canvas bytes][row-pass pixels]; the band's patch
  // image (obuf) reuses the second region once the row pass has consumed it
  float* vw = (float*)sm;                            // [p][TM]
  float* vinv = vw + p * TM;                         // [p]
  int* vy0 = (int*)(vinv + p);                       // [p]
  int* vn = vy0 + p;                                 // [p] (0: row outside the destination rect)
  uint8_t* regA = (uint8_t*)(((uintptr_t)(vn + p) + 15) & ~(uintptr_t)15);
  float* hw = (float*)regA;                          // [OW][TM] horizontal tap weights
  float* hinv = hw + OW * TM;                        // [OW]
  int* hx0 = (int*)(hinv + OW);                      // [OW]
  int* hn = hx0 + OW;                                // [OW] taps
  uint32_t* inpx = (uint32_t*)(((uintptr_t)(hn + OW) + 15) & ~(uintptr_t)15);  // [rcap][cwcap] canvas RGBX
  const size_t szA = (size_t)((uint8_t*)inpx - regA) + (size_t)rcap * cwcap * 4;
  const size_t szO = (size_t)gw * a.kpad * 2;
  uint32_t* hpx = (uint32_t*)(regA + ((((szA > szO ? szA : szO)) + 15) & ~(size_t)15));   // [rcap][OW] RGBX
  uint16_t* obuf = (uint16_t*)regA;                  // [gw * kpad], after the row pass

  const int rx_lo = max(0, -g.dx), rx_hi = min(g.dw, OW - g.dx);
  const int nx = max(0, rx_hi - rx_lo);
  // 0. weights
  for (int i = tid; i < nx; i += blockDim.x) {
    int x0, x1; float center, inv_ss;
    window(rx_lo + i, g.cw, g.dw, a.filter, x0, x1, center, inv_ss);
    float ws = 0.f;
    for (int sx = x0; sx < x1; ++sx) {
      const float w = filt(((float)sx - center + 0.5f) * inv_ss, a.filter);
      if (sx - x0 < TM) hw[i * TM + (sx - x0)] = w;
      ws += w;
    }
    hinv[i] = ws != 0.f ? 1.f / ws : 0.f;
    hx0[i] = x0;
    hn[i] = min(x1 - x0, TM);
  }
  if (tid < p) {
    const int ry = oy0 + tid - g.dy;
    int n = 0, y0 = 0;
    float ws = 0.f;
    if (ry >= 0 && ry < g.dh) {
      int y1; float center, inv_ss;
      window(ry, g.ch, g.dh, a.filter, y0, y1, center, inv_ss);
      for (int sy = y0; sy < y1; ++sy) {
        const float w = filt(((float)sy - center + 0.5f) * inv_ss, a.filter);
        if (sy - y0 < TM) vw[tid * TM + (sy - y0)] = w;
        ws += w;
      }
      n = min(y1 - y0, TM);
    }
    vinv[tid] = ws != 0.f ? 1.f / ws : 0.f;
    vy0[tid] = y0;
    vn[tid] = n;
  }
  __syncthreads();
  // canvas rows / columns the band reads (window starts and ends grow with the index)
  int Y0 = 0, Y1 = 0;
  for (int r = 0; r < p; ++r)
    if (vn[r] > 0) { Y0 = vy0[r]; break; }
  for (int r = p - 1; r >= 0; --r)
    if (vn[r] > 0) { Y1 = vy0[r] + vn[r]; break; }
  const int R = min(max(Y1 - Y0, 0), rcap);          // the host bounds make the clamps no-ops
  const int cx_lo = nx > 0 ? hx0[0] : 0;
  const int cwl = nx > 0 ? min(hx0[nx - 1] + hn[nx - 1] - cx_lo, cwcap) : 0;
  // 1a. stage the canvas pixels as RGBX words (pad outside the image)
  for (int i = tid; i < R * cwl; i += blockDim.x) {
    const int r = i / cwl;
    float c[3];
    canvas_px(img, g, cx_lo + (i - r * cwl), Y0 + r, a.pad, c);
    inpx[r * cwcap + (i - r * cwl)] = pack_rgb(c);
  }
  __syncthreads();
  // 1b. horizontal pass: one destination column per thread (tap weights in registers), every staged row
  for (int j = tid; j < nx; j += blockDim.x) {
    float w[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) w[t] = hw[j * TM + t];
    const int n = hn[j], xo = min(hx0[j] - cx_lo, cwl - 1);
    const int nt = min(n, cwl - xo);
    const float inv = hinv[j];
    for (int r = 0; r < R; ++r) {
      const uint32_t* q = inpx + r * cwcap + xo;
      float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        if (t < nt) {
          const uint32_t v = q[t];
          acc[0] += w[t] * ubyte_f<0>(v);
          acc[1] += w[t] * ubyte_f<1>(v);
          acc[2] += w[t] * ubyte_f<2>(v);
        }
      }
      float c[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) c[k] = fminf(fmaxf(rintf(acc[k] * inv), 0.f), 255.f);
      hpx[r * OW + j] = pack_rgb(c);
    }
  }
  __syncthreads();
  // K padding of the band's patch rows (obuf now reuses the staging region)
  const int pp = p * p, kreal = 3 * pp, npad = a.kpad - kreal;
  for (int i = tid; i < gw * npad; i += blockDim.x) {
    const int pc = i / npad;
    obuf[pc * a.kpad + kreal + (i - pc * npad)] = 0;
  }
  // 2. vertical pass + normalise: one output column per thread, the band's p rows
  for (int ox = tid; ox < OW; ox += blockDim.x) {
    const int rx = ox - g.dx;
    const bool colin = rx >= 0 && rx < g.dw;
    const int pc = ox / p, ix = ox - pc * p;
    uint16_t* ob = obuf + pc * a.kpad + ix;
    for (int iy = 0; iy < p; ++iy) {
      const int n = colin ? vn[iy] : 0;
      float c[3];
      if (n == 0) {
        c[0] = c[1] = c[2] = a.pad;
      } else {
        const int yl0 = vy0[iy] - Y0;                // >= 0
        const float* w = vw + iy * TM;
        float acc[3] = {0.f, 0.f, 0.f};
        for (int t = 0; t < n; ++t) {
          const uint32_t v = hpx[min(yl0 + t, R - 1) * OW + (rx - rx_lo)];
          acc[0] += w[t] * ubyte_f<0>(v);
          acc[1] += w[t] * ubyte_f<1>(v);
          acc[2] += w[t] * ubyte_f<2>(v);
        }
        const float inv = vinv[iy];
#pragma unroll
        for (int k = 0; k < 3; ++k) c[k] = fminf(fmaxf(rintf(acc[k] * inv), 0.f), 255.f);
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int sk = a.swap_rb ? 2 - k : k;
        ob[k * pp + iy * p] = f2bf((c[sk] * a.scale - a.mean[k]) * a.inv_std[k]);
      }
    }
  }
  __syncthreads();
  // 3. the band's gw patch rows are contiguous in the output
  const int64_t base = ((int64_t)b * (a.OH / p) + band) * gw * a.kpad;
  const int nvec = gw * a.kpad / 8;
  for (int i = tid; i < nvec; i += blockDim.x)
    *(u32x4_t*)((uint16_t*)a.out + base + (int64_t)i * 8) = *(const u32x4_t*)(obuf + i * 8);
}

size_t image_prep_band_lds(int OW, int patch, int kpad, int rcap, int cwcap, int TM) {
  const size_t v = (((size_t)patch * (TM + 3) * 4) + 15) & ~(size_t)15;
  const size_t h = (((size_t)OW * (TM + 3) * 4) + 15) & ~(size_t)15;
  const size_t a = h + (size_t)rcap * cwcap * 4;
  const size_t o = (size_t)(OW / patch) * kpad * 2;
  return v + (((a > o ? a : o) + 15) & ~(size_t)15) + (size_t)rcap * OW * 4 + 16;
}

hipError_t image_prep_band(const PrepArgs& a, int B, int rcap, int cwcap, int T, hipStream_t stream) {
  if (a.layout != 2 || a.filter >= 2 || !a.out_bf16 || a.patch <= 0 || a.OH % a.patch || a.OW % a.patch ||
      a.kpad % 8 || rcap <= 0 || cwcap <= 0 || T <= 0 || T > 16)
    return hipErrorInvalidValue;
  const int TM = T <= 8 ? 8 : 16;
  const size_t lds = image_prep_band_lds(a.OW, a.patch, a.kpad, rcap, cwcap, TM);
  if (lds > 96 * 1024) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)prep_band_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    (void)hipFuncSetAttribute((const void*)prep_band_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    attr = true;
  }
  if (TM == 8) hipLaunchKernelGGL(prep_band_kernel<8>, dim3(a.OH / a.patch, B), dim3(256), lds, stream, a, rcap, cwcap);
  else hipLaunchKernelGGL(prep_band_kernel<16>, dim3(a.OH / a.patch, B), dim3(256), lds, stream, a, rcap, cwcap);
  return hipGetLastError();
}

// zero the K padding columns of patch rows (k in [3p^2, kpad))
__global__ void patch_pad_kernel(uint16_t* out, int64_t rows, int k0, int kpad) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  for (int k = k0 + (threadIdx.x & 63); k < kpad; k += 64) out[r * kpad + k] = 0;
}

hipError_t image_prep(const PrepArgs& a, int B, int max_ch, int max_dw, hipStream_t stream) {
  {
    dim3 block(128), grid((max_dw + 127) / 128, max_ch, B);
    hipLaunchKernelGGL(prep_h_kernel, grid, block, 0, stream, a);
  }
  {
    dim3 block(128), grid((a.OW + 127) / 128, a.OH, B);
    hipLaunchKernelGGL(prep_v_kernel, grid, block, 0, stream, a);
  }
  if (a.layout == 2 && a.kpad > 3 * a.patch * a.patch) {
    const int64_t rows = (int64_t)B * (a.OH / a.patch) * (a.OW / a.patch);
    hipLaunchKernelGGL(patch_pad_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                       (uint16_t*)a.out, rows, 3 * a.patch * a.patch, a.kpad);
  }
  return hipGetLastError();
}

}  // namespace lumen
