// Row normalisation kernels: LayerNorm, RMSNorm (optionally fused with the
// residual add that precedes it), row L2-normalise, and the small CLIP
// token-assembly helpers.  One wave64 per row, 16-byte vector loads.
//
// Reference ops replaced: the LayerNorm / RMSNorm nodes inside the ONNX
// towers and the numpy `embedding / ||embedding||` at
// packages/lumen-clip/src/lumen_clip/backends/onnxrt_backend.py:458,545-546 and
// packages/lumen-face/src/lumen_face/backends/onnxrt_backend.py:1341-1343.
#include "common.h"
#include "tuning.h"

namespace lumen {

// mode 0 = LayerNorm (mean/var, weight, bias), 1 = RMSNorm (weight only)
template <int CPL>
__global__ void __launch_bounds__(256)
norm_rows_kernel(const uint16_t* __restrict__ x, int64_t x_stride, const int64_t* __restrict__ row_idx,
                 const uint16_t* __restrict__ add, int64_t add_stride,
                 uint16_t* __restrict__ resid_out, int64_t resid_stride,
                 const uint16_t* __restrict__ w, const uint16_t* __restrict__ b,
                 void* __restrict__ out, int64_t out_stride, int out_f32,
                 int rows, int D, float eps, int mode) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t src_row = row_idx ? row_idx[row] : row;
  const uint16_t* xr = x + src_row * x_stride;
  const int nch = D >> 3;
  float v[CPL][8];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      unpack8(*(const u32x4_t*)(xr + ch * 8), v[c]);
      if (add) {
        float a[8];
        unpack8(*(const u32x4_t*)(add + src_row * add_stride + ch * 8), a);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] += a[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
  }
  if (resid_out) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) *(u32x4_t*)(resid_out + (int64_t)row * resid_stride + ch * 8) = pack8(v[c]);
    }
  }
  float mean = 0.f;
  if (mode == 0) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    mean = wave_sum(s) / (float)D;
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = v[c][i] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch >= nch) continue;
    float wf[8], bfv[8];
    unpack8(*(const u32x4_t*)(w + ch * 8), wf);
    if (b) unpack8(*(const u32x4_t*)(b + ch * 8), bfv);
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o[i] = (v[c][i] - mean) * rstd * wf[i];
      if (b) o[i] += bfv[i];
    }
    if (out_f32) {
      float* op = (float*)out + (int64_t)row * out_stride + ch * 8;
      *(f32x4_t*)op = (f32x4_t){o[0], o[1], o[2], o[3]};
      *(f32x4_t*)(op + 4) = (f32x4_t){o[4], o[5], o[6], o[7]};
    } else {
      *(u32x4_t*)((uint16_t*)out + (int64_t)row * out_stride + ch * 8) = pack8(o);
    }
  }
}

// Few-row variant (decode: 1-16 rows): a whole 256-thread block per row, so a 4096-wide
// row is 2 chunks per lane instead of 8 and the weight / bias chunks are loaded up front,
// beside the x / add loads: one HBM round trip before the reductions instead of a
// load chain per chunk.  One wave per row measured 8.8 us per Llama-3-8B decode norm.
template <int CPB>
__global__ void __launch_bounds__(256)
norm_row_block_kernel(const uint16_t* __restrict__ x, int64_t x_stride, const int64_t* __restrict__ row_idx,
                      const uint16_t* __restrict__ add, int64_t add_stride,
                      uint16_t* __restrict__ resid_out, int64_t resid_stride,
                      const uint16_t* __restrict__ w, const uint16_t* __restrict__ b,
                      void* __restrict__ out, int64_t out_stride, int out_f32,
                      int rows, int D, float eps, int mode) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row = blockIdx.x;
  const int64_t src_row = row_idx ? row_idx[row] : row;
  const uint16_t* xr = x + src_row * x_stride;
  const int nch = D >> 3;
  u32x4_t xv[CPB], av[CPB], wv[CPB], bv[CPB];
#pragma unroll
  for (int c = 0; c < CPB; ++c) {
    const int ch = tid + c * 256;
    const bool ok = ch < nch;
    const int cc = ok ? ch : 0;
    xv[c] = *(const u32x4_t*)(xr + cc * 8);
    av[c] = add ? *(const u32x4_t*)(add + src_row * add_stride + cc * 8) : (u32x4_t){0u, 0u, 0u, 0u};
    wv[c] = *(const u32x4_t*)(w + cc * 8);
    bv[c] = b ? *(const u32x4_t*)(b + cc * 8) : (u32x4_t){0u, 0u, 0u, 0u};
  }
  float v[CPB][8];
#pragma unroll
  for (int c = 0; c < CPB; ++c) {
    const bool ok = tid + c * 256 < nch;
    float a[8];
    unpack8(xv[c], v[c]);
    unpack8(av[c], a);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[c][i] = ok ? v[c][i] + a[i] : 0.f;
    if (resid_out && ok) *(u32x4_t*)(resid_out + (int64_t)row * resid_stride + (tid + c * 256) * 8) = pack8(v[c]);
  }
  float mean = 0.f;
  if (mode == 0) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPB; ++c)
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    s = wave_sum(s);
    if (lane == 0) red[0][wid] = s;
    __syncthreads();
    mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / (float)D;
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPB; ++c) {
    const bool ok = tid + c * 256 < nch;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = ok ? v[c][i] - mean : 0.f;
      ss += d * d;
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) red[1][wid] = ss;
  __syncthreads();
  const float rstd = rsqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)D + eps);
#pragma unroll
  for (int c = 0; c < CPB; ++c) {
    const int ch = tid + c * 256;
    if (ch >= nch) continue;
    float wf[8], bfv[8], o[8];
    unpack8(wv[c], wf);
    unpack8(bv[c], bfv);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * wf[i] + bfv[i];
    if (out_f32) {
      float* op = (float*)out + (int64_t)row * out_stride + ch * 8;
      *(f32x4_t*)op = (f32x4_t){o[0], o[1], o[2], o[3]};
      *(f32x4_t*)(op + 4) = (f32x4_t){o[4], o[5], o[6], o[7]};
    } else {
      *(u32x4_t*)((uint16_t*)out + (int64_t)row * out_stride + ch * 8) = pack8(o);
    }
  }
}

hipError_t norm_rows(const uint16_t* x, int64_t x_stride, const int64_t* row_idx, const uint16_t* add,
                     int64_t add_stride, uint16_t* resid_out, int64_t resid_stride, const uint16_t* w,
                     const uint16_t* b, void* out, int64_t out_stride, int out_f32, int rows, int D,
                     float eps, int mode, hipStream_t stream) {
  const int nch = D / 8;
  if (rows <= 64 && nch <= 4 * 256) {
    const int cpb = (nch + 255) / 256;
#define LNB_CASE(N)                                                                                    \
  case N:                                                                                              \
    hipLaunchKernelGGL(norm_row_block_kernel<N>, dim3(rows), dim3(256), 0, stream, x, x_stride, row_idx, \
                       add, add_stride, resid_out, resid_stride, w, b, out, out_stride, out_f32, rows, D, \
                       eps, mode);                                                                     \
    return hipGetLastError();
    switch (cpb) {
      LNB_CASE(1) LNB_CASE(2) LNB_CASE(3) LNB_CASE(4)
      default: break;
    }
#undef LNB_CASE
  }
  const int cpl = (D / 8 + 63) / 64;
  dim3 grid((rows + 3) / 4), block(256);
#define LN_CASE(N)                                                                                     \
  case N:                                                                                              \
    hipLaunchKernelGGL(norm_rows_kernel<N>, grid, block, 0, stream, x, x_stride, row_idx, add,        \
                       add_stride, resid_out, resid_stride, w, b, out, out_stride, out_f32, rows, D, \
                       eps, mode);                                                                     \
    break;
  switch (cpl) {
    LN_CASE(1) LN_CASE(2) LN_CASE(3) LN_CASE(4) LN_CASE(6) LN_CASE(8) LN_CASE(16)
    default:
      if (cpl == 5) { hipLaunchKernelGGL(norm_rows_kernel<6>, grid, block, 0, stream, x, x_stride, row_idx, add, add_stride, resid_out, resid_stride, w, b, out, out_stride, out_f32, rows, D, eps, mode); }
      else if (cpl == 7) { hipLaunchKernelGGL(norm_rows_kernel<8>, grid, block, 0, stream, x, x_stride, row_idx, add, add_stride, resid_out, resid_stride, w, b, out, out_stride, out_f32, rows, D, eps, mode); }
      else if (cpl <= 16) { hipLaunchKernelGGL(norm_rows_kernel<16>, grid, block, 0, stream, x, x_stride, row_idx, add, add_stride, resid_out, resid_stride, w, b, out, out_stride, out_f32, rows, D, eps, mode); }
      else return hipErrorInvalidValue;
  }
#undef LN_CASE
  return hipGetLastError();
}

// Row L2 normalisation of fp32 rows in place (embedding epilogue).
// LayerNorm statistics only, for a projection with the norm folded in (GemmEpi::row_aff):
// out[row] = (rstd, -mean * rstd).  Same fp32 two-pass arithmetic as norm_rows_kernel mode 0, but
// 8 bytes per row are written instead of the normalised row.  One wave per row, D <= 64 * 8 * CPL.
// With q8 (MX form, the W8A8 vision tower): the raw row also leaves as MX fp8 -- 32-column blocks
// of 4 lanes, E8M0 bytes in K-step planes [D/128][rows][4] (ldqs = plane stride) -- the A operand of
// the LN-folded gemm_mx that consumes it.
template <int CPL>
__global__ void __launch_bounds__(256)
ln_row_stats_kernel(const uint16_t* __restrict__ x, int64_t x_stride, float* __restrict__ out, int rows, int D,
                    float eps, uint8_t* __restrict__ q8, int64_t ldq, uint8_t* __restrict__ qs, int64_t ldqs) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;      // whole waves: the MX shuffles below stay inside a live wave
  const uint16_t* xr = x + (int64_t)row * x_stride;
  const int nch = D >> 3;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      unpack8(*(const u32x4_t*)(xr + ch * 8), v[c]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[c][i];
  }
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    if (lane + c * 64 < nch) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
  if (lane == 0) *(float2*)(out + 2 * (int64_t)row) = make_float2(rstd, -mean * rstd);
  if (q8 != nullptr) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      float am = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(v[c][i]));
      am = fmaxf(am, __shfl_xor(am, 1, 64));
      am = fmaxf(am, __shfl_xor(am, 2, 64));
      if (ch < nch) {
        const int e = mx_exp(am);
        *(uint2*)(q8 + (int64_t)row * ldq + ch * 8) = fp8x8_scaled(v[c], mx_inv(e));
        if ((lane & 3) == 0) qs[(int64_t)(ch >> 4) * ldqs + (int64_t)row * 4 + ((ch >> 2) & 3)] = (uint8_t)(e + 127);
      }
    }
  }
}

// Statistics only, R rows per wave: every row's loads are issued before the first reduction, so a
// wave pays one memory round trip per R rows (ViT-L/14 b256: 65,792 rows of 1,024 -- one row per wave
// left 257 waves per CU each waiting out its own load).
template <int CPL, int R>
__global__ void __launch_bounds__(256)
ln_row_stats_multi_kernel(const uint16_t* __restrict__ x, int64_t x_stride, float* __restrict__ out, int rows, int D,
                          float eps) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  const int nch = D >> 3;
  u32x4_t raw[R][CPL];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint16_t* xr = x + (int64_t)min(row0 + r, rows - 1) * x_stride;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      raw[r][c] = ch < nch ? *(const u32x4_t*)(xr + ch * 8) : (u32x4_t){0u, 0u, 0u, 0u};
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float v[CPL][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      unpack8(raw[r][c], v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (lane + c * 64 < nch) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = v[c][i] - mean;
          ss += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
    if (lane == 0 && row0 + r < rows) *(float2*)(out + 2 * (int64_t)(row0 + r)) = make_float2(rstd, -mean * rstd);
  }
}

hipError_t ln_row_stats(const uint16_t* x, int64_t x_stride, float* out, int rows, int D, float eps,
                        hipStream_t stream, uint8_t* q8, int64_t ldq, uint8_t* qs, int64_t ldqs) {
  if (D % 8 != 0 || D > 64 * 8 * 8 || rows <= 0 || (q8 != nullptr && D % 128 != 0)) return hipErrorInvalidValue;
  if (q8 == nullptr && D <= 1024 && rows >= 16384 && tuning(TUNE_LN_MULTI_ROW)) {   // large row counts: 4 rows per wave
    const dim3 g4((rows + 15) / 16);
    if (D <= 512) hipLaunchKernelGGL((ln_row_stats_multi_kernel<1, 4>), g4, dim3(256), 0, stream, x, x_stride, out, rows, D, eps);
    else hipLaunchKernelGGL((ln_row_stats_multi_kernel<2, 4>), g4, dim3(256), 0, stream, x, x_stride, out, rows, D, eps);
    return hipGetLastError();
  }
  const dim3 grid((rows + 3) / 4);
#define LM_LNS(C) \
  hipLaunchKernelGGL(ln_row_stats_kernel<C>, grid, dim3(256), 0, stream, x, x_stride, out, rows, D, eps, q8, ldq, qs, ldqs)
  if (D <= 512) LM_LNS(1);
  else if (D <= 1024) LM_LNS(2);
  else if (D <= 2048) LM_LNS(4);
  else LM_LNS(8);
#undef LM_LNS
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) l2norm_f32_kernel(float* __restrict__ x, int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float* xr = x + (int64_t)row * D;
  float s = 0.f;
  for (int i = lane; i < D; i += 64) s += xr[i] * xr[i];
  s = wave_sum(s);
  const float inv = 1.0f / fmaxf(sqrtf(s), eps);
  for (int i = lane; i < D; i += 64) xr[i] *= inv;
}

hipError_t l2norm_f32(float* x, int rows, int D, float eps, hipStream_t stream) {
  hipLaunchKernelGGL(l2norm_f32_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, x, rows, D, eps);
  return hipGetLastError();
}

// x[b * S + 0, :] = cls[:] + pos[0, :]   (class token row of a ViT token buffer)
__global__ void cls_fill_kernel(uint16_t* __restrict__ x, int64_t seq_stride, const uint16_t* __restrict__ cls,
                                const uint16_t* __restrict__ pos, int D) {
  const int b = blockIdx.x;
  uint16_t* xr = x + (int64_t)b * seq_stride;
  for (int ch = threadIdx.x; ch < D / 8; ch += blockDim.x) {
    float c[8], p[8];
    unpack8(*(const u32x4_t*)(cls + ch * 8), c);
    unpack8(*(const u32x4_t*)(pos + ch * 8), p);
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] += p[i];
    *(u32x4_t*)(xr + ch * 8) = pack8(c);
  }
}

hipError_t cls_fill(uint16_t* x, int64_t seq_stride, const uint16_t* cls, const uint16_t* pos, int B, int D,
                    hipStream_t stream) {
  hipLaunchKernelGGL(cls_fill_kernel, dim3(B), dim3(128), 0, stream, x, seq_stride, cls, pos, D);
  return hipGetLastError();
}

// out[r, :] = table[ids[r], :] (+ pos[r % S, :])    token / position embedding gather
__global__ void embed_gather_kernel(const int64_t* __restrict__ ids, const uint16_t* __restrict__ table,
                                    const uint16_t* __restrict__ pos, int S, uint16_t* __restrict__ out,
                                    int rows, int D, int64_t vocab, int64_t id_offset) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  int64_t id = ids[row] - id_offset;
  const bool valid = id >= 0 && id < vocab;
  const uint16_t* tr = table + (valid ? id : 0) * D;
  const uint16_t* pr = pos ? pos + (int64_t)(row % S) * D : nullptr;
  for (int ch = lane; ch < D / 8; ch += 64) {
    float t[8];
    if (valid) unpack8(*(const u32x4_t*)(tr + ch * 8), t);
    else for (int i = 0; i < 8; ++i) t[i] = 0.f;
    if (pr) {
      float p[8];
      unpack8(*(const u32x4_t*)(pr + ch * 8), p);
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] += p[i];
    }
    *(u32x4_t*)(out + (int64_t)row * D + ch * 8) = pack8(t);
  }
}

hipError_t embed_gather(const int64_t* ids, const uint16_t* table, const uint16_t* pos, int S, uint16_t* out,
                        int rows, int D, int64_t vocab, int64_t id_offset, hipStream_t stream) {
  hipLaunchKernelGGL(embed_gather_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, ids, table, pos, S, out,
                     rows, D, vocab, id_offset);
  return hipGetLastError();
}

}  // namespace lumen
