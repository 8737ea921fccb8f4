// Convolution and CNN-support kernels (NHWC bf16) for the face (SCRFD/RetinaFace,
// IResNet ArcFace) and OCR (DBNet, LCNet/SVTR recogniser) towers.
//
// conv2d_igemm: implicit-GEMM convolution on MFMA.  GEMM view:
//   M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin,
//   A[m][k] = x[n, ho*sh-ph+ky*dh, wo*sw-pw+kx*dw, ci]  (zero outside),
//   B[n][k] = w[cout][ky][kx][ci]                       ([Cout, KH, KW, Cin] layout)
// A 16-byte A-chunk is 8 consecutive input channels of one tap (Cin % 8 == 0),
// gathered straight from NHWC memory into the XOR-swizzled LDS tile (no im2col
// buffer); the tap / channel cursor of every staging slot advances
// incrementally per K-tile.  The output tile is NHWC = the GEMM C layout, so the
// shared epilogue fuses bias (folded BN), activation, per-channel PReLU and the
// residual add, and can write into a channel slice of a wider tensor (concat).
//
// Replaces the Conv / BatchNormalization / Relu / PRelu / Add ONNX nodes of the
// reference's detection.*.onnx / recognition.*.onnx graphs.
#include <algorithm>
#include <cstdlib>

#include "conv.h"
#include "gemm_epi.h"

namespace lumen {

constexpr int CBK = 64;

template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(WM* WN * 64) conv_igemm_kernel(ConvArgs a, GemmEpi ep) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int CA = BM * 8 / NT;
  constexpr int CB = BN * 8 / NT;
  static_assert(CA >= 1 && CB >= 1 && BM * 8 % NT == 0 && BN * 8 % NT == 0, "tiling");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;
  char* sB = smem + 2 * BM * 128;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int M = a.N * a.Ho * a.Wo, Nn = a.Cout, K = a.KH * a.KW * a.Cin;
  const int tiles_n = (Nn + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;

  // ---- A staging slots: output pixel + incremental (tap, ci) cursor
  const uint16_t* xb[CA];
  int hb[CA], wb[CA], ci[CA], ky[CA], kx[CA], kk[CA], la[CA];
  bool mv[CA];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int id = tid + i * NT, r = id >> 3, c = id & 7;
    const int m = m0 + r;
    mv[i] = m < M;
    const int mm = mv[i] ? m : 0;
    const int img = mm / (a.Ho * a.Wo), rem = mm % (a.Ho * a.Wo);
    const int ho = rem / a.Wo, wo = rem % a.Wo;
    xb[i] = a.x + (int64_t)img * a.H * a.W * a.ldx;
    hb[i] = ho * a.sh - a.ph;
    wb[i] = wo * a.sw - a.pw;
    kk[i] = c * 8;
    const int tap = kk[i] / a.Cin;
    ci[i] = kk[i] % a.Cin;
    ky[i] = tap / a.KW;
    kx[i] = tap % a.KW;
    la[i] = swz(r, c);
  }
  const uint16_t* pb[CB];
  int lb[CB], kb[CB];
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int id = tid + i * NT, r = id >> 3, c = id & 7;
    pb[i] = a.w + (int64_t)min(n0 + r, Nn - 1) * K + c * 8;
    kb[i] = c * 8;
    lb[i] = swz(r, c);
  }

  auto load_a = [&](int i) -> u32x4_t {
    const int hi = hb[i] + ky[i] * a.dh, wi = wb[i] + kx[i] * a.dw;
    const bool ok = mv[i] && kk[i] < K && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
    u32x4_t v = (u32x4_t){0u, 0u, 0u, 0u};
    if (ok) v = *(const u32x4_t*)(xb[i] + ((int64_t)hi * a.W + wi) * a.ldx + ci[i]);
    return v;
  };
  auto advance_a = [&](int i) {
    kk[i] += CBK;
    ci[i] += CBK;
    while (ci[i] >= a.Cin) {
      ci[i] -= a.Cin;
      if (++kx[i] == a.KW) { kx[i] = 0; ++ky[i]; }
    }
  };
  auto load_b = [&](int i, int koff) -> u32x4_t {
    u32x4_t v = (u32x4_t){0u, 0u, 0u, 0u};
    if (kb[i] + koff < K) v = *(const u32x4_t*)(pb[i] + koff);
    return v;
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  u32x4_t ra[CA], rb[CB];
  const int nk = (K + CBK - 1) / CBK;
#pragma unroll
  for (int i = 0; i < CA; ++i) ra[i] = load_a(i);
#pragma unroll
  for (int i = 0; i < CB; ++i) rb[i] = load_b(i, 0);
#pragma unroll
  for (int i = 0; i < CA; ++i) *(u32x4_t*)(sA + la[i]) = ra[i];
#pragma unroll
  for (int i = 0; i < CB; ++i) *(u32x4_t*)(sB + lb[i]) = rb[i];
  __syncthreads();

  const int frow = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
#pragma unroll
      for (int i = 0; i < CA; ++i) { advance_a(i); ra[i] = load_a(i); }
#pragma unroll
      for (int i = 0; i < CB; ++i) rb[i] = load_b(i, (kt + 1) * CBK);
    }
    const char* tA = sA + cur * BM * 128;
    const char* tB = sB + cur * BN * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t fa[MR], fb[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) fa[i] = *(const bf16x8_t*)(tA + swz(wm * TM + i * 16 + frow, s * 4 + fq));
#pragma unroll
      for (int j = 0; j < NR; ++j) fb[j] = *(const bf16x8_t*)(tB + swz(wn * TN + j * 16 + frow, s * 4 + fq));
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      char* nA = sA + (cur ^ 1) * BM * 128;
      char* nB = sB + (cur ^ 1) * BN * 128;
#pragma unroll
      for (int i = 0; i < CA; ++i) *(u32x4_t*)(nA + la[i]) = ra[i];
#pragma unroll
      for (int i = 0; i < CB; ++i) *(u32x4_t*)(nB + lb[i]) = rb[i];
    }
    __syncthreads();
  }

  constexpr int LDSTR = TN + 4;
  float* es = (float*)smem + wid * 16 * LDSTR;
  constexpr int LPR = TN / 16;
  constexpr int RPP = 64 / LPR;
  constexpr int NPASS = RPP >= 16 ? 1 : 16 / RPP;
  Unroll<0, MR>::run([&](const int i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) es[(fq * 4 + r) * LDSTR + j * 16 + frow] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int rr = p * RPP + lane / LPR;
      const int cc = (lane % LPR) * 16;
      if (rr < 16) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
          v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
        }
        if (ep.aff_s)
          epi_store16_t<false, true>(v, m0 + wm * TM + i * 16 + rr, n0 + wn * TN + cc, M, Nn, a.out, a.ldo, ep,
                                     c_rsrc(a.out));
        else
          epi_store16(v, m0 + wm * TM + i * 16 + rr, n0 + wn * TN + cc, M, Nn, a.out, a.ldo, ep);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  });
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_conv(const ConvArgs& a, const GemmEpi& ep, hipStream_t stream) {
  const int M = a.N * a.Ho * a.Wo;
  const int tiles = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  size_t lds = 2 * (size_t)(BM + BN) * 128;
  const size_t epi = (size_t)WM * WN * 16 * (BN / WN + 4) * 4;
  if (epi > lds) lds = epi;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<BM, BN, WM, WN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN>), dim3(tiles), dim3(WM * WN * 64), lds, stream, a, ep);
  return hipGetLastError();
}

bool conv_lds_ok(const ConvArgs& a);
bool conv_lds_small_ok(const ConvArgs& a);
hipError_t conv2d_lds(const ConvArgs& a, const GemmEpi& ep, int variant, hipStream_t stream);
hipError_t conv2d_lds_small(const ConvArgs& a, const GemmEpi& ep, int variant, hipStream_t stream);

// tile: -1 auto, 0..2 register-staged configs, 10 + v the LDS-DMA pipeline (conv_lds.hip, v = variant)
hipError_t conv2d_igemm(const ConvArgs& a0, const GemmEpi& ep, int tile, hipStream_t stream) {
  ConvArgs a = a0;
  a.div_hw = make_fastdiv((uint32_t)(a.Ho * a.Wo));
  a.div_w = make_fastdiv((uint32_t)a.Wo);
  a.div_kw = make_fastdiv((uint32_t)a.KW);
  const int64_t M = (int64_t)a.N * a.Ho * a.Wo;
  if (tile >= 10) return conv2d_lds(a, ep, tile - 10, stream);
  // Cin % 64 == 0 layers (IResNet, SCRFD / DBNet trunks): the LDS-DMA pipeline
  // (profiles/r2_conv_lds_v1.txt); other shapes use the register-staged kernels
  if (tile < 0 && conv_lds_ok(a)) return conv2d_lds(a, ep, 0, stream);
  // Cin 8 / 16 / 32 stems: the same pipeline with several taps per K step -- 128 x 64 tiles for
  // Cout >= 64 (IResNet stem 245 -> 152 us, SCRFD 32 -> 64 stride-2 conv 187 -> 129 us at 128 faces /
  // 32 images), 128 x 32 for Cout 32 (SCRFD 640 px stems 298 -> 276 and 349 -> 327 us)
  // (profiles/r4_conv_small_cin_v2.jsonl)
  if (tile < 0 && a.KH * a.KW >= 9 && conv_lds_small_ok(a))     // spatial stems, not 1x1 pointwise
    return conv2d_lds_small(a, ep, a.Cout >= 64 ? 10 : 9, stream);
  if (tile < 0) {
    const int64_t t128 = ((M + 127) / 128) * ((a.Cout + 127) / 128);
    if (a.Cout >= 128 && t128 >= 256) tile = 0;
    else if (a.Cout >= 64) tile = 1;
    else tile = 2;
  }
  switch (tile) {
    case 0: return launch_conv<128, 128, 2, 2>(a, ep, stream);
    case 1: return launch_conv<128, 64, 2, 2>(a, ep, stream);
    default: return launch_conv<128, 32, 4, 1>(a, ep, stream);
  }
}

// ---------------------------------------------------------------------------- depthwise
// one thread = 8 channels of one output pixel; weights [KH, KW, C]
__global__ void __launch_bounds__(256)
dw_conv_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, const void* __restrict__ bias,
               int bias_f32, void* __restrict__ out, int N, int H, int W, int C, int KH, int KW, int sh, int sw,
               int ph, int pw, int dh, int dw, int Ho, int Wo, int act, int out_f32) {
  const int CG = C >> 3;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * Ho * Wo * CG;
  if (gid >= total) return;
  const int cg = gid % CG;
  const int64_t pix = gid / CG;
  const int wo = pix % Wo, ho = (pix / Wo) % Ho, n = pix / ((int64_t)Wo * Ho);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const uint16_t* xn = x + (int64_t)n * H * W * C + cg * 8;
  for (int ky = 0; ky < KH; ++ky) {
    const int hi = ho * sh - ph + ky * dh;
    if (hi < 0 || hi >= H) continue;
    for (int kx = 0; kx < KW; ++kx) {
      const int wi = wo * sw - pw + kx * dw;
      if (wi < 0 || wi >= W) continue;
      float xv[8], wv[8];
      unpack8(*(const u32x4_t*)(xn + ((int64_t)hi * W + wi) * C), xv);
      unpack8(*(const u32x4_t*)(w + (ky * KW + kx) * C + cg * 8), wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += xv[i] * wv[i];
    }
  }
  if (bias) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      acc[i] += bias_f32 ? ((const float*)bias)[cg * 8 + i] : bf2f(((const uint16_t*)bias)[cg * 8 + i]);
  }
  apply_act_n<8>(acc, act);
  if (out_f32) {
    float* o = (float*)out + pix * C + cg * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = acc[i];
  } else {
    *(u32x4_t*)((uint16_t*)out + pix * C + cg * 8) = pack8(acc);
  }
}

// Register-blocked variant (dilation 1, KW in {3, 5, 7}, stride SW in {1, 2}): one thread =
// 8 channels x PX consecutive output pixels of one row.  Per kernel row it loads the
// (PX-1)*SW + KW input columns once into registers and slides the KW taps over them, so
// a 7x7 stride-1 conv issues 10 instead of 28 16-byte loads per 4 outputs and reads each
// weight row once per 4 outputs (FastViT / MobileCLIP RepMixer, ConvMlp, RepCPE and
// PatchEmbed convs are 3x3 / 7x7 depthwise).  Channel groups are the fastest thread
// index, so a wave reads 64 x 16 contiguous bytes of an NHWC row per load.
template <int KW, int SW, int PX>
__global__ void __launch_bounds__(256)
dw_conv_rb_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, const void* __restrict__ bias,
                  int bias_f32, void* __restrict__ out, int N, int H, int W, int C, int KH, int sh, int ph, int pw,
                  int Ho, int Wo, int act, int out_f32) {
  constexpr int SPAN = (PX - 1) * SW + KW;
  const int CG = C >> 3;
  const int WB = (Wo + PX - 1) / PX;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * Ho * WB * CG;
  if (gid >= total) return;
  const int cg = gid % CG;
  const int64_t r = gid / CG;
  const int wb = r % WB, ho = (r / WB) % Ho, n = r / ((int64_t)WB * Ho);
  const int wo0 = wb * PX;
  const int wi0 = wo0 * SW - pw;
  float acc[PX][8];
#pragma unroll
  for (int p = 0; p < PX; ++p)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[p][i] = 0.f;
  const uint16_t* xn = x + (int64_t)n * H * W * C + cg * 8;
  for (int ky = 0; ky < KH; ++ky) {
    const int hi = ho * sh - ph + ky;
    if (hi < 0 || hi >= H) continue;
    const uint16_t* xr = xn + (int64_t)hi * W * C;
    u32x4_t xv[SPAN];
#pragma unroll
    for (int j = 0; j < SPAN; ++j) {
      const int wi = wi0 + j;
      xv[j] = (wi >= 0 && wi < W) ? *(const u32x4_t*)(xr + (int64_t)wi * C) : (u32x4_t){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int kx = 0; kx < KW; ++kx) {
      float wv[8];
      unpack8(*(const u32x4_t*)(w + (ky * KW + kx) * C + cg * 8), wv);
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        float xf[8];
        unpack8(xv[p * SW + kx], xf);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[p][i] += xf[i] * wv[i];
      }
    }
  }
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      bv[i] = bias_f32 ? ((const float*)bias)[cg * 8 + i] : bf2f(((const uint16_t*)bias)[cg * 8 + i]);
  }
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    if (wo0 + p >= Wo) break;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[p][i] += bv[i];
    apply_act_n<8>(acc[p], act);
    const int64_t pix = ((int64_t)n * Ho + ho) * Wo + wo0 + p;
    if (out_f32) {
      float* o = (float*)out + pix * C + cg * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = acc[p][i];
    } else {
      *(u32x4_t*)((uint16_t*)out + pix * C + cg * 8) = pack8(acc[p]);
    }
  }
}

template <int KW, int SW>
static hipError_t launch_dw_rb(const uint16_t* x, const uint16_t* w, const void* bias, int bias_f32, void* out, int N,
                               int H, int W, int C, int KH, int sh, int ph, int pw, int Ho, int Wo, int act,
                               int out_f32, hipStream_t stream) {
  constexpr int PX = 4;
  const int64_t total = (int64_t)N * Ho * ((Wo + PX - 1) / PX) * (C / 8);
  hipLaunchKernelGGL((dw_conv_rb_kernel<KW, SW, PX>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x,
                     w, bias, bias_f32, out, N, H, W, C, KH, sh, ph, pw, Ho, Wo, act, out_f32);
  return hipGetLastError();
}

hipError_t conv2d_depthwise(const uint16_t* x, const uint16_t* w, const void* bias, int bias_f32, void* out, int N,
                            int H, int W, int C, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw,
                            int Ho, int Wo, int act, int out_f32, hipStream_t stream) {
  if (dh == 1 && dw == 1 && (sw == 1 || sw == 2)) {
#define LM_DW_CASE(K)                                                                                       \
    if (KW == K) return sw == 1 ? launch_dw_rb<K, 1>(x, w, bias, bias_f32, out, N, H, W, C, KH, sh, ph, pw, Ho, Wo, act, \
                                                     out_f32, stream)                                          \
                                : launch_dw_rb<K, 2>(x, w, bias, bias_f32, out, N, H, W, C, KH, sh, ph, pw, Ho, Wo, act, \
                                                     out_f32, stream);
    LM_DW_CASE(3)
    LM_DW_CASE(5)
    LM_DW_CASE(7)
#undef LM_DW_CASE
  }
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(dw_conv_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, w, bias,
                     bias_f32, out, N, H, W, C, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo, act, out_f32);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- per-channel affine (+act/PReLU)
__global__ void channel_affine_kernel(const uint16_t* __restrict__ x, const float* __restrict__ scale,
                                      const float* __restrict__ shift, uint16_t* __restrict__ out, int64_t rows,
                                      int C, int act, const uint16_t* __restrict__ prelu) {
  const int CG = C >> 3;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= rows * CG) return;
  const int cg = gid % CG;
  float v[8];
  unpack8(*(const u32x4_t*)(x + gid * 8), v);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = v[i] * scale[cg * 8 + i] + shift[cg * 8 + i];
  apply_act_n<8>(v, act);
  if (prelu) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float s = bf2f(prelu[cg * 8 + i]);
      v[i] = v[i] > 0.f ? v[i] : v[i] * s;
    }
  }
  *(u32x4_t*)(out + gid * 8) = pack8(v);
}

hipError_t channel_affine(const uint16_t* x, const float* scale, const float* shift, uint16_t* out, int64_t rows,
                          int C, int act, const uint16_t* prelu, hipStream_t stream) {
  const int64_t total = rows * (C / 8);
  hipLaunchKernelGGL(channel_affine_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, scale,
                     shift, out, rows, C, act, prelu);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- pooling
__global__ void pool2d_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out, int N, int H, int W, int C,
                              int KH, int KW, int sh, int sw, int ph, int pw, int Ho, int Wo, int is_max) {
  const int CG = C >> 3;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * Ho * Wo * CG;
  if (gid >= total) return;
  const int cg = gid % CG;
  const int64_t pix = gid / CG;
  const int wo = pix % Wo, ho = (pix / Wo) % Ho, n = pix / ((int64_t)Wo * Ho);
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = is_max ? -INFINITY : 0.f;
  int cnt = 0;
  for (int ky = 0; ky < KH; ++ky) {
    const int hi = ho * sh - ph + ky;
    if (hi < 0 || hi >= H) continue;
    for (int kx = 0; kx < KW; ++kx) {
      const int wi = wo * sw - pw + kx;
      if (wi < 0 || wi >= W) continue;
      float v[8];
      unpack8(*(const u32x4_t*)(x + (((int64_t)n * H + hi) * W + wi) * C + cg * 8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = is_max ? fmaxf(acc[i], v[i]) : acc[i] + v[i];
      ++cnt;
    }
  }
  if (!is_max) {
    const float inv = 1.f / (float)(KH * KW);  // count_include_pad=True (ONNX/PyTorch default)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= inv;
  }
  *(u32x4_t*)(out + pix * C + cg * 8) = pack8(acc);
}

hipError_t pool2d(const uint16_t* x, uint16_t* out, int N, int H, int W, int C, int KH, int KW, int sh, int sw, int ph,
                  int pw, int Ho, int Wo, int is_max, hipStream_t stream) {
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(pool2d_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, out, N, H, W, C,
                     KH, KW, sh, sw, ph, pw, Ho, Wo, is_max);
  return hipGetLastError();
}

// mean over HW per (n, c) -> f32 [N, C]; one block per (n, 256-channel group)
__global__ void global_avgpool_kernel(const uint16_t* __restrict__ x, float* __restrict__ out, int HW, int C) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;  // 4 row-partitions
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < C) {
    const uint16_t* xn = x + (int64_t)n * HW * C + c;
    for (int p = part; p < HW; p += 4) s += bf2f(xn[(int64_t)p * C]);
  }
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && c < C)
    out[(int64_t)n * C + c] = (red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]) / HW;
}

hipError_t global_avgpool(const uint16_t* x, float* out, int N, int HW, int C, hipStream_t stream) {
  hipLaunchKernelGGL(global_avgpool_kernel, dim3((C + 63) / 64, N), dim3(256), 0, stream, x, out, HW, C);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- FPN helpers
// out[n, h, w, :] (pixel stride ldo) = x[n, h/f, w/f, :] (+ add[n, h, w, :])   nearest upsample
__global__ void upsample_add_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ add,
                                    uint16_t* __restrict__ out, int N, int H, int W, int C, int f, int64_t ldo) {
  const int CG = C >> 3;
  const int Ho = H * f, Wo = W * f;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)N * Ho * Wo * CG) return;
  const int cg = gid % CG;
  const int64_t pix = gid / CG;
  const int wo = pix % Wo, ho = (pix / Wo) % Ho, n = pix / ((int64_t)Wo * Ho);
  float v[8];
  unpack8(*(const u32x4_t*)(x + (((int64_t)n * H + ho / f) * W + wo / f) * C + cg * 8), v);
  if (add) {
    float a2[8];
    unpack8(*(const u32x4_t*)(add + pix * C + cg * 8), a2);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += a2[i];
  }
  *(u32x4_t*)(out + pix * ldo + cg * 8) = pack8(v);
}

hipError_t upsample_add(const uint16_t* x, const uint16_t* add, uint16_t* out, int N, int H, int W, int C, int f,
                        int64_t ldo, hipStream_t stream) {
  const int64_t total = (int64_t)N * H * f * W * f * (C / 8);
  hipLaunchKernelGGL(upsample_add_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, add, out,
                     N, H, W, C, f, ldo);
  return hipGetLastError();
}

// SE channel re-weighting: x[n, p, c] *= s[n, c]
__global__ void channel_scale_kernel(uint16_t* __restrict__ x, const float* __restrict__ s, int HW, int C,
                                     int64_t total) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= total) return;
  const int CG = C >> 3;
  const int cg = gid % CG;
  const int64_t n = gid / ((int64_t)HW * CG);
  float v[8];
  unpack8(*(const u32x4_t*)(x + gid * 8), v);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= s[n * C + cg * 8 + i];
  *(u32x4_t*)(x + gid * 8) = pack8(v);
}

hipError_t channel_scale(uint16_t* x, const float* s, int N, int HW, int C, hipStream_t stream) {
  const int64_t total = (int64_t)N * HW * (C / 8);
  hipLaunchKernelGGL(channel_scale_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, s, HW, C,
                     total);
  return hipGetLastError();
}

// ConvTranspose(k=f, s=f) as GEMM + depth-to-space: y [N, H, W, f*f*C] (GEMM output,
// channel index (dy*f + dx)*C + c) -> out [N, H*f, W*f, C]
__global__ void pixel_shuffle_kernel(const uint16_t* __restrict__ y, uint16_t* __restrict__ out, int N, int H, int W,
                                     int C, int f) {
  const int CG = C >> 3;
  const int Ho = H * f, Wo = W * f;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)N * Ho * Wo * CG) return;
  const int cg = gid % CG;
  const int64_t pix = gid / CG;
  const int wo = pix % Wo, ho = (pix / Wo) % Ho, n = pix / ((int64_t)Wo * Ho);
  const int h = ho / f, dy = ho % f, w = wo / f, dx = wo % f;
  const uint16_t* src = y + (((int64_t)n * H + h) * W + w) * (f * f * C) + (dy * f + dx) * C + cg * 8;
  *(u32x4_t*)(out + pix * C + cg * 8) = *(const u32x4_t*)src;
}

hipError_t pixel_shuffle_up(const uint16_t* y, uint16_t* out, int N, int H, int W, int C, int f, hipStream_t stream) {
  const int64_t total = (int64_t)N * H * f * W * f * (C / 8);
  hipLaunchKernelGGL(pixel_shuffle_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, y, out, N, H,
                     W, C, f);
  return hipGetLastError();
}

// DBNet head tail in one pass: up1 (2x2 stride-2 ConvTranspose C -> C, folded BN, ReLU) and up2
// (2x2 stride-2 ConvTranspose C -> 1, sigmoid) of each 1/4-scale pixel are independent of every
// other pixel, so one wave takes 16 pixels through both on the MFMA and writes their 4x4 blocks of
// the full-resolution probability map.  Replaces two GEMMs (K padded 32 -> 64, a 256-wide tile on
// N = 128 / 4), the pixel shuffle and the final permute copy, which between them read and wrote the
// 4C-channel half-scale intermediate several times (~0.9 ms per 16-image batch at 960 px).
//
// up1 runs transposed, X^T[ch][px] = W1[ch][:] . h[px][:] (A = W1 rows, B = the pixels' channels), so
// the accumulator of channel block (s1, blk) holds channels 4*hq + r on lane (px, hq).  ReLU'd and
// rounded to bf16, the two blocks of sub-position s1 ARE the B operand of up2's k-step s1 (k order
// permuted: element j of lane-quarter hq is channel j < 4 ? 4hq + j : 12 + 4hq + j); the host packs
// up2's weights in that order into w2p [4 s1][64 lanes][8], nonzero only on A rows 4*s1 .. 4*s1+3,
// so the four k-steps accumulate Y[4*s1 + s2][px] and every lane ends with its own (s1, 4 x s2).
// The rounding points match the unfused path (bf16 up1 output, fp32 up2 accumulate + sigmoid).
template <int C>
__global__ void __launch_bounds__(256) db_head_up_kernel(const uint16_t* __restrict__ h, const uint16_t* __restrict__ w1,
                                                         const float* __restrict__ b1, const uint16_t* __restrict__ w2p,
                                                         const float* __restrict__ b2, float* __restrict__ out,
                                                         int64_t P, int H4, int W4) {
  constexpr int NB = C / 16;     // up1 16-channel blocks per sub-position
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, hq = lane >> 4;
  const bool kin = 8 * hq < C;   // this lane-quarter's 8 input channels exist
  bf16x8_t a1[4 * NB];
  float bias1[4 * NB][4];
#pragma unroll
  for (int b = 0; b < 4 * NB; ++b) {
    u32x4_t v = {0u, 0u, 0u, 0u};
    if (kin) v = *(const u32x4_t*)(w1 + (int64_t)(16 * b + r16) * C + 8 * hq);
    a1[b] = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
    for (int r = 0; r < 4; ++r) bias1[b][r] = b1[16 * b + 4 * hq + r];
  }
  bf16x8_t a2[4];
#pragma unroll
  for (int s1 = 0; s1 < 4; ++s1) a2[s1] = __builtin_bit_cast(bf16x8_t, *(const u32x4_t*)(w2p + (s1 * 64 + lane) * 8));
  const float c0 = b2[0], c1 = b2[1], c2 = b2[2], c3 = b2[3];
  const int64_t groups = (P + 15) / 16;
  const int64_t HW = (int64_t)H4 * W4, Wo = 4LL * W4;
  const f32x4_t zero = {0.f, 0.f, 0.f, 0.f};
  for (int64_t g = (int64_t)blockIdx.x * 4 + wave; g < groups; g += (int64_t)gridDim.x * 4) {
    const int64_t p = g * 16 + r16;
    u32x4_t xv = {0u, 0u, 0u, 0u};
    if (p < P && kin) xv = *(const u32x4_t*)(h + p * C + 8 * hq);
    const bf16x8_t bx = __builtin_bit_cast(bf16x8_t, xv);
    f32x4_t y = zero;
#pragma unroll
    for (int s1 = 0; s1 < 4; ++s1) {
      const f32x4_t x0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s1 * NB], bx, zero, 0, 0, 0);
      float t[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) t[r] = fmaxf(x0[r] + bias1[s1 * NB][r], 0.f);
      if constexpr (NB == 2) {
        const f32x4_t x1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s1 * NB + 1], bx, zero, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) t[4 + r] = fmaxf(x1[r] + bias1[s1 * NB + 1][r], 0.f);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) t[4 + r] = 0.f;
      }
      y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[s1], __builtin_bit_cast(bf16x8_t, pack8(t)), y, 0, 0, 0);
    }
    if (p < P) {     // lane = (pixel r16, s1 = hq): rows 2*kh1 + {0, 1}, columns 2*kw1 + {0, 1} of its 4x4 block
      const int64_t n = p / HW;
      const int rem = (int)(p - n * HW);
      const int yy = rem / W4, xx = rem - yy * W4;
      float* o = out + (n * 4 * H4 + 4 * yy + 2 * (hq >> 1)) * Wo + 4 * xx + 2 * (hq & 1);
      *(float2*)o = make_float2(act_fn<ACT_SIGMOID>(y[0] + c0), act_fn<ACT_SIGMOID>(y[1] + c1));
      *(float2*)(o + Wo) = make_float2(act_fn<ACT_SIGMOID>(y[2] + c2), act_fn<ACT_SIGMOID>(y[3] + c3));
    }
  }
}

hipError_t db_head_up(const uint16_t* h, const uint16_t* w1, const float* b1, const uint16_t* w2p, const float* b2,
                      float* out, int N, int H4, int W4, int C, hipStream_t stream) {
  const int64_t P = (int64_t)N * H4 * W4;
  const int64_t groups = (P + 15) / 16;
  const int wgs = (int)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, 2048));   // 8 per CU of 256, grid-stride
  if (C == 32)
    hipLaunchKernelGGL(db_head_up_kernel<32>, dim3(wgs), dim3(256), 0, stream, h, w1, b1, w2p, b2, out, P, H4, W4);
  else if (C == 16)
    hipLaunchKernelGGL(db_head_up_kernel<16>, dim3(wgs), dim3(256), 0, stream, h, w1, b1, w2p, b2, out, P, H4, W4);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace lumen
