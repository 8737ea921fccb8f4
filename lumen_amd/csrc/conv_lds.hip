// Implicit-GEMM convolution on the 128 x BN LDS-DMA pipeline of gemm_f8.hip (bf16 form):
// NSTAGE K-stages of global_load_lds (16 B per lane, XOR swizzle on the source address),
// one counted vmcnt + raw barrier per K-step, 2 x WN waves with 64 x (BN/WN) wave tiles of
// v_mfma_f32_16x16x32_bf16.  For Cin % 64 == 0 one 64-wide K-step is 64 channels of ONE
// filter tap, so every LDS row of the A stage is a single contiguous 128-byte run of an
// NHWC input pixel -- the gather is pure address arithmetic on the DMA source (taps that
// fall into the zero padding read past the end of the buffer descriptor: zeros).  Replaces the register-staged
// 2-stage conv_igemm_kernel on the IResNet / SCRFD / DBNet layers with Cin >= 64
// (r1: 55 us per call, 1.3 % of peak on face).
//
// GEMM view (conv.hip): M = N*Ho*Wo, N = Cout, K = KH*KW*Cin, A[m][k] = x[n, ho*sh-ph+ky*dh,
// wo*sw-pw+kx*dw, ci], B = w [Cout, KH, KW, Cin]; C = NHWC output (pixel stride ldo) through
// the shared GemmEpi epilogue (folded-BN bias, activation, PReLU, residual, post-ReLU).
#include <cstdlib>

#include "common.h"
#include "conv.h"
#include "gemm_epi.h"

namespace lumen {

// SMALLC: Cin in {8, 16, 32} (detector / recogniser stems): one 64-wide K step spans 64 / Cin
// filter taps, so a lane's 16-byte chunk picks its own tap -- tap = step * (64 / Cin) + chunk / (Cin / 8)
// -- and its offset comes from a per-workgroup LDS table of tap offsets; taps past KH * KW (the
// last, partial step) read zeros, and the B side's columns past K meet those zeros.
template <int NSTAGE, int WN, int BN, bool SMALLC = false>
__global__ void __launch_bounds__(128 * WN) conv_lds_kernel(ConvArgs a, GemmEpi ep) {
  constexpr int NW = 2 * WN;
  constexpr int TN = BN / WN;
  constexpr int NR = TN / 16;
  constexpr int PERA = 16 / NW;             // A: 128 rows = 16 x 8-row DMA units
  constexpr int PERB = BN / 8 / NW;          // B: BN rows
  static_assert(PERA >= 1 && PERB >= 1 && NR >= 1, "tiling");
  constexpr int ASZ = 128 * 128, STAGE = ASZ + BN * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t_start = ep.dbg ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  int64_t t_pro = 0, t_loop = 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int M = a.N * a.Ho * a.Wo, N = a.Cout, K = a.KH * a.KW * a.Cin;
  const int tiles_m = (M + 127) / 128, tiles_n = (N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = lin % tiles_m, tn = lin / tiles_m;
  const int m0 = tm * 128, n0 = tn * BN;

  // Operands through buffer descriptors, so the per-K-step source address is one 32-bit add:
  //   A row (output pixel) -> byte offset of its top-left input tap + this lane's 16 channels,
  //   plus a wave-uniform tap offset; a tap in the zero padding gets an offset past the end of
  //   the buffer, which the range check turns into 16 zero bytes in LDS.
  //   B row -> byte offset of this lane's 16 B in filter row n; the K step goes in soffset.
  // Tap validity is a per-row bit mask built once (bit t: tap t inside the image), so the
  // K loop does no division and no bounds arithmetic: r2 measured 5.6 VALU per MFMA on this
  // kernel from exactly that per-step index math (profiles/r2_face_pmc_sq_v1.jsonl).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)((int64_t)a.N * a.H * a.W * a.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, (int)((int64_t)N * K * 2), 0x00020000);
  int rofs[PERA];
  uint64_t tmask[PERA];
  int cchunk[PERA];
  const int row_step = a.dh * a.W * a.ldx * 2, col_step = a.dw * a.ldx * 2;
#pragma unroll
  for (int i = 0; i < PERA; ++i) {
    const int r = (PERA * wid + i) * 8 + (lane >> 3);
    cchunk[i] = (lane & 7) ^ ((r >> 1) & 7);                      // logical 16-byte chunk of the row
    const int ca = SMALLC ? 0 : cchunk[i] * 8;                     // channel offset of this lane's 16 B
    const int m = min(m0 + r, M - 1);
    const int img = (int)fdiv((uint32_t)m, a.div_hw), rem = m - img * (a.Ho * a.Wo);
    const int ho = (int)fdiv((uint32_t)rem, a.div_w), wo = rem - ho * a.Wo;
    const int hb = ho * a.sh - a.ph, wb = wo * a.sw - a.pw;
    rofs[i] = (((img * a.H + hb) * a.W + wb) * a.ldx + ca) * 2;   // wraps for padding rows: never used then
    // tap validity is separable: (row ky inside) x (column kx inside)
    uint32_t rok = 0, cok = 0;
    for (int ky = 0; ky < a.KH; ++ky) rok |= (uint32_t)((unsigned)(hb + ky * a.dh) < (unsigned)a.H) << ky;
    for (int kx = 0; kx < a.KW; ++kx) cok |= (uint32_t)((unsigned)(wb + kx * a.dw) < (unsigned)a.W) << kx;
    uint64_t msk = 0;
    for (int ky = 0; ky < a.KH; ++ky)
      if ((rok >> ky) & 1u) msk |= (uint64_t)cok << (ky * a.KW);
    tmask[i] = msk;
  }
  int wofs[PERB];
#pragma unroll
  for (int i = 0; i < PERB; ++i) {
    const int r = (PERB * wid + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    wofs[i] = (min(n0 + r, N - 1) * K + c * 8) * 2;
  }
  // wave-uniform walk over (tap, 64-channel block): advanced once per stage() call, in K order
  int ky = 0, kx = 0, c0 = 0, tofs = 0;
  uint64_t tbit = 1;
  const int cpt_log = a.Cin == 8 ? 0 : (a.Cin == 16 ? 1 : 2);   // SMALLC: 16-byte chunks per tap (log2)
  const int khw = a.KH * a.KW;
  auto stage = [&](int s, int kt) {
    char* baseA = smem + s * STAGE + wid * PERA * 1024;
#pragma unroll
    for (int i = 0; i < PERA; ++i) {
      int off;
      if constexpr (SMALLC) {
        const int t = (kt << (3 - cpt_log)) + (cchunk[i] >> cpt_log);
        const int ch = (cchunk[i] & ((1 << cpt_log) - 1)) * 16;
        // tap t -> (t / KW, t % KW) by multiply-high: no LDS table, so the stage buffers are the whole
        // LDS footprint (2 x 160 rows x 128 B = 40 KiB for 128 x 32 tiles: 4 workgroups per CU, not 3)
        const int ty = (int)fdiv((uint32_t)t, a.div_kw), tx = t - ty * a.KW;
        off = (t < khw && ((tmask[i] >> t) & 1ull)) ? rofs[i] + ty * row_step + tx * col_step + ch : (int)0x80000000;
      } else {
        off = (tmask[i] & tbit) ? rofs[i] + tofs : (int)0x80000000;
      }
      buf_load_lds16(xr, baseA + i * 1024, off, 0);
    }
    char* baseB = smem + s * STAGE + ASZ + wid * PERB * 1024;
#pragma unroll
    for (int i = 0; i < PERB; ++i)
      buf_load_lds16(wr, baseB + i * 1024, wofs[i], kt * 128);
    c0 += 64;
    tofs += 128;
    if (c0 == a.Cin) {
      c0 = 0;
      tbit <<= 1;
      if (++kx == a.KW) {
        kx = 0;
        ++ky;
      }
      tofs = ky * row_step + kx * col_step;
    }
  };

  f32x4_t acc[4][NR];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = SMALLC ? (K + 63) / 64 : K / 64;
  const int frow = lane & 15, g = lane >> 4;
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NSTAGE - 2 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((PERA + PERB) * (NSTAGE - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (ep.dbg && kt == 0) t_pro = (int64_t)__builtin_amdgcn_s_memrealtime();
    if (kt + NSTAGE - 1 < nk) stage((kt + NSTAGE - 1) % NSTAGE, kt + NSTAGE - 1);
    const char* sA = smem + (kt % NSTAGE) * STAGE;
    const char* sW = sA + ASZ;
    u32x4_t fa[4][2], fb[NR][2];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int r = wn * TN + j * 16 + frow;
      fb[j][0] = *(const u32x4_t*)(sW + swz(r, g));
      fb[j][1] = *(const u32x4_t*)(sW + swz(r, g + 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + i * 16 + frow;
      fa[i][0] = *(const u32x4_t*)(sA + swz(r, g));
      fa[i][1] = *(const u32x4_t*)(sA + swz(r, g + 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i][0]),
                                                            __builtin_bit_cast(bf16x8_t, fb[j][0]), acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i][1]),
                                                            __builtin_bit_cast(bf16x8_t, fb[j][1]), acc[i][j], 0, 0, 0);
      }
  }
  __syncthreads();
  if (ep.dbg) t_loop = (int64_t)__builtin_amdgcn_s_memrealtime();
  auto stamp = [&]() {   // profiling (tools/conv_timeline.py): wave 0's view of the tile
    if (ep.dbg && tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int64_t* d = ep.dbg + 4 * (int64_t)blockIdx.x;
      d[0] = t_start; d[1] = t_pro; d[2] = t_loop; d[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
  };

  constexpr int LDSTR = TN + 4;
  constexpr int LPR = TN / 16;
  constexpr int RPP = 64 / LPR;
  constexpr int NPASS = RPP >= 16 ? 1 : 16 / RPP;
  float* es = (float*)smem + wid * 16 * LDSTR;
  const int cc = (lane % LPR) * 16;
  const int n = n0 + wn * TN + cc;
  const __amdgpu_buffer_rsrc_t crs = c_rsrc(a.out);
  if (NPASS == 1 && !ep.out_f32 && !ep.bias_f32 && !ep.table && !ep.row_aff && !ep.out_group && !ep.glu &&
      ep.alpha == 1.f) {
    // Prefetched epilogue: a lane's 16 columns are the same in all 4 row slabs, so bias / PReLU /
    // output-affine vectors load once, and the 4 slabs' residual rows are all in flight before the
    // first slab is finished -- the generic path waits one L2 / HBM round trip per slab.  SL row
    // slabs go through LDS per pass, so all 64 lanes work when a wave tile is only 32 (16) columns
    // wide (RPP = 32 (64) rows per pass): half (a quarter) as many epilogue instructions per output.
    constexpr int SL = RPP >= 64 ? 4 : (RPP >= 32 ? 2 : 1);
    constexpr int NP = 4 / SL;
    constexpr int PR = 16 * SL;                 // rows per pass
    float* es2 = (float*)smem + wid * PR * LDSTR;
    const int rr = lane / LPR;                  // row within a pass
    const bool live = rr < PR && n < N;
    u32x4_t pb0 = {}, pb1 = {}, pp0 = {}, pp1 = {};
    u32x4_t pr[NP][2];
    f32x4_t ps[4], pt[4];
    if (live) {
      if (ep.bias) {
        const uint16_t* zb = (const uint16_t*)ep.bias + n;
        pb0 = *(const u32x4_t*)zb;
        pb1 = *(const u32x4_t*)(zb + 8);
      }
      if (ep.prelu) {
        pp0 = *(const u32x4_t*)(ep.prelu + n);
        pp1 = *(const u32x4_t*)(ep.prelu + n + 8);
      }
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int m = min(m0 + wm * 64 + p * PR + rr, M - 1);
        if (ep.residual) {
          const uint16_t* t = ep.residual + (int64_t)m * ep.ldr + n;
          pr[p][0] = *(const u32x4_t*)t;
          pr[p][1] = *(const u32x4_t*)(t + 8);
        }
      }
      if (ep.aff_s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ps[q] = *(const f32x4_t*)(ep.aff_s + n + 4 * q);
          pt[q] = *(const f32x4_t*)(ep.aff_t + n + 4 * q);
        }
      }
    }
    Unroll<0, NP>::run([&](const int p) {
#pragma unroll
      for (int sl = 0; sl < SL; ++sl)
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) es2[(sl * 16 + g * 4 + r) * LDSTR + j * 16 + frow] = acc[p * SL + sl][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int m = m0 + wm * 64 + p * PR + rr;
      if (live && m < M) {
        float v[16], f[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4_t t = *(const f32x4_t*)(es2 + rr * LDSTR + cc + q * 4);
          v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
        }
        if (ep.bias) {
          unpack8(pb0, f);
          unpack8(pb1, f + 8);
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] += f[q];
        }
        if (ep.act) apply_act_n<16>(v, ep.act);
        if (ep.prelu) {
          unpack8(pp0, f);
          unpack8(pp1, f + 8);
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = v[q] > 0.f ? v[q] : v[q] * f[q];
        }
        if (ep.residual) {
          unpack8(pr[p][0], f);
          unpack8(pr[p][1], f + 8);
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] += f[q];
        }
        if (ep.post_act) {
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = fmaxf(v[q], 0.f);
        }
        const int64_t o = (int64_t)m * a.ldo + n;
        if (ep.aff_s) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) f[4 * q + r] = bf2f(f2bf(v[4 * q + r])) * ps[q][r] + pt[q][r];
          if (ep.aff_out) {
            uint16_t* o2 = ep.aff_out + (int64_t)m * ep.ld_aff + n;
            *(u32x4_t*)o2 = pack8(f);
            *(u32x4_t*)(o2 + 8) = pack8(f + 8);
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = f[q];
          }
        }
        st16<false>(a.out, crs, o * 2, pack8(v));
        st16<false>(a.out, crs, (o + 8) * 2, pack8(v + 8));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    });
    stamp();
    return;
  }
  Unroll<0, 4>::run([&](const int i) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) es[(g * 4 + r) * LDSTR + j * 16 + frow] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int rr = p * RPP + lane / LPR;
      if (rr >= 16) continue;
      const int m = m0 + wm * 64 + i * 16 + rr;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4_t t = *(const f32x4_t*)(es + rr * LDSTR + cc + q * 4);
        v[q * 4 + 0] = t[0]; v[q * 4 + 1] = t[1]; v[q * 4 + 2] = t[2]; v[q * 4 + 3] = t[3];
      }
      if (ep.aff_s) epi_store16_t<false, true>(v, m, n, M, N, a.out, a.ldo, ep, crs);
      else epi_store16_t<false>(v, m, n, M, N, a.out, a.ldo, ep, crs);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  });
  stamp();
}

template <int NS, int WN, int BN, bool SMALLC = false>
static hipError_t launch_conv_lds(const ConvArgs& a, const GemmEpi& ep, hipStream_t stream) {
  const size_t lds = (size_t)NS * (128 + BN) * 128;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_lds_kernel<NS, WN, BN, SMALLC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int M = a.N * a.Ho * a.Wo;
  const int tiles = ((M + 127) / 128) * ((a.Cout + BN - 1) / BN);
  hipLaunchKernelGGL((conv_lds_kernel<NS, WN, BN, SMALLC>), dim3(tiles), dim3(128 * WN), lds, stream, a, ep);
  return hipGetLastError();
}

bool conv_lds_small_ok(const ConvArgs& a) {
  // the small-Cin form: Cin 8 / 16 / 32, K steps of 64 / Cin taps
  return (a.Cin == 8 || a.Cin == 16 || a.Cin == 32) && a.Cout % 16 == 0 && a.ldx % 8 == 0 && a.ldo % 8 == 0 &&
         ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.w & 15) == 0 && (int64_t)a.N * a.Ho * a.Wo < (1LL << 31) &&
         (int64_t)a.N * a.H * a.W * a.ldx * 2 < (1LL << 31) && (int64_t)a.Cout * a.KH * a.KW * a.Cin * 2 < (1LL << 31) &&
         a.KH * a.KW <= 64;
}

bool conv_lds_ok(const ConvArgs& a) {
  // 32-bit buffer offsets: input and filter below 2 GiB (the padding sentinel 0x80000000 lies
  // past both); <= 64 filter taps (the per-row validity mask)
  return a.Cin % 64 == 0 && a.Cout % 16 == 0 && a.ldx % 8 == 0 && a.ldo % 8 == 0 &&
         ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.w & 15) == 0 && (int64_t)a.N * a.Ho * a.Wo < (1LL << 31) &&
         (int64_t)a.N * a.H * a.W * a.ldx * 2 < (1LL << 31) && (int64_t)a.Cout * a.KH * a.KW * a.Cin * 2 < (1LL << 31) &&
         a.KH * a.KW <= 64;
}

// variant: 0 auto; 1 = 128x128 3 stages 8 waves, 2 = 128x128 2 stages 4 waves, 3 = 128x64 3 stages 4 waves,
// 4 = 128x64 2 stages 4 waves (two workgroups per CU), 5 = 128x128 4 stages 4 waves, 6 = 128x128 3 stages
// 4 waves, 7 = 128x64 4 stages 4 waves, 8 = 128x128 4 stages 8 waves
// small-Cin form: 9 = 128x32 2 stages 4 waves, 10 = 128x64 2 stages 4 waves, 11 = 128x128 2 stages 4 waves
hipError_t conv2d_lds_small(const ConvArgs& a, const GemmEpi& ep, int variant, hipStream_t stream) {
  if (!conv_lds_small_ok(a)) return hipErrorInvalidValue;
  if (variant == 0) variant = a.Cout <= 32 ? 9 : (a.Cout <= 64 ? 10 : 11);
  switch (variant) {
    case 9: return launch_conv_lds<2, 2, 32, true>(a, ep, stream);
    case 10: return launch_conv_lds<2, 2, 64, true>(a, ep, stream);
    case 11: return launch_conv_lds<2, 2, 128, true>(a, ep, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t conv2d_lds(const ConvArgs& a, const GemmEpi& ep, int variant, hipStream_t stream) {
  if (variant >= 9) return conv2d_lds_small(a, ep, variant, stream);
  if (!conv_lds_ok(a)) return hipErrorInvalidValue;
  if (variant == 0) {
    const int64_t M = (int64_t)a.N * a.Ho * a.Wo;
    const int64_t t128 = ((M + 127) / 128) * ((a.Cout + 127) / 128);
    if (a.Cout >= 128) variant = t128 > 256 ? 2 : 1;
    else variant = 4;
  }
  switch (variant) {
    case 1: return launch_conv_lds<3, 4, 128>(a, ep, stream);
    case 2: return launch_conv_lds<2, 2, 128>(a, ep, stream);
    case 3: return launch_conv_lds<3, 2, 64>(a, ep, stream);
    case 5: return launch_conv_lds<4, 2, 128>(a, ep, stream);
    case 6: return launch_conv_lds<3, 2, 128>(a, ep, stream);
    case 7: return launch_conv_lds<4, 2, 64>(a, ep, stream);
    case 8: return launch_conv_lds<4, 4, 128>(a, ep, stream);
    default: return launch_conv_lds<2, 2, 64>(a, ep, stream);
  }
}

}  // namespace lumen
