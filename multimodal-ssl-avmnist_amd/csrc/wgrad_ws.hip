// Conv weight gradient (bf16 NHWC, v_mfma_f32_16x16x32_bf16) for the mid-layer shapes of the
// CentralNet encoders (unimodal.py:105-221): audio conv2-4 and the image conv2, the autograd
// of nn.Conv2d w.r.t. its weight:
//     dW[co][ci][kh][kw] = sum_{n, oy, ox} dY[n][oy][ox][co] * X[n][oy+kh-p][ox+kw-p][ci]
// as a GEMM  M = co,  N = columns (tap, 16-channel tile; for 8 input channels a column tile is
// a PAIR of taps x 8 channels),  K = output pixels.
//
// Why a second wgrad kernel: wgrad_cl_kernel gives every block only a few column tiles, so the
// same strip of dY / X is staged from HBM into LDS by several blocks (PMC traffic 5.35x the
// algorithmic bytes on the 14x14 shapes), stages synchronously, and its transposed LDS reads
// conflict 2-way.  Here
//   * one block computes ALL columns of its sample chunk (the 4 waves split the columns NCW
//     ways and the pixels NPW ways; pixel-split partials are summed through LDS at the end),
//     so each dY / X byte is staged once;
//   * a block walks its strips with the next strip's 16-byte loads in registers while the
//     MFMAs run (halo lanes load a zero vector, so nothing waits on them early);
//   * both operands come from ds_read_b64_tr_b16 (4 pixels x 16 channels per read, two reads
//     per fragment); a k-group's 8 pixels are two runs of 4 chosen so that each half-wave reads
//     8 consecutive pixels, and the LDS pixel strides (16 / 48 / 80 elements for 16 / 32 / 64
//     channels) put those 8 pixels on disjoint banks.
// Deterministic: block b owns slab parts[b] = its chunk's partial dW; avd_sum_rows reduces the
// slabs in fixed order.  No atomics.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "bnapply.h"

// Measured and removed (round 4): incremental X-image pixel indices in the k-step loop (14^2:
// 168 vs 158 us), two strips' input loads in flight (two register sets: slower).

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(4))) short s4;
typedef __attribute__((ext_vector_type(2))) unsigned u2;

__device__ const u4 kZeroW = {0u, 0u, 0u, 0u};

constexpr int cdv(int a, int b) { return (a + b - 1) / b; }

// NTHR threads = WAVES waves split NMW ways over output-channel tiles, NCW ways over column
// tiles and NPW = WAVES / (NMW NCW) ways over pixels; a strip is TR output rows of NSS samples.
template <int CIN_, int COUT_, int K_, int PAD_, int H_, int W_, int TR_, int NCW_, int OCC_,
          int PF_ = 3, int NTHR_ = 256, int NMW_ = 1, int NSS_ = 1>
struct Wg {
  static constexpr int CIN = CIN_, COUT = COUT_, K = K_, PAD = PAD_, H = H_, W = W_;
  static constexpr int OCC = OCC_, PF = PF_, NTHR = NTHR_, WAVES = NTHR / 64;
  static constexpr int HO = H + 2 * PAD - K + 1, WO = W + 2 * PAD - K + 1;
  static constexpr int WO8 = (WO + 7) & ~7;                 // 8-pixel runs never cross a row
  static constexpr int TR = TR_, SPS = HO / TR, NSS = NSS_; // strip rows / strips per sample
  static constexpr int XR = TR + K - 1, XW = WO8 + K - 1;   // X strip (+ halo)
  static constexpr int MT = COUT / 16, TAPS = K * K;
  static constexpr bool PAIR = CIN == 8;
  static constexpr int NCT = PAIR ? cdv(TAPS, 2) : TAPS * (CIN / 16);   // column tiles
  static constexpr int NMW = NMW_, MTW = MT / NMW, NCW = NCW_, NPW = WAVES / (NMW * NCW);
  static constexpr int NW = cdv(NCT, NCW);
  static constexpr int DYS = COUT == 16 ? 16 : COUT + 16;   // LDS pixel strides (elements)
  static constexpr int XS = CIN <= 16 ? CIN : CIN + 16;
  static constexpr int SPIX = TR * WO8;                     // strip pixels per sample
  static constexpr int NPIX = NSS * SPIX, KST = cdv(NPIX, 32), DYP = KST * 32;
  static constexpr int DY_T = NSS * TR * WO * (COUT / 8), X_T = NSS * XR * XW * (CIN / 8);
  static constexpr int SLOTS = cdv(DY_T + X_T, NTHR);
  static constexpr int DY_ELEMS = DYP * DYS, X_ELEMS = NSS * XR * XW * XS;
  static constexpr int RED = NPW > 1 ? (NPW - 1) * NCW * NMW * MTW * NW * 64 : 0;   // f4
  static_assert(HO % TR == 0 && (NSS == 1 || SPS == 1), "strips tile the map");
  static_assert(COUT % 16 == 0 && (CIN == 8 || CIN % 16 == 0), "channel tiles");
  static_assert(WAVES % (NCW * NMW) == 0 && MT % NMW == 0, "wave split");
  static constexpr int SMEM = (DY_ELEMS + X_ELEMS) > RED * 8 ? DY_ELEMS + X_ELEMS : RED * 8;
  static_assert(SMEM * 2 <= 160 * 1024, "LDS");
};

__device__ __forceinline__ u2 tr4(const bf16* p) {
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(reinterpret_cast<uintptr_t>(p)));
  return __builtin_bit_cast(u2, v);
}
__device__ __forceinline__ bf16x8 frag8(u2 lo, u2 hi) {
  return __builtin_bit_cast(bf16x8, u4{lo.x, lo.y, hi.x, hi.y});
}
__device__ __forceinline__ f4 mma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// pixel (within a 32-pixel k-step) of k = 8 g + 4 h + q: half-waves read 8 consecutive pixels
__device__ __forceinline__ int kpix(int g, int h, int q) { return 16 * (g >> 1) + 8 * h + 4 * (g & 1) + q; }

// AP: 0 = dy is the conv-output gradient; 1 / 2 = dy is the conv output y and the staging
// applies the layer's BatchNorm backward (bnapply.h) with the pooled gradient in layout 0 / 2
template <class L, int AP = 0>
__global__ __launch_bounds__(L::NTHR, L::OCC) void wgrad_ws_kernel(const bf16* __restrict__ x,
                                                                   const bf16* __restrict__ dy,
                                                                   float* __restrict__ parts,
                                                                   int N, int chunks,
                                                                   ApplyArgs aa) {
  __shared__ __attribute__((aligned(16))) bf16 smem[L::SMEM];
  __shared__ __attribute__((aligned(16))) float ctab[AP ? APPLY_GMAX * 5 * L::COUT : 4];
  bf16* dys = smem;                       // [DYP][DYS]: pixel (s * TR + r) * WO8 + ox
  bf16* xs = smem + L::DY_ELEMS;          // [NSS][XR][XW][XS]: X[y0 - PAD + r][c - PAD]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15, q4 = r16 >> 2, p4 = r16 & 3;
  const int wm = wave % L::NMW, wc = (wave / L::NMW) % L::NCW, wp = wave / (L::NMW * L::NCW);

  // the chunk's strips (strip = TR rows of NSS samples)
  const int ngrp = N / L::NSS;
  const int g0 = (int)(((long long)blockIdx.x * ngrp) / chunks);
  const int g1 = (int)(((long long)(blockIdx.x + 1) * ngrp) / chunks);
  const int st0 = g0 * L::SPS, st1 = g1 * L::SPS;

  // this lane's column offsets in the X image (tap (kh, kw), channel quad) per column tile
  int xo[L::NW];
  bool cv[L::NW];
#pragma unroll
  for (int j = 0; j < L::NW; ++j) {
    const int ct = wc * L::NW + j;
    int tap, ch;
    if constexpr (L::PAIR) { tap = 2 * ct + (p4 >> 1); ch = 4 * (p4 & 1); }
    else { tap = ct / (L::CIN / 16); ch = 16 * (ct % (L::CIN / 16)) + 4 * p4; }
    cv[j] = ct < L::NCT;
    if (!cv[j] || tap >= L::TAPS) { tap = 0; }
    xo[j] = ((tap / L::K) * L::XW + tap % L::K) * L::XS + ch;
  }

  f4 acc[L::MTW][L::NW];
#pragma unroll
  for (int m = 0; m < L::MTW; ++m)
#pragma unroll
    for (int j = 0; j < L::NW; ++j) acc[m][j] = f4{0.f, 0.f, 0.f, 0.f};

  // dY pixels outside the map (ox >= WO, and the k-step tail) stay zero for the whole launch
  for (int i = tid; i < L::DYP * (L::DYS / 8); i += L::NTHR) {
    const int pix = i / (L::DYS / 8), ox = pix % L::WO8;
    if (ox >= L::WO || pix >= L::NPIX) *reinterpret_cast<u4*>(dys + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};
  }

  // staging slots: the strip-invariant parts of each 16-byte task's source offset (relative
  // to the strip's first dY row / first X row incl. halo), LDS offset and halo row
  int goff[L::SLOTS], loff[L::SLOTS], xrow[L::SLOTS];
#pragma unroll
  for (int i = 0; i < L::SLOTS; ++i) {
    const int task = tid + L::NTHR * i;
    goff[i] = -1; loff[i] = 0; xrow[i] = 0;
    if (task < L::DY_T) {
      constexpr int V = L::COUT / 8;
      const int q = task % V, pix = task / V;
      const int rs = pix / L::WO, ox = pix - rs * L::WO;     // rs = s * TR + r
      const int sm = rs / L::TR, r = rs - sm * L::TR;
      goff[i] = ((sm * L::HO + r) * L::WO + ox) * L::COUT + 8 * q;
      loff[i] = (rs * L::WO8 + ox) * L::DYS + 8 * q;
      xrow[i] = -1;                                  // dY: always in range
    } else if (task < L::DY_T + L::X_T) {
      constexpr int V = L::CIN / 8;
      const int t = task - L::DY_T;
      const int q = t % V, pix = t / V;
      const int rs = pix / L::XW, c = pix - rs * L::XW;      // rs = s * XR + r
      const int sm = rs / L::XR, r = rs - sm * L::XR;
      const int ix = c - L::PAD;
      loff[i] = L::DY_ELEMS + pix * L::XS + 8 * q;
      xrow[i] = r;
      if (ix >= 0 && ix < L::W) goff[i] = ((sm * L::H + r) * L::W + ix) * L::CIN + 8 * q;
    }
  }
  u4 pre[L::SLOTS];
  auto load_into = [&](u4 (&dst)[L::SLOTS], int st) {
    if constexpr (AP) return;
    const int sg = st / L::SPS, y0 = (st - sg * L::SPS) * L::TR;
    const int n = sg * L::NSS;
    const bf16* bdy = dy + ((size_t)n * L::HO + y0) * L::WO * L::COUT;
    const bf16* bx = x + ((long long)n * L::H + y0 - L::PAD) * L::W * L::CIN;   // row y0 - PAD
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) {
      const u4* src = &kZeroW;
      if (xrow[i] < 0) {
        if (goff[i] >= 0) src = reinterpret_cast<const u4*>(bdy + goff[i]);
      } else if (goff[i] >= 0 && (unsigned)(y0 - L::PAD + xrow[i]) < (unsigned)L::H) {
        src = reinterpret_cast<const u4*>(bx + goff[i]);
      }
      dst[i] = ldg16(src);
    }
  };
  auto load_strip = [&](int st) { load_into(pre, st); };
  auto store_from = [&](const u4 (&src)[L::SLOTS]) {
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i)
      if (tid + L::NTHR * i < L::DY_T + L::X_T) *reinterpret_cast<u4*>(smem + loff[i]) = src[i];
  };
  auto store_strip = [&]() { store_from(pre); };

  // AP: dY comes from windows of y (2x2 x 8 channels + the pooled gradient -> 4 dY vectors);
  // X keeps its 16-byte tasks in their own slots
  constexpr int HOP = L::HO / 2, WOP = L::WO / 2;
  constexpr int WT = AP ? L::NSS * (L::TR / 2) * WOP * (L::COUT / 8) : 0;
  constexpr int WSL = AP ? cdv(WT, L::NTHR) : 1;
  constexpr int XSL = AP ? cdv(L::X_T, L::NTHR) : 1;
  int wgo[WSL], wgg[WSL], wlo[WSL];
  int xgo[XSL], xlo[XSL], xrw[XSL];
  WinIn wpre[WSL];
  u4 xpre[XSL];
  if constexpr (AP) {
    static_assert(L::TR % 2 == 0 && L::HO % 2 == 0 && L::WO % 2 == 0, "windows");
    apply_load_ctab<L::COUT>(ctab, aa, tid, L::NTHR);
#pragma unroll
    for (int i = 0; i < WSL; ++i) {
      const int task = tid + L::NTHR * i;
      constexpr int V = L::COUT / 8;
      const int q = task % V, w = task / V;
      const int wc2 = w % WOP, t = w / WOP;
      const int wr = t % (L::TR / 2), sm = t / (L::TR / 2);
      wgo[i] = task < WT ? ((sm * L::HO + 2 * wr) * L::WO + 2 * wc2) * L::COUT + 8 * q : -1;
      wlo[i] = ((sm * L::TR + 2 * wr) * L::WO8 + 2 * wc2) * L::DYS + 8 * q;
      wgg[i] = AP == 1 ? ((sm * HOP + wr) * WOP + wc2) * L::COUT + 8 * q
                       : (sm * L::COUT + 8 * q) * HOP * WOP + wr * WOP + wc2;
    }
#pragma unroll
    for (int i = 0; i < XSL; ++i) {
      const int t = tid + L::NTHR * i;
      constexpr int V = L::CIN / 8;
      const int q = t % V, pix = t / V;
      const int rs = pix / L::XW, c = pix - rs * L::XW;
      const int sm = rs / L::XR, r = rs - sm * L::XR;
      const int ix = c - L::PAD;
      xlo[i] = L::DY_ELEMS + pix * L::XS + 8 * q;
      xrw[i] = r;
      xgo[i] = (t < L::X_T && ix >= 0 && ix < L::W) ? ((sm * L::H + r) * L::W + ix) * L::CIN + 8 * q : -1;
    }
  }
  auto load_strip_ap = [&](int st) {
    const int sg = st / L::SPS, y0 = (st - sg * L::SPS) * L::TR;
    const int n = sg * L::NSS;
    const bf16* by = dy + ((size_t)n * L::HO + y0) * L::WO * L::COUT;
    const bf16* bx = x + ((long long)n * L::H + y0 - L::PAD) * L::W * L::CIN;
#pragma unroll
    for (int i = 0; i < WSL; ++i) {
      const bool ok = wgo[i] >= 0;
      const bf16* p = by + (ok ? wgo[i] : 0);
      wpre[i].y[0] = ldg16(ok ? (const void*)(p) : &kZeroW);
      wpre[i].y[1] = ldg16(ok ? (const void*)(p + L::COUT) : &kZeroW);
      wpre[i].y[2] = ldg16(ok ? (const void*)(p + L::WO * L::COUT) : &kZeroW);
      wpre[i].y[3] = ldg16(ok ? (const void*)(p + (L::WO + 1) * L::COUT) : &kZeroW);
      if constexpr (AP == 1) {
        const bf16* gb = reinterpret_cast<const bf16*>(aa.gout) + ((size_t)n * HOP + y0 / 2) * WOP * L::COUT;
        wpre[i].g0 = ldg16(ok ? (const void*)(gb + wgg[i]) : &kZeroW);
      } else {
        const float* gp = reinterpret_cast<const float*>(aa.gout) + (size_t)n * L::COUT * HOP * WOP +
                          (size_t)(y0 / 2) * WOP + (ok ? wgg[i] : 0);
        float gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) gv[e] = ok ? gp[(size_t)e * HOP * WOP] : 0.f;
        wpre[i].g0 = u4{__float_as_uint(gv[0]), __float_as_uint(gv[1]), __float_as_uint(gv[2]), __float_as_uint(gv[3])};
        wpre[i].g1 = u4{__float_as_uint(gv[4]), __float_as_uint(gv[5]), __float_as_uint(gv[6]), __float_as_uint(gv[7])};
      }
    }
#pragma unroll
    for (int i = 0; i < XSL; ++i) {
      const bool ok = xgo[i] >= 0 && (unsigned)(y0 - L::PAD + xrw[i]) < (unsigned)L::H;
      xpre[i] = ldg16(ok ? (const void*)(bx + xgo[i]) : &kZeroW);
    }
  };
  auto store_strip_ap = [&](int st) {
    const int n = (st / L::SPS) * L::NSS;
    const float* ct = ctab + (n / aa.B) * 5 * L::COUT;
#pragma unroll
    for (int i = 0; i < WSL; ++i) {
      if (wgo[i] < 0) continue;
      u4 o[4];
      apply_window<AP == 1 ? 0 : 2, L::COUT>(wpre[i], ct + 8 * ((tid + L::NTHR * i) % (L::COUT / 8)), o);
      *reinterpret_cast<u4*>(smem + wlo[i]) = o[0];
      *reinterpret_cast<u4*>(smem + wlo[i] + L::DYS) = o[1];
      *reinterpret_cast<u4*>(smem + wlo[i] + L::WO8 * L::DYS) = o[2];
      *reinterpret_cast<u4*>(smem + wlo[i] + (L::WO8 + 1) * L::DYS) = o[3];
    }
#pragma unroll
    for (int i = 0; i < XSL; ++i)
      if (tid + L::NTHR * i < L::X_T) *reinterpret_cast<u4*>(smem + xlo[i]) = xpre[i];
  };

  auto strip_body = [&]() {
    for (int ks = wp; ks < L::KST; ks += L::NPW) {
      const int P0 = 32 * ks;
      int xb[2];
      bf16x8 a[L::MTW];
#pragma unroll
      for (int m = 0; m < L::MTW; ++m) {
        const int co = 16 * (wm * L::MTW + m) + 4 * p4;
        const bf16* pa0 = dys + (P0 + kpix(g, 0, q4)) * L::DYS + co;
        const bf16* pa1 = dys + (P0 + kpix(g, 1, q4)) * L::DYS + co;
        a[m] = frag8(tr4(pa0), tr4(pa1));
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int P = min(P0 + kpix(g, h, q4), L::NPIX - 1);   // tail pixels: dY is 0 there
        const int sm = P / L::SPIX, rem = P - sm * L::SPIX;
        const int r = rem / L::WO8, ox = rem - r * L::WO8;
        xb[h] = ((sm * L::XR + r) * L::XW + ox) * L::XS;
      }
      // B fragments PF columns ahead of their MFMAs
      constexpr int PF = L::PF;
      u2 bq[PF + 1][2];
#pragma unroll
      for (int j = 0; j < PF && j < L::NW; ++j) {
        bq[j][0] = tr4(xs + xb[0] + xo[j]);
        bq[j][1] = tr4(xs + xb[1] + xo[j]);
      }
#pragma unroll
      for (int j = 0; j < L::NW; ++j) {
        if (j + PF < L::NW) {
          bq[(j + PF) % (PF + 1)][0] = tr4(xs + xb[0] + xo[j + PF]);
          bq[(j + PF) % (PF + 1)][1] = tr4(xs + xb[1] + xo[j + PF]);
        }
        const bf16x8 b = frag8(bq[j % (PF + 1)][0], bq[j % (PF + 1)][1]);
#pragma unroll
        for (int m = 0; m < L::MTW; ++m) acc[m][j] = mma(a[m], b, acc[m][j]);
      }
      // pin the interleave (hipcc otherwise pulls each fragment's reads down to its MFMAs and
      // waits lgkmcnt(0) every few MFMAs): A + PF columns of reads, then MTW MFMAs per column
      // with the reads of column j + PF between them
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * L::MTW + 2 * (PF < L::NW ? PF : L::NW), 0);
#pragma unroll
      for (int j = 0; j < L::NW; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, L::MTW, 0);
        if (j + PF < L::NW) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
    }
  };

  if (st0 < st1) { if constexpr (AP) load_strip_ap(st0); else load_strip(st0); }
  for (int st = st0; st < st1; ++st) {
    __syncthreads();
    if constexpr (AP) store_strip_ap(st); else store_strip();
    __syncthreads();
    if (st + 1 < st1) { if constexpr (AP) load_strip_ap(st + 1); else load_strip(st + 1); }
    strip_body();
  }

  // pixel-split partials -> wave wp = 0 (fixed order), then the slab write
  if constexpr (L::NPW > 1) {
    f4* red = reinterpret_cast<f4*>(smem);
    const int slot = wm * L::NCW + wc;
    __syncthreads();
    if (wp > 0) {
#pragma unroll
      for (int m = 0; m < L::MTW; ++m)
#pragma unroll
        for (int j = 0; j < L::NW; ++j)
          red[((((wp - 1) * L::NCW * L::NMW + slot) * L::MTW + m) * L::NW + j) * 64 + lane] = acc[m][j];
    }
    __syncthreads();
    if (wp == 0) {
#pragma unroll
      for (int w = 1; w < L::NPW; ++w)
#pragma unroll
        for (int m = 0; m < L::MTW; ++m)
#pragma unroll
          for (int j = 0; j < L::NW; ++j)
            acc[m][j] += red[((((w - 1) * L::NCW * L::NMW + slot) * L::MTW + m) * L::NW + j) * 64 + lane];
    }
  }
  // slab write [co][ci][tap], staged through LDS RC output-channel tiles at a time so the HBM
  // stores are contiguous float4s (written straight from the MFMA layout they were 4-byte
  // scatters at a 25-float stride: ~110 us of a 270 us launch on the 14x14 shapes)
  constexpr int PER_CO = L::CIN * L::TAPS;
  constexpr int RC0 = (L::SMEM * 2) / (16 * PER_CO * 4);
  constexpr int RC = RC0 < L::MT ? RC0 : L::MT;
  static_assert(RC >= 1, "one output-channel tile must fit in LDS");
  float* tb = reinterpret_cast<float*>(smem);
  float* out = parts + (size_t)blockIdx.x * L::COUT * PER_CO;
  for (int r0 = 0; r0 < L::MT; r0 += RC) {
    __syncthreads();
    if (wp == 0) {
#pragma unroll
      for (int m = 0; m < L::MTW; ++m) {
        const int mt = wm * L::MTW + m;
        if (mt < r0 || mt >= r0 + RC) continue;
#pragma unroll
        for (int j = 0; j < L::NW; ++j) {
          if (!cv[j]) continue;
          const int ct = wc * L::NW + j;
          int tap, ci;
          if constexpr (L::PAIR) { tap = 2 * ct + (r16 >> 3); ci = r16 & 7; }
          else { tap = ct / (L::CIN / 16); ci = 16 * (ct % (L::CIN / 16)) + r16; }
          if (tap >= L::TAPS) continue;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            tb[(16 * (mt - r0) + 4 * g + i) * PER_CO + ci * L::TAPS + tap] = acc[m][j][i];
        }
      }
    }
    __syncthreads();
    const int n = min(RC, L::MT - r0) * 16 * PER_CO;     // a multiple of 4 floats
    float4* o4 = reinterpret_cast<float4*>(out + (size_t)r0 * 16 * PER_CO);
    const float4* t4 = reinterpret_cast<const float4*>(tb);
    for (int e = tid; e < n / 4; e += L::NTHR) o4[e] = t4[e];
  }
}

//        CIN COUT K PAD  H   W  TR NCW OCC PF NTHR NMW NSS
typedef Wg<8, 16, 5, 2, 56, 56, 8, 1, 2> WgA2;      // audio conv2
typedef Wg<16, 32, 5, 2, 28, 28, 14, 4, 2> WgA3;    // audio conv3
typedef Wg<32, 64, 5, 2, 14, 14, 14, 2, 1, 3, 256, 2> WgA4;   // audio conv4: 2x2 waves over (M, columns); 170 vs 161 us alone, step 5.279 vs 5.317 ms
typedef Wg<32, 64, 5, 0, 14, 14, 10, 4, 1> WgI2;    // image conv2


// avd_options.generic_conv: every bf16 weight gradient on the generic wgrad_cl kernel
bool wg_disabled() { return g_opts.generic_conv != 0; }

int wg_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

template <class L>
bool wg_is(int Cin, int H, int W, int Cout, int K, int pad) {
  return Cin == L::CIN && Cout == L::COUT && K == L::K && pad == L::PAD && H == L::H && W == L::W;
}

}  // namespace

// Slabs (= blocks) of the weights-stationary wgrad for (Cout, Cin, K); 0 if not served.  One
// block per CU per occupancy slot, so the grid is a single wave of persistent blocks.
int avd_wg_chunks(int N, int Cout, int Cin, int K) {
  if (wg_disabled()) return 0;
  int occ = 0;
  if (Cin == 8 && Cout == 16 && K == 5) occ = WgA2::OCC;
  else if (Cin == 16 && Cout == 32 && K == 5) occ = WgA3::OCC;
  else if (Cin == 32 && Cout == 64 && K == 5) occ = WgA4::OCC;
  else return 0;
  // (a grid on a fraction of the CUs, leaving CUs to the input-gradient chain beside it, measured
  // within noise in round 4)
  return std::max(1, grid_cap(std::min(N, wg_cus() * occ)));
}

// 1 = launched, 0 = not served, < 0 = error.  parts must hold avd_wg_chunks(...) slabs.
int avd_wg_conv_wgrad(const void* x, const void* dy, int dt, float* parts, int N, int Cin, int H,
                      int W, int Cout, int K, int pad, hipStream_t st) {
  if (dt != AVD_BF16 || wg_disabled()) return 0;
  const int chunks = avd_wg_chunks(N, Cout, Cin, K);
  if (!chunks) return 0;
  const ApplyArgs aa{};
#define AVD_WG(LL)                                                                              \
  if (wg_is<LL>(Cin, H, W, Cout, K, pad)) {                                                    \
    if (N % LL::NSS) return 0;                                                                 \
    wgrad_ws_kernel<LL, 0><<<chunks, LL::NTHR, 0, st>>>((const bf16*)x, (const bf16*)dy, parts, N, chunks, aa); \
    AVD_CHECK_LAUNCH();                                                                         \
    return 1;                                                                                   \
  }
  AVD_WG(WgA2) AVD_WG(WgA3) AVD_WG(WgA4) AVD_WG(WgI2)
#undef AVD_WG
  return 0;
}
