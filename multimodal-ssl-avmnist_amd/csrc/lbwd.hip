// One fused launch for the whole backward of the audio conv2 layer (56x56, 8 -> 16, 5x5 pad 2;
// CentralUnimodalAudio, unimodal.py:185-221 -> nn.Conv2d -> BatchNorm2d -> ReLU -> MaxPool2d):
//
//   dY = BN-backward apply (bnapply.h) of y and the pooled gradient    [N, 56, 56, 16]
//   dX = conv_transpose(dY, W)            (the input gradient)         [N, 56, 56, 8]
//   dW = sum_{n, p} dY[n, p] (x) X[n, p + tap - 2]   (weight gradient) [16][8][25]
//
// from ONE staged tile of dY.  Before, the step ran the apply (y + pooled gradient -> dY in HBM,
// bn_cl.hip), then the input gradient (conv_ws.hip) and the weight gradient (wgrad_ws.hip) side
// by side on two streams, each streaming the 719 MB dY at config-2 size: 3.8 GB of HBM traffic
// for the layer and two latency-bound kernels inflating each other.  Here a
// persistent block walks TH-row tiles of its samples; per tile it
//   * stages the dY tile with its 2-row / 2-column halo, formed in registers from y and the
//     pooled gradient (AP = 1; one 2x2 window x 8 channels per task, bit-identical to
//     bwd_apply_cl_kernel) or loaded from a dY tensor (AP = 0), and the X tile with its halo;
//   * runs the input gradient on it exactly as conv_ws_kernel's DgrA2 does (weights resident in
//     VGPRs, B fragments = one ds_read_b128 of the (tap, channel) k-group per pixel, same k
//     order: bit-identical dX);
//   * accumulates dW exactly as wgrad_ws_kernel's WgA2 does (M = dY channels, N = 13 column tiles
//     of (tap pair, 8 X channels), K = the tile's pixels, both operands by ds_read_b64_tr_b16),
//     in registers across all of the block's tiles; the four waves split the pixels and are
//     summed through LDS at the end; one deterministic f32 slab per block (avd_sum_rows).
// HBM per launch: y + pooled gradient + X read once, dX written once (1.6 GB at N = 7168), no dY.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "bnapply.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(4))) short s4;
typedef __attribute__((ext_vector_type(2))) unsigned u2;

__device__ const u4 kZeroL = {0u, 0u, 0u, 0u};

constexpr int cdv(int a, int b) { return (a + b - 1) / b; }

template <int V> using IC = std::integral_constant<int, V>;
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<I + 1, N>(f);
  }
}

template <int TH_, int OCC_, int PFD_ = 6, int GB_ = 1, int NCW_ = 1, int RP_ = 0>
struct Lb {
  static constexpr int CIN = 8, COUT = 16, K = 5, PAD = 2, H = 56, W = 56;   // the forward conv
  static constexpr int TH = TH_, TPS = H / TH, OCC = OCC_, PFD = PFD_, GB = GB_;
  static constexpr int ITH = TH + K - 1, ITW = W + K - 1;        // staged rows / columns (halo)
  // dY tile [ITH][RS][PS]: DgrA2's conflict-free image (pixel stride 16 channels, rows padded
  // by 4 pixels); X tile [ITH][XW][XS]: WgA2's
  static constexpr int PS = COUT, RS = ITW + 4, XW = ITW, XS = CIN;
  static constexpr int DY_ELEMS = ITH * RS * PS, X_ELEMS = ITH * XW * XS;
  // input gradient: M = dX channels (8 rows of a 16-row tile), N = 16-pixel groups,
  // K = (tap, dY channel) in conv_ws's order, 13 k-steps of 32
  static constexpr int KK = K * K, KPAD = cdv(KK * COUT, 32) * 32;
  // RP (row pairs): one MFMA row tile = dX channels of TWO output rows (m < 8: row y, m >= 8: row
  // y + 1) over the 6 x 5 dY taps both rows need -- 15 k-steps per 16 pixels of a row pair
  // instead of 2 x 13, and no padding rows in the D tile (the layer is LDS-read bound: every
  // k-step reads a 16-byte im2col fragment per lane)
  static constexpr int RP = RP_, KTAPS = RP ? (K + 1) * K : KK;
  static constexpr int KS = cdv(KTAPS * COUT, 32);
  static constexpr int PIX = TH * W, NG = (RP ? PIX / 2 : PIX) / 16, GW = cdv(NG, 4);
  // weight gradient: 13 column tiles (tap pair x 8 channels), K = PIX pixels in 32-pixel steps;
  // the 4 waves split NCW ways over column tiles (NW per wave) and NPW = 4 / NCW over k-steps
  static constexpr int NCT = cdv(KK, 2), WKS = PIX / 32;
  static constexpr int NCW = NCW_, NW = cdv(NCT, NCW), NPW = 4 / NCW;
  static constexpr int WT = (ITH / 2) * (ITW / 2) * (COUT / 8);   // AP: window x channel-half tasks
  static constexpr int DT = ITH * ITW * (COUT / 8);               // AP = 0: 16-byte dY tasks
  static constexpr int XT = ITH * ITW * (CIN / 8);                // 16-byte X tasks
  static constexpr int RED = (NPW - 1) * NCW * NW * 64;           // f4 slots: pixel partials
  // two tile images (double buffer): tile i + 1 is staged while tile i's MFMAs run, one barrier
  // per tile (the apply's VALU work beside the MFMAs instead of between two barriers)
  static constexpr int BUF = DY_ELEMS + X_ELEMS;
  static constexpr int SMEM = 2 * BUF > RED * 8 ? 2 * BUF : RED * 8;
  static_assert(H % TH == 0 && TH % 2 == 0 && PIX % 32 == 0 && PIX % 16 == 0, "tiles");
  static_assert(SMEM * 2 <= 76 * 1024, "LDS (two blocks per CU: 160 KB)");
  static_assert(4 % NCW == 0, "wave split");
  static_assert(!RP || (KTAPS * COUT) % 32 == 0, "row-pair k-steps");
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
// bnapply.h's apply_window (gout layout 0), one channel pair at a time: the same IEEE operations
// in the same order (bit-identical dY), but only one pair's coefficients and values live at
// once -- the full-width version keeps ~80 temporaries across the window and spills here
__device__ __forceinline__ void apply_window_lean(const WinIn& in, const float* ct, int C, u4 (&out)[4]) {
  const unsigned yw[4][4] = {{in.y[0].x, in.y[0].y, in.y[0].z, in.y[0].w},
                             {in.y[1].x, in.y[1].y, in.y[1].z, in.y[1].w},
                             {in.y[2].x, in.y[2].y, in.y[2].z, in.y[2].w},
                             {in.y[3].x, in.y[3].y, in.y[3].z, in.y[3].w}};
  const unsigned gw[4] = {in.g0.x, in.g0.y, in.g0.z, in.g0.w};
  unsigned ow[4][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float2 sc = *reinterpret_cast<const float2*>(ct + 2 * e);
    const float2 sf = *reinterpret_cast<const float2*>(ct + C + 2 * e);
    const float2 k1 = *reinterpret_cast<const float2*>(ct + 2 * C + 2 * e);
    const float2 kx = *reinterpret_cast<const float2*>(ct + 3 * C + 2 * e);
    const float2 k0 = *reinterpret_cast<const float2*>(ct + 4 * C + 2 * e);
    float d[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float s_ = h ? sc.y : sc.x, f_ = h ? sf.y : sf.x;
      float yv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) yv[k] = h ? __uint_as_float(yw[k][e] & 0xffff0000u) : __uint_as_float(yw[k][e] << 16);
      float best = fmaxf(fmaf(yv[0], s_, f_), 0.f);
      int am = 0;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float r = fmaxf(fmaf(yv[k], s_, f_), 0.f);
        if (r > best) { best = r; am = k; }
      }
      const float gg = h ? __uint_as_float(gw[e] & 0xffff0000u) : __uint_as_float(gw[e] << 16);
      const float dz = best > 0.f ? gg : 0.f;
      const float a1 = h ? k1.y : k1.x, ax = h ? kx.y : kx.x, a0 = h ? k0.y : k0.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k][h] = fmaf(a1, am == k ? dz : 0.f, fmaf(ax, yv[k], a0));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) ow[k][e] = pack_bf16x2(d[k][0], d[k][1]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = u4{ow[k][0], ow[k][1], ow[k][2], ow[k][3]};
}

// pixel (within a 32-pixel k-step) of k = 8 g + 4 h + q (wgrad_ws.hip's kpix)
__device__ __forceinline__ int kpix(int g, int h, int q) { return 16 * (g >> 1) + 8 * h + 4 * (g & 1) + q; }

// dgrad k-groups (conv_ws.hip koff with CIN = 16): k-group 4 ks + g is tap (4 ks + g) / 2,
// channel chunk 8 (g & 1); padded k-groups (tap >= 25) read tap 0 against zero weights
template <class L>
constexpr int tapoff(int tap) { return ((tap / L::K) * L::RS + tap % L::K) * L::PS; }

template <class L, int AP>
__global__ __launch_bounds__(256, L::OCC) void lbwd_kernel(const bf16* __restrict__ ysrc,
                                                          const bf16* __restrict__ x,
                                                          const bf16* __restrict__ wk,
                                                          bf16* __restrict__ dx,
                                                          float* __restrict__ parts, int ntiles,
                                                          ApplyArgs aa) {
  __shared__ __attribute__((aligned(16))) bf16 smem[L::SMEM];
  __shared__ __attribute__((aligned(16))) float ctab[AP ? APPLY_GMAX * 5 * L::COUT : 4];
  // dY tile (row ty0 - PAD + r, column c - PAD) then the X tile (same origin), per buffer
  bf16* dys = smem;
  bf16* xs = smem + L::DY_ELEMS;
  auto set_buf = [&](int b) {
    dys = smem + b * L::BUF;
    xs = dys + L::DY_ELEMS;
  };
  const int tid = threadIdx.x, wp = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15, q4 = r16 >> 2, p4 = r16 & 3;
  const int wc = wp / L::NPW, wq = wp % L::NPW;     // weight gradient: column group, pixel part

  // ---- input-gradient weights (flipped, [16 rows][KPAD], rows 8-15 zero), resident
  bf16x8 a[L::KS];
  if constexpr (L::RP) {
    // row m = (output row m >> 3, dX channel m & 7); k-group 4 j + g = staged-row offset /
    // filter column t = 2 j + (g >> 1) of the 6 x 5 window, dY channel half 8 (g & 1): the
    // filter row is t / 5 - (m >> 3) -- outside [0, 5) the weight is 0
#pragma unroll
    for (int j = 0; j < L::KS; ++j) {
      const int t = 2 * j + (g >> 1), kh = t / L::K - (r16 >> 3), kw = t % L::K;
      constexpr bf16x8 z = {};
      a[j] = (kh >= 0 && kh < L::K)
                 ? *reinterpret_cast<const bf16x8*>(wk + (size_t)(r16 & 7) * L::KPAD + (kh * L::K + kw) * L::COUT + 8 * (g & 1))
                 : z;
    }
  } else {
#pragma unroll
    for (int j = 0; j < L::KS; ++j) a[j] = *reinterpret_cast<const bf16x8*>(wk + (size_t)r16 * L::KPAD + 32 * j + 8 * g);
  }
  // k-group (ks, g) = taps 2 ks (g < 2) / 2 ks + 1 (g >= 2), channel half g & 1: the k-step part
  // of its offset is a compile-time immediate (tapoff), the lane part one of three registers
  const int ln_a = (g >> 1) * L::PS + 8 * (g & 1);                  // tap + 1 on the same row
  const int ln_b = (g >> 1) * (L::RS - (L::K - 1)) * L::PS + 8 * (g & 1);   // next filter row
  const int ln_c = (g >> 1) ? -tapoff<L>(L::KK - 1) : 8 * (g & 1);  // past the last tap: tap 0

  // ---- weight-gradient column offsets in the X tile (PAIR layout of wgrad_ws.hip)
  int xo[L::NW];
#pragma unroll
  for (int j = 0; j < L::NW; ++j) {
    int tap = 2 * (wc * L::NW + j) + (p4 >> 1);
    const int ch = 4 * (p4 & 1);
    if (tap >= L::KK) tap = 0;
    xo[j] = ((tap / L::K) * L::XW + tap % L::K) * L::XS + ch;
  }
  f4 wacc[L::NW];
#pragma unroll
  for (int j = 0; j < L::NW; ++j) wacc[j] = f4{0.f, 0.f, 0.f, 0.f};

  // ---- contiguous tile range of this block (tile = TH rows of one sample)
  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);

  // ---- staging slots: dY (AP: 2x2 windows of y + pooled gradient; else 16-byte dY tasks), X
  constexpr int HP = L::H / 2, WP = L::W / 2;
  constexpr int YT = AP ? L::WT : L::DT;
  constexpr int YSL = cdv(YT, 256), XSL = cdv(L::XT, 256);
  int ygo[YSL], ylo[YSL], yrow[YSL], ygg[YSL];
  int xgo[XSL], xlo[XSL], xrow[XSL];
#pragma unroll
  for (int i = 0; i < YSL; ++i) {
    const int task = tid + 256 * i;
    const int q = task & 1, w = task >> 1;             // COUT / 8 = 2 channel halves
    if constexpr (AP) {
      const int wc2 = w % (L::ITW / 2), wr = w / (L::ITW / 2);
      const int r = 2 * wr, c = 2 * wc2, ix = c - L::PAD;
      yrow[i] = r;
      ylo[i] = (r * L::RS + c) * L::PS + 8 * q;
      ygo[i] = (task < YT && ix >= 0 && ix < L::W) ? (r * L::W + ix) * L::COUT + 8 * q : -1;
      ygg[i] = (wr * WP + ix / 2) * L::COUT + 8 * q;
    } else {
      const int c = w % L::ITW, r = w / L::ITW, ix = c - L::PAD;
      yrow[i] = r;
      ylo[i] = (r * L::RS + c) * L::PS + 8 * q;
      ygo[i] = (task < YT && ix >= 0 && ix < L::W) ? (r * L::W + ix) * L::COUT + 8 * q : -1;
      ygg[i] = 0;
    }
  }
#pragma unroll
  for (int i = 0; i < XSL; ++i) {
    const int task = tid + 256 * i;
    const int c = task % L::ITW, r = task / L::ITW, ix = c - L::PAD;
    xrow[i] = r;
    xlo[i] = (r * L::XW + c) * L::XS;
    xgo[i] = (task < L::XT && ix >= 0 && ix < L::W) ? (r * L::W + ix) * L::CIN : -1;
  }
  if constexpr (AP) apply_load_ctab<L::COUT>(ctab, aa, tid, 256);

  WinIn wpre[AP ? YSL : 1];
  u4 ypre[AP ? 1 : YSL];
  u4 xpre[XSL];
  // cont: the block's previous tile is the rows just above this one in the same sample, so the
  // first 2 * PAD staged rows (dY and X) are copied from that tile's last rows instead of loaded
  // and recomputed (a third of the BN-backward apply and of the y / x loads)
  constexpr int RR = 2 * L::PAD;
  auto load_tile = [&](int ti, bool cont) {
    const int n = ti / L::TPS, ty0 = (ti - n * L::TPS) * L::TH;
    const long long row0 = (long long)n * L::H + ty0 - L::PAD;     // first staged row
    const bf16* by = ysrc + row0 * L::W * L::COUT;
    const bf16* bx = x + row0 * L::W * L::CIN;
#pragma unroll
    for (int i = 0; i < YSL; ++i) {
      const bool ok = ygo[i] >= 0 && (unsigned)(ty0 - L::PAD + yrow[i]) < (unsigned)L::H &&
                      !(cont && yrow[i] < RR);
      const bf16* p = by + (ok ? ygo[i] : 0);
      if constexpr (AP) {
        wpre[i].y[0] = ldg16(ok ? (const void*)(p) : &kZeroL);
        wpre[i].y[1] = ldg16(ok ? (const void*)(p + L::COUT) : &kZeroL);
        wpre[i].y[2] = ldg16(ok ? (const void*)(p + L::W * L::COUT) : &kZeroL);
        wpre[i].y[3] = ldg16(ok ? (const void*)(p + (L::W + 1) * L::COUT) : &kZeroL);
        const bf16* gb = reinterpret_cast<const bf16*>(aa.gout) + ((long long)n * HP + (ty0 - L::PAD) / 2) * WP * L::COUT;
        wpre[i].g0 = ldg16(ok ? (const void*)(gb + ygg[i]) : &kZeroL);
      } else {
        ypre[i] = ldg16(ok ? (const void*)p : &kZeroL);
      }
    }
#pragma unroll
    for (int i = 0; i < XSL; ++i) {
      const bool ok = xgo[i] >= 0 && (unsigned)(ty0 - L::PAD + xrow[i]) < (unsigned)L::H &&
                      !(cont && xrow[i] < RR);
      xpre[i] = ldg16(ok ? (const void*)(bx + xgo[i]) : &kZeroL);
    }
  };
  auto store_tile = [&](int ti, bool cont, const bf16* pdys, const bf16* pxs) {
    const int n = ti / L::TPS, ty0 = (ti - n * L::TPS) * L::TH;
    if (cont) {
      // rows 0 .. RR-1 of this tile = rows TH .. TH+RR-1 of the previous one (other buffer)
      constexpr int DQ = RR * L::RS * L::PS / 8, XQ = RR * L::XW * L::XS / 8;   // 16-byte chunks
      const u4* sd = reinterpret_cast<const u4*>(pdys + L::TH * L::RS * L::PS);
      u4* dd = reinterpret_cast<u4*>(dys);
      for (int c = tid; c < DQ; c += 256) dd[c] = sd[c];
      const u4* sx = reinterpret_cast<const u4*>(pxs + L::TH * L::XW * L::XS);
      u4* dxs = reinterpret_cast<u4*>(xs);
      for (int c = tid; c < XQ; c += 256) dxs[c] = sx[c];
    }
#pragma unroll
    for (int i = 0; i < YSL; ++i) {
      const int task = tid + 256 * i;
      if (task >= YT || (cont && yrow[i] < RR)) continue;
      if constexpr (AP) {
        u4 o[4] = {u4{0u, 0u, 0u, 0u}, u4{0u, 0u, 0u, 0u}, u4{0u, 0u, 0u, 0u}, u4{0u, 0u, 0u, 0u}};
        if (ygo[i] >= 0 && (unsigned)(ty0 - L::PAD + yrow[i]) < (unsigned)L::H)
          apply_window_lean(wpre[i], ctab + (n / aa.B) * 5 * L::COUT + 8 * (task & 1), L::COUT, o);
        *reinterpret_cast<u4*>(dys + ylo[i]) = o[0];
        *reinterpret_cast<u4*>(dys + ylo[i] + L::PS) = o[1];
        *reinterpret_cast<u4*>(dys + ylo[i] + L::RS * L::PS) = o[2];
        *reinterpret_cast<u4*>(dys + ylo[i] + (L::RS + 1) * L::PS) = o[3];
      } else {
        *reinterpret_cast<u4*>(dys + ylo[i]) = ypre[i];
      }
    }
#pragma unroll
    for (int i = 0; i < XSL; ++i)
      if (tid + 256 * i < L::XT && !(cont && xrow[i] < RR))
        *reinterpret_cast<u4*>(xs + xlo[i]) = xpre[i];
  };

  // ---- input gradient of one tile (conv_ws_kernel<DgrA2, false>'s tile body)
  auto dgrad_tile = [&](int ti) {
    const int n = ti / L::TPS, ty0 = (ti - n * L::TPS) * L::TH;
#pragma unroll 1
    for (int i0 = 0; i0 < L::GW; i0 += L::GB) {
      int base[L::GB], opix[L::GB];
      bool gv[L::GB];
#pragma unroll
      for (int b = 0; b < L::GB; ++b) {
        const int grp = wp + 4 * (i0 + b);
        const int p = grp * 16 + r16;
        gv[b] = i0 + b < L::GW && grp < L::NG;
        int ry = p / L::W;
        const int rx = p - ry * L::W;
        if constexpr (L::RP) ry *= 2;                     // p enumerates (row pair, column)
        base[b] = gv[b] ? (ry * L::RS + rx) * L::PS : 0;
        opix[b] = ((n * L::H) + ty0 + ry + (L::RP ? (g >> 1) : 0)) * L::W + rx;
      }
      f4 acc[L::GB];
#pragma unroll
      for (int b = 0; b < L::GB; ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};
      constexpr int PF = L::PFD;
      bf16x8 bq[PF + 1][L::GB];
      // k-step j: taps 2j, 2j + 1 -- the lane register by whether 2j + 1 starts a filter row
      // or lies past the last tap (compile-time per j)
      auto ld = [&](bf16x8 (&dst)[L::GB], auto jc) {
        constexpr int J = decltype(jc)::value;
        constexpr int t0 = 2 * J;
        const int ln = (!L::RP && t0 + 1 >= L::KK) ? ln_c : ((t0 % L::K) == L::K - 1 ? ln_b : ln_a);
#pragma unroll
        for (int b = 0; b < L::GB; ++b)
          dst[b] = *reinterpret_cast<const bf16x8*>(dys + base[b] + ln + tapoff<L>(t0));
      };
      static_for<0, (PF < L::KS ? PF : L::KS)>([&](auto jc) { ld(bq[decltype(jc)::value], jc); });
      // the fragment of k-step j + PF is read before the MFMA of k-step j, and scheduling
      // barriers keep it there: without them (round-6 ISA) the scheduler sank every read to its
      // MFMA, the ring collapsed to one register and each k-step waited out a whole LDS latency
      static_for<0, L::KS>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j + PF < L::KS) ld(bq[(j + PF) % (PF + 1)], IC<j + PF>{});
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int b = 0; b < L::GB; ++b) acc[b] = mma(a[j], bq[j % (PF + 1)][b], acc[b]);
        __builtin_amdgcn_sched_barrier(0);
      });
      // rows 4g..4g+3 of the D tile: dX channels 4 (g & 1).. of row y (g < 2) or, with RP, of
      // row y + 1 (g >= 2); without RP rows 8-15 are padding
      if (L::RP || g < 2) {
#pragma unroll
        for (int b = 0; b < L::GB; ++b) {
          if (!gv[b]) continue;
          const uint32_t lo = pack_bf16x2(acc[b][0], acc[b][1]), hi = pack_bf16x2(acc[b][2], acc[b][3]);
          *reinterpret_cast<uint2*>(dx + (size_t)opix[b] * L::CIN + 4 * (g & 1)) = make_uint2(lo, hi);
        }
      }
    }
  };

  // ---- weight gradient of one tile (wgrad_ws_kernel<WgA2>'s strip body), software-pipelined over k-steps: k-step ks + NPW's fragments (address
  // math included) are read before k-step ks's MFMAs, pinned by scheduling barriers
  auto wg_load = [&](int ks, u2 (&af)[2], u2 (&bb)[L::NW][2]) {
    int pa[2], xb[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int P = 32 * ks + kpix(g, h, q4);
      const int r = P / L::W, ox = P - r * L::W;
      pa[h] = ((r + L::PAD) * L::RS + ox + L::PAD) * L::PS + 4 * p4;
      xb[h] = (r * L::XW + ox) * L::XS;
    }
    af[0] = tr4(dys + pa[0]);
    af[1] = tr4(dys + pa[1]);
#pragma unroll
    for (int j = 0; j < L::NW; ++j) {
      bb[j][0] = tr4(xs + xb[0] + xo[j]);
      bb[j][1] = tr4(xs + xb[1] + xo[j]);
    }
  };
  // the tile's interior pixel P (row P / W, column P % W) sits at dY tile row + PAD, column + PAD
  auto wgrad_tile = [&]() {
    int ks = wq;
    if (ks >= L::WKS) return;
    u2 af[2][2], bb[2][L::NW][2];
    wg_load(ks, af[0], bb[0]);
#pragma unroll 2
    for (int it = 0; ks < L::WKS; ks += L::NPW, ++it) {
      const int c = it & 1;
      if (ks + L::NPW < L::WKS) wg_load(ks + L::NPW, af[c ^ 1], bb[c ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 a8 = frag8(af[c][0], af[c][1]);
#pragma unroll
      for (int j = 0; j < L::NW; ++j) wacc[j] = mma(a8, frag8(bb[c][j][0], bb[c][j][1]), wacc[j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  {
    // tile ti in buffer (ti - t0) & 1: its MFMAs, then tile ti + 1 staged into the other buffer
    // (its loads were issued one tile earlier), then the loads of tile ti + 2; one barrier
    if (t0 < t1) {
      load_tile(t0, false);
      __syncthreads();   // ctab is written
      set_buf(0);
      store_tile(t0, false, nullptr, nullptr);
      if (t0 + 1 < t1) load_tile(t0 + 1, (t0 + 1) % L::TPS != 0);
      __syncthreads();
    }
    for (int ti = t0; ti < t1; ++ti) {
      const int b = (ti - t0) & 1;
      set_buf(b);
      dgrad_tile(ti);
      wgrad_tile();
      if (ti + 1 < t1) {
        const bf16* pd = dys;     // tile ti's images: its last rows may seed tile ti + 1
        const bf16* px = xs;
        set_buf(b ^ 1);   // last read by tile ti - 1, before the previous barrier
        store_tile(ti + 1, (ti + 1) % L::TPS != 0, pd, px);
        if (ti + 2 < t1) load_tile(ti + 2, (ti + 2) % L::TPS != 0);
      }
      __syncthreads();
    }
  }

  // ---- pixel-split dW partials -> wave 0 (fixed order), slab [co][ci][tap] through LDS
  f4* red = reinterpret_cast<f4*>(smem);
  __syncthreads();
  if (wq > 0) {
#pragma unroll
    for (int j = 0; j < L::NW; ++j) red[(((wq - 1) * L::NCW + wc) * L::NW + j) * 64 + lane] = wacc[j];
  }
  __syncthreads();
  if (wq == 0) {
#pragma unroll
    for (int w = 1; w < L::NPW; ++w)
#pragma unroll
      for (int j = 0; j < L::NW; ++j) wacc[j] += red[(((w - 1) * L::NCW + wc) * L::NW + j) * 64 + lane];
  }
  __syncthreads();
  constexpr int PER_CO = L::CIN * L::KK;
  float* tb = reinterpret_cast<float*>(smem);
  static_assert(L::COUT * PER_CO * 4 <= L::SMEM * 2, "slab tile fits");
  if (wq == 0) {
#pragma unroll
    for (int j = 0; j < L::NW; ++j) {
      const int tap = 2 * (wc * L::NW + j) + (r16 >> 3), ci = r16 & 7;
      if (tap >= L::KK) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) tb[(4 * g + i) * PER_CO + ci * L::KK + tap] = wacc[j][i];
    }
  }
  __syncthreads();
  float4* o4 = reinterpret_cast<float4*>(parts + (size_t)blockIdx.x * L::COUT * PER_CO);
  const float4* t4 = reinterpret_cast<const float4*>(tb);
  for (int e = tid; e < L::COUT * PER_CO / 4; e += 256) o4[e] = t4[e];
}

//          TH OCC PFD GB NCW RP
typedef Lb<8, 2, 3, 1, 4, 1> LbA2;

int lb_occ_ap() {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, lbwd_kernel<LbA2, 1>, 256, 0) != hipSuccess || occ <= 0)
      occ = 1;
  }
  return occ;
}

int lb_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

bool lb_serves(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad) {
  return dt == AVD_BF16 && !g_opts.generic_conv && N > 0 && Cin == LbA2::CIN && Cout == LbA2::COUT &&
         K == LbA2::K && pad == LbA2::PAD && H == LbA2::H && W == LbA2::W;
}

}  // namespace

int avd_cl_layer_bwd_slabs(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad) {
  if (!lb_serves(dt, N, Cin, H, W, Cout, K, pad)) return 0;
  const int ntiles = N * LbA2::TPS;
  return std::max(1, grid_cap(std::min(ntiles, lb_cus() * lb_occ_ap())));
}

int avd_cl_layer_bwd(const void* y, const void* gout, const float* scale, const float* shift,
                     const float* coef, const void* dy, const void* x, const void* wk_d, void* dx,
                     float* parts, int slabs, int dt, int N, int B, int Cin, int H, int W, int Cout,
                     int K, int pad, void* stream) {
  if (!lb_serves(dt, N, Cin, H, W, Cout, K, pad)) {
    avd_set_error(hipErrorInvalidValue);
    return AVD_ERR_SHAPE;
  }
  if (!x || !wk_d || !dx || !parts) return AVD_ERR_ARG;
  const bool ap = y != nullptr;
  if (ap ? (!gout || !scale || !shift || !coef) : !dy) return AVD_ERR_ARG;
  if (ap && (B <= 0 || N % B || N / B > APPLY_GMAX)) return AVD_ERR_SHAPE;
  const int ntiles = N * LbA2::TPS;
  // the caller's slab count (the parts buffer it sized) is the grid: no re-derivation here
  if (slabs < 1 || slabs > ntiles) return AVD_ERR_ARG;
  ApplyArgs aa{};
  aa.gout = gout; aa.scale = scale; aa.shift = shift; aa.coef = coef;
  aa.B = ap ? B : N; aa.G = ap ? N / B : 1;
  hipStream_t st = avd_stream(stream);
  if (ap)
    lbwd_kernel<LbA2, 1><<<slabs, 256, 0, st>>>((const bf16*)y, (const bf16*)x, (const bf16*)wk_d, (bf16*)dx,
                                                 parts, ntiles, aa);
  else
    lbwd_kernel<LbA2, 0><<<slabs, 256, 0, st>>>((const bf16*)dy, (const bf16*)x, (const bf16*)wk_d, (bf16*)dx,
                                                 parts, ntiles, aa);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}
