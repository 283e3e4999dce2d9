// Weights-stationary, persistent NHWC convolution (bf16, v_mfma_f32_16x16x32_bf16) for the
// fixed mid-layer shapes of the CentralNet encoders (unimodal.py:105-221): audio conv2-4
// (56x56 8->16, 28x28 16->32, 14x14 32->64, 5x5 p2) and the image conv2 (14x14 32->64, 5x5 p0),
// forward (bias + BatchNorm partials in the epilogue) and input gradient (flipped weights).
//
// Why a second conv kernel: the generic conv_cl_kernel re-reads its weight fragments from L2
// on every k-step in every wave and stages each tile synchronously, so it spends most cycles
// waiting (SQ_WAIT_ANY 56-75 %).  Here
//   * every wave loads its slice of the weights ONCE into registers (A fragments, up to 200
//     VGPRs) and keeps them for the whole launch;
//   * a persistent block walks a contiguous range of tiles (neighbouring row strips of one
//     sample stay on one XCD, so their halo rows hit L2);
//   * the next tile's input is loaded into registers while the MFMAs run on the current one
//     (one LDS buffer: barrier, write, barrier, issue next loads, compute).
// GEMM view per tile: M = output channels (A = weights [co][tap*CIN + c]), N = 16-pixel groups,
// K = (tap, channel); the B fragment (8 channels of one pixel and tap) is one ds_read_b128 of
// the channels-last LDS tile.  The K order and per-k-step accumulation order are those of
// conv_cl_kernel, so for CIN <= 32 both kernels return bit-identical maps.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "bnapply.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

__device__ const u4 kZero16 = {0u, 0u, 0u, 0u};

constexpr int cdv(int a, int b) { return (a + b - 1) / b; }

// One layer shape.  Tiles are TH full-width output rows of NS samples.  The 4 waves of a block
// split NCW ways over output channels, NKW ways over K (halves of the (tap, channel) range,
// summed through LDS in fixed order) and NPW = 4 / (NCW NKW) ways over the tile's pixel
// groups; a wave processes GB groups at a time (GB x NTW independent accumulator chains).
template <int CIN_, int COUT_, int K_, int PAD_, int H_, int W_, int TH_, int NS_, int NCW_,
          int NKW_, int GB_, int OCC_, int PF_ = 2>
struct Ws {
  static constexpr int OCC = OCC_;                         // target waves per SIMD
  static constexpr int PF = PF_;                           // k-steps of B reads in flight
  static constexpr int CIN = CIN_, COUT = COUT_, K = K_, PAD = PAD_, H = H_, W = W_;
  static constexpr int HO = H + 2 * PAD - K + 1, WO = W + 2 * PAD - K + 1;
  static constexpr int TH = TH_, TW = WO, NS = NS_;
  static constexpr int ITH = TH + K - 1, ITW = TW + K - 1;
  static constexpr int TPS = HO / TH;                      // tiles per sample group
  static constexpr int VPP = CIN / 8;                      // 16-byte vectors per pixel
  // LDS image [NS][ITH][RS][PS]: the pixel stride (PS elements) and the row pad (RS - ITW
  // pixels) make the B-fragment ds_read_b128 conflict-free across its four 16-lane groups for
  // every tap (found by simulating the gfx950 lane groups over all k-steps: ~4.2 LDS cycles per
  // read instead of 8-11.5 with the odd-16-byte strides)
  static constexpr int PS = VPP <= 2 ? CIN : CIN + 16;
  static constexpr int RS = ITW + (VPP == 1 ? 8 : 4);
  static constexpr int KK = K * K, KPAD = cdv(KK * CIN, 32) * 32, KS = KPAD / 32;
  static constexpr int NT = COUT <= 16 ? 1 : COUT / 16;
  static constexpr int NCW = NCW_, NKW = NKW_, NTW = NT / NCW, NPW = 4 / (NCW * NKW);
  static constexpr int KSH = cdv(KS, NKW);                 // k-steps per wave
  static constexpr int PIX = NS * TH * TW, G = cdv(PIX, 16), GW = cdv(G, NPW);
  static constexpr int GB = GB_;
  static constexpr int TASKS = NS * ITH * ITW * VPP, SLOTS = cdv(TASKS, 256);
  static constexpr int LDS_ELEMS = NS * ITH * RS * PS;
  static constexpr int RED = NKW > 1 ? 2 * NCW * GB * NTW * 64 : 1;   // f4 partial-sum slots
  static_assert(HO % TH == 0, "strips must tile the map");
  static_assert(NT % NCW == 0 && 4 % (NCW * NKW) == 0, "wave split");
  static_assert(NKW == 1 || CIN >= 32, "K split only where tap offsets are compile-time");
  static_assert(LDS_ELEMS * 2 + RED * 16 <= 96 * 1024, "LDS");
};

template <int V> using IC = std::integral_constant<int, V>;

// The tile loop advances pixel indices incrementally and forms bias / statistics on the packed
// fp32 ALU (round 4: fewer VALU per MFMA, bit-identical); B-fragment reads are pinned PF k-steps
// ahead of their MFMAs by sched_group_barrier (round 4: 188.9 k -> 191.7 k pairs/s).  Measured
// and removed: two tiles' input loads in flight (two register sets; 172-173 k vs 190-191 k).
typedef __attribute__((ext_vector_type(2))) float f2;

__device__ __forceinline__ f4 mma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Element offset, inside a pixel tile, of the B fragment of k-step ks for lane group g:
// tap (kh, kw) and channel chunk.  Padded k-groups (tap >= K*K) read tap 0 (weights are 0).
template <class L>
__device__ __forceinline__ int koff(int ks, int g) {
  const unsigned k0 = (unsigned)(4 * ks + g) * 8u;
  unsigned tap = k0 / (unsigned)L::CIN, c = k0 % (unsigned)L::CIN;
  if (tap >= (unsigned)L::KK) { tap = 0; c = 0; }
  return (int)(((tap / L::K) * L::RS + tap % L::K) * L::PS + c);
}

// AP (input gradient only): 0 = x is the staged operand itself (dY); 1 / 2 = x is the conv
// output y of the layer whose gradient this is, and the staging applies that layer's
// BatchNorm backward (bnapply.h) to produce dY in LDS, with the pooled gradient in layout 0 / 2
//
// RD (input gradient only, AP = 0): the epilogue also forms the BatchNorm-backward partial sums of
// the PREVIOUS layer, whose pooled output p is this conv's input and whose pooled gradient is
// the dX this kernel writes (what bwd_reduce_pooled_cl_kernel, bn_cl.hip, reads back from HBM):
// per channel sum dz and sum dz * xhat with dz = (p > 0 ? dX : 0) and xhat = (p - beta) / gamma
// (aa.gout = p, aa.scale = gamma, aa.shift = beta; sum dz * p is accumulated and turned into the
// xhat sum per row at the flush, so no per-channel constants occupy registers in the tile loop),
// as per-block running sums per BN group into
// stats [C][G][R = grid * NPW][2].  Channels with |beta| >> |gamma| contribute 0 to the second sum
// here; the launcher follows with bwd_reduce_pooled's fix-up pass, which rewrites every row
// from y when any channel needs it.
template <class L, bool FWD, int AP = 0, bool RD = false>
__global__ __launch_bounds__(256, (AP || (RD && L::OCC > 2)) ? (L::OCC > 1 ? L::OCC - 1 : 1) : L::OCC) void conv_ws_kernel(const bf16* __restrict__ x,
                                                      const bf16* __restrict__ wk,
                                                      const float* __restrict__ bias,
                                                      bf16* __restrict__ y,
                                                      float* __restrict__ stats, int ntiles,
                                                      int ngroups, ApplyArgs aa,
                                                      const float* __restrict__ pivot) {
  __shared__ __attribute__((aligned(16))) bf16 xs[L::LDS_ELEMS];
  __shared__ f4 red[L::RED];
  __shared__ __attribute__((aligned(16))) float ctab[AP ? APPLY_GMAX * 5 * L::CIN : 4];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int wc = wave % L::NCW, kw = (wave / L::NCW) % L::NKW, wp = wave / (L::NCW * L::NKW);
  const int cob = wc * L::NTW * 16;

  // ---- this wave's weight slice (k-steps kw*KSH ...), resident for the whole launch
  bf16x8 a[L::KSH][L::NTW];
  auto load_w = [&](auto kwc) {
    constexpr int KW = decltype(kwc)::value;
#pragma unroll
    for (int j = 0; j < L::KSH; ++j)
#pragma unroll
      for (int t = 0; t < L::NTW; ++t) {
        constexpr bf16x8 z = {};
        a[j][t] = KW * L::KSH + j < L::KS
                      ? *reinterpret_cast<const bf16x8*>(wk + (size_t)(cob + 16 * t + r16) * L::KPAD +
                                                         32 * (KW * L::KSH + j) + 8 * g)
                      : z;
      }
  };
  if constexpr (L::NKW == 1) load_w(IC<0>{});
  else if (kw == 0) load_w(IC<0>{});
  else load_w(IC<1>{});
  // per-lane tap offsets: for CIN >= 32 the lane part is just its channel chunk (8 g) and the
  // k-step part folds into the LDS read's immediate offset
  int toff[L::CIN >= 32 ? 1 : L::KS];
  if constexpr (L::CIN < 32) {
#pragma unroll
    for (int ks = 0; ks < L::KS; ++ks) toff[ks] = koff<L>(ks, g);
  } else {
    toff[0] = 8 * g;
  }
  // bias, and the statistics pivot: forward partials are shifted sums of (y - K[c]) and
  // (y - K[c])^2 about a per-channel K near the batch mean (the layer's running mean), so the
  // variance E[(y-K)^2] - E[y-K]^2 does not cancel when |mean| >> std (avd_bn_finalize pivot)
  f2 bv[L::NTW][2], pv[L::NTW][2];   // channel pairs
#pragma unroll
  for (int t = 0; t < L::NTW; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = cob + 16 * t + 4 * g + i;
      bv[t][i >> 1][i & 1] = (FWD && bias && co < L::COUT) ? bias[co] : 0.f;
      const float k = (FWD && pivot && co < L::COUT) ? pivot[co] : 0.f;
      pv[t][i >> 1][i & 1] = isfinite(k) ? k : 0.f;
    }
  constexpr bool STATS = FWD || RD;

  // ---- contiguous tile range of this block
  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);

  // staging slots (AP = 0): tile-invariant parts of each 16-byte task (source offset relative to the
  // tile's first sample and first input row incl. halo, LDS offset, halo row)
  int goff[L::SLOTS], loff[L::SLOTS], srow[L::SLOTS];
#pragma unroll
  for (int i = 0; i < L::SLOTS; ++i) {
    const int task = tid + 256 * i;
    const int q = task % L::VPP, pix = task / L::VPP;
    const int c = pix % L::ITW, rs = pix / L::ITW;
    const int r = rs % L::ITH, s = rs / L::ITH;
    const int ix = c - L::PAD;
    srow[i] = r;
    loff[i] = (rs * L::RS + c) * L::PS + 8 * q;
    goff[i] = (task < L::TASKS && ix >= 0 && ix < L::W)
                  ? ((s * L::H + r) * L::W + ix) * L::CIN + 8 * q : -1;
  }
  u4 pre[AP ? 1 : L::SLOTS];
  auto load_into = [&](u4 (&dst)[AP ? 1 : L::SLOTS], int ti) {
    const int sg = ti / L::TPS, tt = ti - sg * L::TPS;
    const int n0 = sg * L::NS, ty0 = tt * L::TH;
    // row ty0 - PAD of sample n0 (only dereferenced for in-range rows)
    const bf16* bx = x + ((long long)n0 * L::H + ty0 - L::PAD) * L::W * L::CIN;
    if constexpr (AP) return;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) {
      // halo / padding lanes load from a zero vector: no select on the loaded value, so
      // nothing waits for these loads before the next tile's LDS write
      const bool ok = goff[i] >= 0 && (unsigned)(ty0 - L::PAD + srow[i]) < (unsigned)L::H;
      const u4* src = ok ? reinterpret_cast<const u4*>(bx + goff[i]) : &kZero16;
      dst[i] = ldg16(src);
    }
  };
  auto load_tile = [&](int ti) { load_into(pre, ti); };
  auto store_pre = [&](const u4 (&src)[AP ? 1 : L::SLOTS]) {
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i)
      if (tid + 256 * i < L::TASKS) *reinterpret_cast<u4*>(xs + loff[i]) = src[i];
  };

  // staging slots (AP != 0): one task = one 2x2 pooling window x 8 channels of y (windows
  // are aligned: PAD and the tile rows are even), its pooled gradient, 4 dY vectors out
  constexpr int HP = L::H / 2, WP = L::W / 2;
  constexpr int WT = AP ? L::NS * (L::ITH / 2) * (L::ITW / 2) * L::VPP : 0;
  constexpr int WSL = AP ? cdv(WT, 256) : 1;
  int wgo[WSL], wgg[WSL], wlo[WSL], wrow[WSL];
  WinIn prew[WSL];
  if constexpr (AP) {
    static_assert(L::PAD % 2 == 0 && L::TH % 2 == 0 && L::H % 2 == 0 && L::W % 2 == 0, "windows");
    apply_load_ctab<L::CIN>(ctab, aa, tid, 256);
#pragma unroll
    for (int i = 0; i < WSL; ++i) {
      const int task = tid + 256 * i;
      const int q = task % L::VPP, w = task / L::VPP;
      const int wc2 = w % (L::ITW / 2), t = w / (L::ITW / 2);
      const int wr = t % (L::ITH / 2), s = t / (L::ITH / 2);
      const int r = 2 * wr, c = 2 * wc2, ix = c - L::PAD;
      wrow[i] = r;
      wlo[i] = ((s * L::ITH + r) * L::RS + c) * L::PS + 8 * q;
      wgo[i] = (task < WT && ix >= 0 && ix < L::W) ? ((s * L::H + r) * L::W + ix) * L::CIN + 8 * q : -1;
      wgg[i] = AP == 1 ? ((s * HP + wr) * WP + ix / 2) * L::CIN + 8 * q
                       : (s * L::CIN + 8 * q) * HP * WP + wr * WP + ix / 2;
    }
  }
  auto load_win_tile = [&](int ti) {
    const int sg = ti / L::TPS, tt = ti - sg * L::TPS;
    const int n0 = sg * L::NS, ty0 = tt * L::TH;
    const bf16* by = x + ((long long)n0 * L::H + ty0 - L::PAD) * L::W * L::CIN;
    const long long prow = (ty0 - L::PAD) / 2;   // exact: both even
#pragma unroll
    for (int i = 0; i < WSL; ++i) {
      const bool ok = wgo[i] >= 0 && (unsigned)(ty0 - L::PAD + wrow[i]) < (unsigned)L::H;
      const bf16* p = by + (ok ? wgo[i] : 0);
      prew[i].y[0] = ldg16(ok ? (const void*)(p) : &kZero16);
      prew[i].y[1] = ldg16(ok ? (const void*)(p + L::CIN) : &kZero16);
      prew[i].y[2] = ldg16(ok ? (const void*)(p + L::W * L::CIN) : &kZero16);
      prew[i].y[3] = ldg16(ok ? (const void*)(p + (L::W + 1) * L::CIN) : &kZero16);
      if constexpr (AP == 1) {
        const bf16* gb = reinterpret_cast<const bf16*>(aa.gout) + ((long long)n0 * HP + prow) * WP * L::CIN;
        prew[i].g0 = ldg16(ok ? (const void*)(gb + wgg[i]) : &kZero16);
      } else {
        const float* gb = reinterpret_cast<const float*>(aa.gout) + (long long)n0 * L::CIN * HP * WP + prow * WP;
        const float* gp = gb + (ok ? wgg[i] : 0);
        float gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) gv[e] = ok ? gp[(size_t)e * HP * WP] : 0.f;
        prew[i].g0 = u4{__float_as_uint(gv[0]), __float_as_uint(gv[1]), __float_as_uint(gv[2]), __float_as_uint(gv[3])};
        prew[i].g1 = u4{__float_as_uint(gv[4]), __float_as_uint(gv[5]), __float_as_uint(gv[6]), __float_as_uint(gv[7])};
      }
    }
  };
  auto store_win_tile = [&](int ti) {
    const int sg = ti / L::TPS, tt = ti - sg * L::TPS;
    const int n0 = sg * L::NS, ty0 = tt * L::TH;
    const float* ct = ctab + (n0 / aa.B) * 5 * L::CIN;
#pragma unroll
    for (int i = 0; i < WSL; ++i) {
      const int task = tid + 256 * i;
      if (task >= WT) continue;
      u4 o[4] = {u4{0u, 0u, 0u, 0u}, u4{0u, 0u, 0u, 0u}, u4{0u, 0u, 0u, 0u}, u4{0u, 0u, 0u, 0u}};
      if (wgo[i] >= 0 && (unsigned)(ty0 - L::PAD + wrow[i]) < (unsigned)L::H) {
        apply_window<AP == 1 ? 0 : 2, L::CIN>(prew[i], ct + 8 * (task % L::VPP), o);
        // dY out for the weight gradient: each window of the map once, from the tile whose
        // interior rows [PAD, PAD + TH) of the staged strip hold it (windows never straddle)
        if (aa.dy && (unsigned)(wrow[i] - L::PAD) < (unsigned)L::TH) {
          bf16* d = reinterpret_cast<bf16*>(aa.dy) + ((long long)n0 * L::H + ty0 - L::PAD) * L::W * L::CIN + wgo[i];
          *reinterpret_cast<u4*>(d) = o[0];
          *reinterpret_cast<u4*>(d + L::CIN) = o[1];
          *reinterpret_cast<u4*>(d + L::W * L::CIN) = o[2];
          *reinterpret_cast<u4*>(d + (L::W + 1) * L::CIN) = o[3];
        }
      }
      *reinterpret_cast<u4*>(xs + wlo[i]) = o[0];
      *reinterpret_cast<u4*>(xs + wlo[i] + L::PS) = o[1];
      *reinterpret_cast<u4*>(xs + wlo[i] + L::RS * L::PS) = o[2];
      *reinterpret_cast<u4*>(xs + wlo[i] + (L::RS + 1) * L::PS) = o[3];
    }
  };

  // BN partial sums (forward): per-block running sums over the block's tiles of one
  // BatchNorm group, one row per (block, pixel wave set) and group: [COUT][G][R = grid*NPW][2]
  f2 run_s[L::NTW][2], run_q[L::NTW][2];   // channel pairs (packed fp32 updates)
  int cur_g = -1;
  const int tilesPG = ntiles / ngroups, R = (int)gridDim.x * L::NPW;
  auto zero_run = [&]() {
#pragma unroll
    for (int t = 0; t < L::NTW; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i) { run_s[t][i] = f2{0.f, 0.f}; run_q[t][i] = f2{0.f, 0.f}; }
  };
  auto flush = [&](int gp) {   // wave-uniform call: the row sums are DPP across the 16 lanes
    if (kw != 0) return;
#pragma unroll
    for (int t = 0; t < L::NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        run_s[t][i >> 1][i & 1] = row16_sum(run_s[t][i >> 1][i & 1]);
        run_q[t][i >> 1][i & 1] = row16_sum(run_q[t][i >> 1][i & 1]);
      }
    if (r16 != 0) return;
#pragma unroll
    for (int t = 0; t < L::NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = cob + 16 * t + 4 * g + i;
        if (co < L::COUT) {
          float q = run_q[t][i >> 1][i & 1];
          if constexpr (RD) {
            // sum dz * xhat = (sum dz * p - beta * sum dz) / gamma; 0 for the fix-up channels
            const float ga = aa.scale[co], bb = aa.shift[co];
            q = (ga == 0.f || fabsf(bb) > 8.f * fabsf(ga)) ? 0.f : (q - bb * run_s[t][i >> 1][i & 1]) / ga;
          }
          *reinterpret_cast<float2*>(stats + (((size_t)co * ngroups + gp) * R + blockIdx.x * L::NPW + wp) * 2) =
              make_float2(run_s[t][i >> 1][i & 1], q);
        }
      }
  };
  zero_run();

  auto tile_body = [&](int ti) {
    const int sg = ti / L::TPS, tt = ti - sg * L::TPS;
    const int n0 = sg * L::NS, ty0 = tt * L::TH;
    // statistics: a new BN group starts a new running sum (lane-local over the block's tiles
    // of that group; summed across the 16 pixel lanes once, at the flush)
    if constexpr (STATS) {
      if (stats && kw == 0) {
        const int gi = ti / tilesPG;
        if (gi != cur_g) {
          if (cur_g >= 0) flush(cur_g);
          cur_g = gi;
          zero_run();
        }
      }
    }
    auto& ss = run_s;
    auto& sq = run_q;

    // per-lane pixel (sample, row, column) of each of the GB groups: divided out once per tile,
    // then advanced by DP pixels per step (one carry each way), not re-divided per group
    constexpr int DP = L::NPW * L::GB * 16, DRY = DP / L::TW, DRX = DP % L::TW;
    static_assert(DRY + 1 <= L::TH, "one row carry per step");
    int lp[L::GB], ls[L::GB], lry[L::GB], lrx[L::GB];
#pragma unroll
    for (int b = 0; b < L::GB; ++b) {
      lp[b] = (wp + L::NPW * b) * 16 + r16;
      ls[b] = lp[b] / (L::TH * L::TW);
      const int rem = lp[b] - ls[b] * (L::TH * L::TW);
      lry[b] = rem / L::TW;
      lrx[b] = rem - lry[b] * L::TW;
    }
#pragma unroll 1
    for (int i0 = 0; i0 < L::GW; i0 += L::GB) {
      int base[L::GB], opix[L::GB];
      bool gv[L::GB];
#pragma unroll
      for (int b = 0; b < L::GB; ++b) {
        const int p = lp[b], s = ls[b], ry = lry[b], rx = lrx[b];
        lp[b] += DP;
        lrx[b] += DRX;
        lry[b] += DRY;
        if (lrx[b] >= L::TW) { lrx[b] -= L::TW; ++lry[b]; }
        if constexpr (L::NS > 1) {
          if (lry[b] >= L::TH) { lry[b] -= L::TH; ++ls[b]; }
        }
        gv[b] = i0 + b < L::GW && p < L::PIX;
        base[b] = gv[b] ? ((s * L::ITH + ry) * L::RS + rx) * L::PS : 0;
        opix[b] = ((n0 + s) * L::HO + ty0 + ry) * L::WO + rx;
      }
      // RD: the pooled map at this wave's output elements, in flight under the MFMAs
      uint2 pq[RD ? L::GB : 1][RD ? L::NTW : 1];
      if constexpr (RD) {
#pragma unroll
        for (int b = 0; b < L::GB; ++b)
#pragma unroll
          for (int t = 0; t < L::NTW; ++t) {
            const int co = cob + 16 * t + 4 * g;
            pq[b][t] = (kw == 0 && gv[b] && co < L::COUT)
                           ? *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(aa.gout) +
                                                             (size_t)opix[b] * L::COUT + co)
                           : make_uint2(0u, 0u);
          }
      }
      f4 acc[L::GB][L::NTW];
#pragma unroll
      for (int b = 0; b < L::GB; ++b)
#pragma unroll
        for (int t = 0; t < L::NTW; ++t) acc[b][t] = f4{0.f, 0.f, 0.f, 0.f};
      // k-loop: B fragments PF k-steps ahead of their MFMAs
      auto kloop = [&](auto kwc) {
        constexpr int KW = decltype(kwc)::value;
        constexpr int PF = L::PF;
        bf16x8 bq[PF + 1][L::GB];
        auto ld = [&](bf16x8 (&dst)[L::GB], int j) {
#pragma unroll
          for (int b = 0; b < L::GB; ++b) {
            const int o = L::CIN >= 32 ? base[b] + toff[0] + koff<L>(KW * L::KSH + j, 0)
                                       : base[b] + toff[L::CIN >= 32 ? 0 : j];
            dst[b] = *reinterpret_cast<const bf16x8*>(xs + o);
          }
        };
#pragma unroll
        for (int j = 0; j < PF && j < L::KSH; ++j) ld(bq[j], j);
#pragma unroll
        for (int j = 0; j < L::KSH; ++j) {
          if (j + PF < L::KSH) ld(bq[(j + PF) % (PF + 1)], j + PF);
#pragma unroll
          for (int b = 0; b < L::GB; ++b)
#pragma unroll
            for (int t = 0; t < L::NTW; ++t)
              acc[b][t] = mma(a[j][t], bq[j % (PF + 1)][b], acc[b][t]);
        }
        // pin the interleave (hipcc otherwise pulls each B read down to one MFMA before its use
        // and waits lgkmcnt right there): PF k-steps of reads, then per k-step its MFMAs and the
        // reads of k-step j + PF
        __builtin_amdgcn_sched_group_barrier(0x100, L::GB * (PF < L::KSH ? PF : L::KSH), 0);
#pragma unroll
        for (int j = 0; j < L::KSH; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, L::GB * L::NTW, 0);
          if (j + PF < L::KSH) __builtin_amdgcn_sched_group_barrier(0x100, L::GB, 0);
        }
      };
      if constexpr (L::NKW == 1) {
        kloop(IC<0>{});
      } else {
        if (kw == 0) kloop(IC<0>{});
        else kloop(IC<1>{});
        // second K half -> first, through a double-buffered LDS slot (one barrier per batch)
        f4* r = red + (((i0 / L::GB) & 1) * L::NCW + wc) * L::GB * L::NTW * 64;
        if (kw == 1) {
#pragma unroll
          for (int b = 0; b < L::GB; ++b)
#pragma unroll
            for (int t = 0; t < L::NTW; ++t) r[(b * L::NTW + t) * 64 + lane] = acc[b][t];
        }
        __syncthreads();
        if (kw == 0) {
#pragma unroll
          for (int b = 0; b < L::GB; ++b)
#pragma unroll
            for (int t = 0; t < L::NTW; ++t) acc[b][t] += r[(b * L::NTW + t) * 64 + lane];
        }
      }
      if (kw != 0) continue;
      // ---- epilogue: (bias,) bf16 rounding, NHWC store of 4 channels per lane, BN partials
#pragma unroll
      for (int b = 0; b < L::GB; ++b) {
        if (!gv[b]) continue;
#pragma unroll
        for (int t = 0; t < L::NTW; ++t) {
          const int co = cob + 16 * t + 4 * g;
          if (co >= L::COUT) continue;
          uint32_t lo, hi;
          if constexpr (FWD) {
            // pairs through the packed fp32 ALU (v_pk_add / v_pk_fma: the same IEEE ops)
            const f2 y01 = f2{acc[b][t][0], acc[b][t][1]} + bv[t][0];
            const f2 y23 = f2{acc[b][t][2], acc[b][t][3]} + bv[t][1];
            lo = pack_bf16x2(y01.x, y01.y);
            hi = pack_bf16x2(y23.x, y23.y);
            const f2 d01 = f2{__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u)} - pv[t][0];
            const f2 d23 = f2{__uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)} - pv[t][1];
            ss[t][0] += d01;
            ss[t][1] += d23;
            sq[t][0] = __builtin_elementwise_fma(d01, d01, sq[t][0]);
            sq[t][1] = __builtin_elementwise_fma(d23, d23, sq[t][1]);
          } else {
            lo = pack_bf16x2(acc[b][t][0], acc[b][t][1]);
            hi = pack_bf16x2(acc[b][t][2], acc[b][t][3]);
            if constexpr (RD) {   // sums over the stored (rounded) gradient, as the reduce reads it
              const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                  __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
              const float pv[4] = {__uint_as_float(pq[b][t].x << 16), __uint_as_float(pq[b][t].x & 0xffff0000u),
                                   __uint_as_float(pq[b][t].y << 16), __uint_as_float(pq[b][t].y & 0xffff0000u)};
#pragma unroll
              for (int i = 0; i < 4; ++i) {   // sum dz and sum dz * p (xhat applied at the flush)
                const float dz = pv[i] > 0.f ? v[i] : 0.f;
                ss[t][i >> 1][i & 1] += dz;
                sq[t][i >> 1][i & 1] = fmaf(dz, pv[i], sq[t][i >> 1][i & 1]);
              }
            }
          }
          *reinterpret_cast<uint2*>(y + (size_t)opix[b] * L::COUT + co) = make_uint2(lo, hi);
        }
      }
    }
  };

  if (t0 < t1) { if constexpr (AP) load_win_tile(t0); else load_tile(t0); }
  for (int ti = t0; ti < t1; ++ti) {
    __syncthreads();   // every wave is done reading the previous tile (and ctab is written)
    if constexpr (AP) store_win_tile(ti); else store_pre(pre);
    __syncthreads();
    if (ti + 1 < t1) {   // in flight under this tile's MFMAs
      if constexpr (AP) load_win_tile(ti + 1); else load_tile(ti + 1);
    }
    tile_body(ti);
  }
  if constexpr (STATS) {
    if (stats) {
      if (cur_g >= 0) flush(cur_g);
      // groups this block never reached (its tiles cover groups [first, last]): zero rows
      const int first = t0 < t1 ? t0 / tilesPG : 0, last = t0 < t1 ? (t1 - 1) / tilesPG : -1;
      zero_run();
      for (int gp = 0; gp < ngroups; ++gp)
        if (gp < first || gp > last) flush(gp);
    }
  }
}

// ----------------------------------------------------------------------------- layer table
//        CIN COUT K PAD  H   W  TH NS NCW NKW GB OCC
// (PF 6 everywhere: the step A/B above; the times are the round-3/4 per-layer picks at their
// earlier PF)
typedef Ws<8, 16, 5, 2, 56, 56, 14, 1, 1, 1, 2, 2, 6> FwdA2;  // audio conv2        273 us
typedef Ws<16, 32, 5, 2, 28, 28, 14, 1, 2, 1, 1, 2, 6> FwdA3; // audio conv3 194 us (NCW 1: 236 us, spilled)
typedef Ws<32, 64, 5, 2, 14, 14, 14, 1, 4, 1, 2, 2, 6> FwdA4; // audio conv4        168 us
typedef Ws<32, 64, 5, 0, 14, 14, 10, 2, 4, 1, 2, 2, 6> FwdI2; // image conv2         87 us
typedef Ws<16, 8, 5, 2, 56, 56, 8, 1, 1, 1, 1, 3, 6> DgrA2;   // audio conv2 dgrad  275 us
typedef Ws<32, 16, 5, 2, 28, 28, 14, 1, 1, 1, 2, 2, 6> DgrA3; // audio conv3 dgrad  145 us
typedef Ws<64, 32, 5, 2, 14, 14, 14, 1, 2, 2, 2, 2, 6> DgrA4; // audio conv4 dgrad  158 us
typedef Ws<64, 32, 5, 4, 10, 10, 14, 1, 2, 2, 2, 2, 6> DgrI2; // image conv2 dgrad  154 us

// avd_options.generic_conv: every bf16 mid layer on the generic conv_cl kernels (parity tests)
bool ws_disabled() { return g_opts.generic_conv != 0; }

int num_cus() {
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

// resident blocks per CU of one instantiation (cached per instantiation: the device's CU
// count and register file are the same for every device of a homogeneous node)
template <class L, bool FWD, int AP, bool RD>
int ws_occ() {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv_ws_kernel<L, FWD, AP, RD>, 256, 0) !=
            hipSuccess || occ <= 0)
      occ = 1;
  }
  return occ;
}

// the grid of a launch that writes BatchNorm partials (forward statistics, or the RD dgrad's
// backward sums): one resident wave of blocks, so R = grid * NPW rows per group is fixed
template <class L, bool FWD = true, bool RD = false>
int ws_stat_grid() {
  return grid_cap(num_cus() * ws_occ<L, FWD, 0, RD>());
}

template <class L, bool FWD, int AP = 0, bool RD = false>
int launch_ws(const void* x, const void* wk, const float* bias, void* y, float* stats, int N,
              int B, hipStream_t st, const ApplyArgs& aa = ApplyArgs{}, const float* pivot = nullptr) {
  constexpr bool STATS = FWD || RD;
  if (N % L::NS || (STATS && stats && B % L::NS)) return AVD_ERR_SHAPE;
  if (AP && (aa.B % L::NS || aa.G > APPLY_GMAX || aa.G * aa.B != N)) return AVD_ERR_SHAPE;
  const int ntiles = (N / L::NS) * L::TPS;
  const int grid = STATS && stats ? ws_stat_grid<L, FWD, RD>()
                                  : grid_cap(std::min(ntiles, num_cus() * ws_occ<L, FWD, AP, RD>()));
  conv_ws_kernel<L, FWD, AP, RD><<<grid, 256, 0, st>>>((const bf16*)x, (const bf16*)wk, bias, (bf16*)y,
                                                       stats, ntiles, STATS && stats ? N / B : 1, aa,
                                                       FWD ? pivot : nullptr);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

template <class L>
bool is(int Cin, int H, int W, int Cout, int K, int pad) {
  return Cin == L::CIN && Cout == L::COUT && K == L::K && pad == L::PAD && H == L::H && W == L::W;
}

template <class L>
bool out_is(int Cin, int Ho, int Wo, int Cout, int K) {
  return Cin == L::CIN && Cout == L::COUT && K == L::K && Ho == L::HO && Wo == L::WO;
}

}  // namespace

// Rows of BN partials per group written by the weights-stationary forward, 0 if it does not
// serve the shape (bf16 only).
int avd_ws_stat_rows(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt) {
  if (dt != AVD_BF16 || ws_disabled()) return 0;
  auto rows = [&](auto l) -> int {
    typedef decltype(l) L;
    return B % L::NS ? 0 : ws_stat_grid<L>() * L::NPW;
  };
  if (out_is<FwdA2>(Cin, Ho, Wo, Cout, K)) return rows(FwdA2{});
  if (out_is<FwdA3>(Cin, Ho, Wo, Cout, K)) return rows(FwdA3{});
  if (out_is<FwdA4>(Cin, Ho, Wo, Cout, K)) return rows(FwdA4{});
  if (out_is<FwdI2>(Cin, Ho, Wo, Cout, K)) return rows(FwdI2{});
  return 0;
}

// 1 = launched, 0 = shape not served (caller falls back), < 0 = error
int avd_ws_conv_fwd(const void* x, const void* wk, const float* bias, void* y, float* stats,
                    int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                    hipStream_t st, const float* pivot) {
  if (dt != AVD_BF16 || ws_disabled()) return 0;
  int r = 0;
  const ApplyArgs aa{};
  if (is<FwdA2>(Cin, H, W, Cout, K, pad)) r = launch_ws<FwdA2, true>(x, wk, bias, y, stats, N, B, st, aa, pivot);
  else if (is<FwdA3>(Cin, H, W, Cout, K, pad)) r = launch_ws<FwdA3, true>(x, wk, bias, y, stats, N, B, st, aa, pivot);
  else if (is<FwdA4>(Cin, H, W, Cout, K, pad)) r = launch_ws<FwdA4, true>(x, wk, bias, y, stats, N, B, st, aa, pivot);
  else if (is<FwdI2>(Cin, H, W, Cout, K, pad)) r = launch_ws<FwdI2, true>(x, wk, bias, y, stats, N, B, st, aa, pivot);
  else return 0;
  return r == AVD_OK ? 1 : (r == AVD_ERR_SHAPE ? 0 : r);
}

// dgrad of a forward conv (Cin -> Cout over H x W, pad): the kernel runs on dY (Cout channels,
// Ho x Wo) with the flipped weights and padding K-1-pad, producing dX (Cin channels, H x W).
int avd_ws_conv_dgrad(const void* dy, const void* wk_d, void* dx, int dt, int N, int Cin, int H,
                      int W, int Cout, int K, int pad, hipStream_t st) {
  if (dt != AVD_BF16 || ws_disabled()) return 0;
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1, dp = K - 1 - pad;
  int r = 0;
  if (is<DgrA2>(Cout, Ho, Wo, Cin, K, dp)) r = launch_ws<DgrA2, false>(dy, wk_d, nullptr, dx, nullptr, N, N, st);
  else if (is<DgrA3>(Cout, Ho, Wo, Cin, K, dp)) r = launch_ws<DgrA3, false>(dy, wk_d, nullptr, dx, nullptr, N, N, st);
  else if (is<DgrA4>(Cout, Ho, Wo, Cin, K, dp)) r = launch_ws<DgrA4, false>(dy, wk_d, nullptr, dx, nullptr, N, N, st);
  else if (is<DgrI2>(Cout, Ho, Wo, Cin, K, dp)) r = launch_ws<DgrI2, false>(dy, wk_d, nullptr, dx, nullptr, N, N, st);
  else return 0;
  return r == AVD_OK ? 1 : (r == AVD_ERR_SHAPE ? 0 : r);
}

