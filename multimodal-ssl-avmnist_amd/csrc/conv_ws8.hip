// fp8 (OCP e4m3fn) weights-stationary convolution on the BLOCK-SCALED MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 (gfx950: 2x the bf16 MFMA rate, half the LDS bytes per k)
// for the mid-layer convs of the CentralNet encoders (unimodal.py:105-221): forward (+bias,
// BatchNorm partial sums) and input gradient, BASELINE config 5's "fp8 MFMA conv path".
//
// Same persistent tiling as conv_ws_kernel (conv_ws.hip): a block walks a contiguous range of
// TH-row strips, the next strip's bf16 input is loaded into registers under the current strip's
// MFMAs, the weights stay in registers for the whole launch.  What changes:
//   * operands are e4m3 with E8M0 block scales (the MX form).  The WEIGHTS are quantised once per
//     step (avd_mx_weight_layout) with one scale per (output channel, 32-k block) -- the
//     instruction's own A-scale granularity; the INPUT map stays bf16 in HBM (BatchNorm, pooling
//     and the other consumers read it) and is quantised while staged, with one power-of-two
//     scale per staged strip (its max |x| maps into [128, 256): no overflow, exact rescaling)
//     passed as the B scale of every MFMA of the strip;
//   * K = (tap, channel) runs 128 per MFMA: a lane holds two 16-k pieces of one output pixel
//     (mx_k below: the instruction's operand layout, measured), read from the staged fp8 strip
//     as 4 x ds_read_b64 (8 channels: 2 taps per piece) or 2 x ds_read_b128 (16 channels: one
//     tap per piece; 32 / 64 channels: 16 channels of one tap); pixel stride and row pad of the
//     strip from tools/lds_bank_sim8.py.
// Accumulation is f32 in the MFMA; y = bf16(acc + bias) and the statistics epilogue are those of
// conv_ws_kernel.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace avd;

// 1: LDS reads pinned PF k-steps / columns ahead of their MFMAs by sched_group_barrier

namespace {

typedef __attribute__((ext_vector_type(8))) int i8v;     // 32 fp8 bytes: one MX operand
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

__device__ const u4 kZero8 = {0u, 0u, 0u, 0u};

constexpr int cdv(int a, int b) { return (a + b - 1) / b; }

// One layer shape (as conv_ws.hip's Ws) plus the fp8 strip geometry: PS bytes per staged pixel,
// RP pixels of row pad.
template <int CIN_, int COUT_, int K_, int PAD_, int H_, int W_, int TH_, int NS_, int NCW_,
          int NKW_, int GB_, int OCC_, int PS_, int RP_, int PF_ = 2>
struct W8 {
  static constexpr int OCC = OCC_, PF = PF_;
  static constexpr int CIN = CIN_, COUT = COUT_, K = K_, PAD = PAD_, H = H_, W = W_;
  static constexpr int HO = H + 2 * PAD - K + 1, WO = W + 2 * PAD - K + 1;
  static constexpr int TH = TH_, TW = WO, NS = NS_;
  static constexpr int ITH = TH + K - 1, ITW = TW + K - 1;
  static constexpr int TPS = HO / TH;
  static constexpr int VPP = CIN / 8;                      // 16-byte bf16 loads per pixel
  static constexpr int PS = PS_, RS = ITW + RP_;
  static constexpr int KK = K * K, KPAD = cdv(KK * CIN, 128) * 128, KS = KPAD / 128;
  static constexpr int NT = COUT <= 16 ? 1 : COUT / 16;
  static constexpr int NCW = NCW_, NKW = NKW_, NTW = NT / NCW, NPW = 4 / (NCW * NKW);
  static constexpr int KSH = cdv(KS, NKW);
  static constexpr int PIX = NS * TH * TW, G = cdv(PIX, 16), GW = cdv(G, NPW);
  static constexpr int GB = GB_;
  static constexpr int TASKS = NS * ITH * ITW * VPP, SLOTS = cdv(TASKS, 256);
  static constexpr int LDS_BYTES = NS * ITH * RS * PS;
  static constexpr int NR = CIN == 8 ? 4 : 2;              // LDS reads per fragment
  static constexpr int RED = NKW > 1 ? 2 * NCW * GB * NTW * 64 : 1;
  static_assert(HO % TH == 0, "strips must tile the map");
  static_assert(NT % NCW == 0 && 4 % (NCW * NKW) == 0, "wave split");
  static_assert(CIN % 8 == 0 && PS % 8 == 0 && PS >= CIN, "pixel stride");
  static_assert(LDS_BYTES + RED * 16 <= 96 * 1024, "LDS");
};

// The MX operand layout of v_mfma_scale_f32_16x16x128_f8f6f4 (measured with exact data and
// per-lane scales, tools/probe/mx_probe.hip): lane l of row / column r = l & 15 and group
// g = l >> 4 holds k = 16 g .. 16 g + 15 in its bytes 0-15 and k = 64 + 16 g .. + 15 in bytes
// 16-31; the scale register of lane r + 16 b is the scale of k-block b = [32 b, 32 b + 32).
// k of byte piece p (0, 1) of lane group g in k-step ks:
__device__ __forceinline__ int mx_k(int ks, int g, int p) { return 128 * ks + 64 * p + 16 * g; }

// byte offset, inside the staged strip, of read u of the fragment of k-step ks for lane group
// g: 8 channels -> four 8-byte reads (two taps per piece), else one 16-byte read per piece
template <class L>
__device__ __forceinline__ int koff8(int ks, int g, int u) {
  const int k0 = L::CIN == 8 ? mx_k(ks, g, u >> 1) + 8 * (u & 1) : mx_k(ks, g, u);
  int tap = k0 / L::CIN, c = k0 % L::CIN;
  if (tap >= L::KK) { tap = 0; c = 0; }                    // padded k: weights are zero there
  return ((tap / L::K) * L::RS + tap % L::K) * L::PS + c;
}

__device__ __forceinline__ unsigned absmax_bf16x8(u4 v, unsigned m) {
#pragma unroll
  for (int i = 0; i < 4; ++i) m = max(m, max(v[i] & 0x7fffu, (v[i] >> 16) & 0x7fffu));
  return m;
}

// 8 bf16 * mul -> 8 e4m3 bytes (RNE; |x * mul| < 256 by construction of mul)
__device__ __forceinline__ uint2 q8(u4 v, float mul) {
  float f[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16) * mul;
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u) * mul;
  }
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}

// power-of-two scale for a block whose max |v| is am: v * 2^s in [128, 256) at the max; E8M0 of
// the inverse factor 2^-s is 127 - s (kept inside the finite E8M0 range)
__device__ __forceinline__ int mx_shift(float am) {
  if (!(am > 0.f)) return 0;
  int e;
  (void)frexpf(am, &e);                                    // am in [2^(e-1), 2^e)
  return min(max(8 - e, -126), 126);
}

// D += A B on the block-scaled MFMA, e4m3 x e4m3; the A scale is byte `sel` of sa (the
// operand's byte select), the B scale the low byte of sb.  sel folds to a constant when unrolled.
template <int SEL>
__device__ __forceinline__ f4 mxmma_(i8v a, i8v b, f4 c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, SEL, sa, 0, sb);
}
__device__ __forceinline__ f4 mxmma(int sel, i8v a, i8v b, f4 c, int sa, int sb) {
  switch (sel) {
    case 0: return mxmma_<0>(a, b, c, sa, sb);
    case 1: return mxmma_<1>(a, b, c, sa, sb);
    case 2: return mxmma_<2>(a, b, c, sa, sb);
    default: return mxmma_<3>(a, b, c, sa, sb);
  }
}

template <class L, bool FWD>
__global__ __launch_bounds__(256, L::OCC) void conv_ws8_kernel(
    const bf16* __restrict__ x, const unsigned char* __restrict__ wq,
    const unsigned char* __restrict__ wsc, const float* __restrict__ bias, bf16* __restrict__ y,
    float* __restrict__ stats, int ntiles, int ngroups, const float* __restrict__ pivot) {
  __shared__ __attribute__((aligned(16))) unsigned char xs[L::LDS_BYTES];
  __shared__ f4 red[L::RED];
  __shared__ unsigned amx[4];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int wc = wave % L::NCW, kw = (wave / L::NCW) % L::NKW, wp = wave / (L::NCW * L::NKW);
  const int cob = wc * L::NTW * 16;

  // ---- this wave's weight slice and its block scales (4 per register, picked by the MFMA's
  // scale-operand byte select), resident for the whole launch
  constexpr int KSH4 = cdv(L::KSH, 4);
  i8v a[L::KSH][L::NTW];
  int sa[KSH4][L::NTW];
  int toff[L::KSH][L::NR];
#pragma unroll
  for (int j = 0; j < KSH4; ++j)
#pragma unroll
    for (int t = 0; t < L::NTW; ++t) sa[j][t] = 0x7f7f7f7f;
#pragma unroll
  for (int j = 0; j < L::KSH; ++j) {
    const int ks = kw * L::KSH + j;
    const bool live = ks < L::KS;
#pragma unroll
    for (int t = 0; t < L::NTW; ++t) {
      const int row = cob + 16 * t + r16;
      if (live) {
        const u4 lo = *reinterpret_cast<const u4*>(wq + (size_t)row * L::KPAD + mx_k(ks, g, 0));
        const u4 hi = *reinterpret_cast<const u4*>(wq + (size_t)row * L::KPAD + mx_k(ks, g, 1));
        a[j][t] = i8v{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      } else {
        a[j][t] = i8v{0, 0, 0, 0, 0, 0, 0, 0};
      }
      const int sc = live ? (int)wsc[(size_t)row * (L::KPAD / 32) + 4 * ks + g] : 127;
      sa[j / 4][t] = (sa[j / 4][t] & ~(0xff << (8 * (j % 4)))) | (sc << (8 * (j % 4)));
    }
#pragma unroll
    for (int u = 0; u < L::NR; ++u) toff[j][u] = koff8<L>(live ? ks : 0, g, u);
  }
  float bv[L::NTW][4], pv[L::NTW][4];
#pragma unroll
  for (int t = 0; t < L::NTW; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = cob + 16 * t + 4 * g + i;
      bv[t][i] = (FWD && bias && co < L::COUT) ? bias[co] : 0.f;
      const float k = (FWD && pivot && co < L::COUT) ? pivot[co] : 0.f;
      pv[t][i] = isfinite(k) ? k : 0.f;
    }

  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);

  // staging slot i = 16-byte task tid + 256 i of the strip (8 channels of one input pixel):
  // its offsets are recomputed per strip (compile-time divisors) instead of held in registers
  struct Slot { int goff, loff, row; };
  auto slot = [&](int i) -> Slot {
    const int task = tid + 256 * i;
    const int q = task % L::VPP, pix = task / L::VPP;
    const int c = pix % L::ITW, rs = pix / L::ITW;
    const int r = rs % L::ITH, s = rs / L::ITH;
    const int ix = c - L::PAD;
    return Slot{(task < L::TASKS && ix >= 0 && ix < L::W) ? ((s * L::H + r) * L::W + ix) * L::CIN + 8 * q : -1,
                (rs * L::RS + c) * L::PS + 8 * q, r};
  };
  u4 pre[L::SLOTS];
  auto load_tile = [&](int ti) {
    const int sg = ti / L::TPS, tt = ti - sg * L::TPS;
    const int n0 = sg * L::NS, ty0 = tt * L::TH;
    const bf16* bx = x + ((long long)n0 * L::H + ty0 - L::PAD) * L::W * L::CIN;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) {
      const Slot sl = slot(i);
      const bool ok = sl.goff >= 0 && (unsigned)(ty0 - L::PAD + sl.row) < (unsigned)L::H;
      pre[i] = ldg16(ok ? (const void*)(bx + sl.goff) : (const void*)&kZero8);
    }
  };

  float run_s[L::NTW][4], run_q[L::NTW][4];
  int cur_g = -1;
  const int tilesPG = ntiles / ngroups, R = (int)gridDim.x * L::NPW;
  auto zero_run = [&]() {
#pragma unroll
    for (int t = 0; t < L::NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) { run_s[t][i] = 0.f; run_q[t][i] = 0.f; }
  };
  auto flush = [&](int gp) {
    if (kw != 0) return;
#pragma unroll
    for (int t = 0; t < L::NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        run_s[t][i] = row16_sum(run_s[t][i]);
        run_q[t][i] = row16_sum(run_q[t][i]);
      }
    if (r16 != 0) return;
#pragma unroll
    for (int t = 0; t < L::NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = cob + 16 * t + 4 * g + i;
        if (co < L::COUT)
          *reinterpret_cast<float2*>(stats + (((size_t)co * ngroups + gp) * R + blockIdx.x * L::NPW + wp) * 2) =
              make_float2(run_s[t][i], run_q[t][i]);
      }
  };
  zero_run();

  if (t0 < t1) load_tile(t0);
  for (int ti = t0; ti < t1; ++ti) {
    // the strip's max |x| (its loads are in pre[]): per wave, then through LDS
    unsigned m = 0u;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) m = absmax_bf16x8(pre[i], m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
    if (lane == 0) amx[wave] = m;
    __syncthreads();   // every wave is done reading the previous strip; amx complete
    m = max(max(amx[0], amx[1]), max(amx[2], amx[3]));
    const int sh = mx_shift(__uint_as_float(m << 16));
    const float mul = ldexpf(1.f, sh);
    const int sb = 127 - sh;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i)
      if (tid + 256 * i < L::TASKS) *reinterpret_cast<uint2*>(xs + slot(i).loff) = q8(pre[i], mul);
    __syncthreads();
    if (ti + 1 < t1) load_tile(ti + 1);   // in flight under this strip's MFMAs

    const int sg = ti / L::TPS, tt = ti - sg * L::TPS;
    const int n0 = sg * L::NS, ty0 = tt * L::TH;
    if (FWD && stats && kw == 0) {
      const int gi = ti / tilesPG;
      if (gi != cur_g) {
        if (cur_g >= 0) flush(cur_g);
        cur_g = gi;
        zero_run();
      }
    }

    for (int i0 = 0; i0 < L::GW; i0 += L::GB) {
      int base[L::GB], opix[L::GB];
      bool gv[L::GB];
#pragma unroll
      for (int b = 0; b < L::GB; ++b) {
        const int p = (wp + L::NPW * (i0 + b)) * 16 + r16;
        gv[b] = i0 + b < L::GW && p < L::PIX;
        const int s = p / (L::TH * L::TW), rem = p - s * (L::TH * L::TW);
        const int ry = rem / L::TW, rx = rem - ry * L::TW;
        base[b] = gv[b] ? ((s * L::ITH + ry) * L::RS + rx) * L::PS : 0;
        opix[b] = ((n0 + s) * L::HO + ty0 + ry) * L::WO + rx;
      }
      f4 acc[L::GB][L::NTW];
#pragma unroll
      for (int b = 0; b < L::GB; ++b)
#pragma unroll
        for (int t = 0; t < L::NTW; ++t) acc[b][t] = f4{0.f, 0.f, 0.f, 0.f};
      {
        constexpr int PF = L::PF;
        i8v bq[PF + 1][L::GB];
        auto ld = [&](i8v (&dst)[L::GB], int j) {
#pragma unroll
          for (int b = 0; b < L::GB; ++b) {
            if constexpr (L::CIN == 8) {
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const uint2 v = *reinterpret_cast<const uint2*>(xs + base[b] + toff[j][u]);
                dst[b][2 * u] = (int)v.x;
                dst[b][2 * u + 1] = (int)v.y;
              }
            } else {
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const u4 v = *reinterpret_cast<const u4*>(xs + base[b] + toff[j][u]);
                dst[b][4 * u] = (int)v.x;
                dst[b][4 * u + 1] = (int)v.y;
                dst[b][4 * u + 2] = (int)v.z;
                dst[b][4 * u + 3] = (int)v.w;
              }
            }
          }
        };
        constexpr int KN = L::KS - (L::NKW - 1) * L::KSH;   // k-steps of the last K part
        const int kn = kw == L::NKW - 1 ? KN : L::KSH;
#pragma unroll
        for (int j = 0; j < PF && j < L::KSH; ++j) ld(bq[j], j);
#pragma unroll
        for (int j = 0; j < L::KSH; ++j) {
          if (j + PF < L::KSH) ld(bq[(j + PF) % (PF + 1)], j + PF);
          if (j < kn) {
#pragma unroll
            for (int b = 0; b < L::GB; ++b)
#pragma unroll
              for (int t = 0; t < L::NTW; ++t)
                acc[b][t] = mxmma(j % 4, a[j][t], bq[j % (PF + 1)][b], acc[b][t], sa[j / 4][t], sb);
          }
        }
      }
      if constexpr (L::NKW > 1) {
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
#pragma unroll
      for (int b = 0; b < L::GB; ++b) {
        if (!gv[b]) continue;
#pragma unroll
        for (int t = 0; t < L::NTW; ++t) {
          const int co = cob + 16 * t + 4 * g;
          if (co >= L::COUT) continue;
          uint32_t lo, hi;
          if constexpr (FWD) {
            lo = pack_bf16x2(acc[b][t][0] + bv[t][0], acc[b][t][1] + bv[t][1]);
            hi = pack_bf16x2(acc[b][t][2] + bv[t][2], acc[b][t][3] + bv[t][3]);
            if (stats) {
              const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                  __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float d = v[i] - pv[t][i];
                run_s[t][i] += d;
                run_q[t][i] = fmaf(d, d, run_q[t][i]);
              }
            }
          } else {
            lo = pack_bf16x2(acc[b][t][0], acc[b][t][1]);
            hi = pack_bf16x2(acc[b][t][2], acc[b][t][3]);
          }
          *reinterpret_cast<uint2*>(y + (size_t)opix[b] * L::COUT + co) = make_uint2(lo, hi);
        }
      }
    }
  }
  if (FWD && stats) {
    if (cur_g >= 0) flush(cur_g);
    const int first = t0 < t1 ? t0 / tilesPG : 0, last = t0 < t1 ? (t1 - 1) / tilesPG : -1;
    zero_run();
    for (int gp = 0; gp < ngroups; ++gp)
      if (gp < first || gp > last) flush(gp);
  }
}

// ----------------------------------------------------------------------------- layer table
//        CIN COUT K PAD  H   W  TH NS NCW NKW GB OCC PS RP
typedef W8<8, 16, 5, 2, 56, 56, 14, 1, 1, 1, 2, 3, 8, 7> F8A2;     // audio conv2 forward
typedef W8<16, 32, 5, 2, 28, 28, 14, 1, 1, 1, 1, 2, 16, 12> F8A3;  // audio conv3
typedef W8<32, 64, 5, 2, 14, 14, 14, 1, 2, 2, 1, 2, 32, 4> F8A4;   // audio conv4
typedef W8<32, 64, 5, 0, 14, 14, 10, 2, 2, 2, 1, 2, 32, 4> F8I2;   // image conv2
typedef W8<16, 8, 5, 2, 56, 56, 8, 1, 1, 1, 1, 3, 16, 12> D8A2;    // audio conv2 input gradient
typedef W8<32, 16, 5, 2, 28, 28, 14, 1, 1, 1, 1, 2, 32, 4> D8A3;   // audio conv3
typedef W8<64, 32, 5, 2, 14, 14, 14, 1, 2, 2, 2, 2, 96, 4> D8A4;   // audio conv4
typedef W8<64, 32, 5, 4, 10, 10, 14, 1, 2, 2, 2, 2, 96, 4> D8I2;   // image conv2

int num_cus8() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <class L, bool FWD>
int occ8() {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv_ws8_kernel<L, FWD>, 256, 0) != hipSuccess ||
        occ <= 0)
      occ = 1;
  }
  return occ;
}

template <class L>
int stat_grid8() { return grid_cap(num_cus8() * occ8<L, true>()); }

template <class L, bool FWD>
int launch8(const void* x, const void* wq, const void* wsc, const float* bias, void* y, float* stats,
            int N, int B, hipStream_t st, const float* pivot) {
  const bool S = FWD && stats;
  if (N % L::NS || (S && B % L::NS)) return AVD_ERR_SHAPE;
  const int ntiles = (N / L::NS) * L::TPS;
  int grid = grid_cap(std::min(ntiles, num_cus8() * occ8<L, FWD>()));
  if constexpr (FWD)
    if (S) grid = stat_grid8<L>();
  conv_ws8_kernel<L, FWD><<<grid, 256, 0, st>>>((const bf16*)x, (const unsigned char*)wq,
                                               (const unsigned char*)wsc, bias, (bf16*)y,
                                               S ? stats : nullptr, ntiles, S ? N / B : 1,
                                               FWD ? pivot : nullptr);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

template <class L>
bool is8(int Cin, int H, int W, int Cout, int K, int pad) {
  return Cin == L::CIN && Cout == L::COUT && K == L::K && pad == L::PAD && H == L::H && W == L::W;
}

// MX weight layout: rows o (forward: output channels; input gradient: input channels, with
// the taps flipped), k = tap * C + c zero-padded to KPAD = 128 * ceil(K*K*C / 128); one e4m3
// byte per k and one E8M0 byte per 32-k block (its max |w| into [128, 256))
__device__ __forceinline__ void mx_weight_block(const float* __restrict__ w, unsigned char* __restrict__ wq,
                                                unsigned char* __restrict__ wsc, int Cout, int Cin,
                                                int KK, int dgrad, int kpad, int i) {
  const int nb = kpad / 32;
  const int o = i / nb, kb = i - o * nb;
  const int O = dgrad ? Cin : Cout, C = dgrad ? Cout : Cin;
  float v[32];
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int k = 32 * kb + j;
    float t = 0.f;
    if (o < O && k < KK * C) {
      const int tap = k / C, c = k % C;
      t = dgrad ? w[((size_t)c * Cin + o) * KK + (KK - 1 - tap)] : w[((size_t)o * Cin + c) * KK + tap];
    }
    v[j] = t;
    am = fmaxf(am, fabsf(t));
  }
  const int sh = mx_shift(am);
  const float mul = ldexpf(1.f, sh);
  unsigned word[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * q] * mul, v[4 * q + 1] * mul, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * q + 2] * mul, v[4 * q + 3] * mul, r, true);
    word[q] = (unsigned)r;
  }
  unsigned* dst = reinterpret_cast<unsigned*>(wq + (size_t)o * kpad + 32 * kb);
#pragma unroll
  for (int q = 0; q < 8; ++q) dst[q] = word[q];
  wsc[i] = (unsigned char)(127 - sh);
}

__global__ void mx_weight_layout_kernel(const float* __restrict__ w, unsigned char* __restrict__ wq,
                                        unsigned char* __restrict__ wsc, int Cout, int Cin, int KK,
                                        int dgrad, int rows, int kpad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows * (kpad / 32)) mx_weight_block(w, wq, wsc, Cout, Cin, KK, dgrad, kpad, i);
}

// several layouts in one launch (blockIdx.y = entry): a conv stack's per-step MX weights
constexpr int MXB_MAX = 16;
struct MXBatch {
  const float* w[MXB_MAX];
  unsigned char* wq[MXB_MAX];
  unsigned char* wsc[MXB_MAX];
  int cout[MXB_MAX], cin[MXB_MAX], kk[MXB_MAX], dgrad[MXB_MAX], n[MXB_MAX], kpad[MXB_MAX];
};

__global__ void mx_weight_layout_batch_kernel(MXBatch b) {
  const int e = blockIdx.y;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < b.n[e]; i += gridDim.x * blockDim.x)
    mx_weight_block(b.w[e], b.wq[e], b.wsc[e], b.cout[e], b.cin[e], b.kk[e], b.dgrad[e], b.kpad[e], i);
}

int mx_rows(int O) { return O > 32 ? (O + 63) / 64 * 64 : (O + 15) / 16 * 16; }
int mx_kpad(int C, int K) { return (K * K * C + 127) / 128 * 128; }

// ============================================================================ weight gradient
// dW[co][ci][kh][kw] = sum_{n, oy, ox} dY[n][oy][ox][co] X[n][oy+kh-p][ox+kw-p][ci] on the MX
// MFMA: M = output channels (A = dY^T), N = columns (tap, 16 input channels; for 8 input
// channels a PAIR of taps x 8 channels), K = output pixels, 128 per MFMA.  One persistent block
// per slab walks a contiguous range of strips (TR output rows of NSS samples) as wgrad_ws_kernel
// does; the strip's dY and X (+ halo) are staged as e4m3 with one power-of-two scale each (their
// max |.| into [128, 256)), pixel-major; both operands need 16-pixel runs of ONE channel per
// lane piece, which ds_read_b64_tr_b8 delivers (per 16-lane group: lane 2q+p addresses row q,
// bytes 8p..8p+7; lane i receives byte i of rows 0..7 -- measured, tools/probe/tr8_probe.hip):
// each piece is two transposed reads of 8 pixels.
template <int CIN_, int COUT_, int K_, int PAD_, int H_, int W_, int TR_, int NCW_, int OCC_,
          int NSS_, int DYS_, int XS_, int NTHR_ = 256, int NMW_ = 1, int PF_ = 2>
struct G8 {
  static constexpr int CIN = CIN_, COUT = COUT_, K = K_, PAD = PAD_, H = H_, W = W_;
  static constexpr int OCC = OCC_, PF = PF_, NTHR = NTHR_, WAVES = NTHR / 64;
  static constexpr int HO = H + 2 * PAD - K + 1, WO = W + 2 * PAD - K + 1;
  static constexpr int TR = TR_, SPS = HO / TR, NSS = NSS_;
  static constexpr int XR = TR + K - 1, XW = WO + K - 1;
  static constexpr int MT = COUT / 16, TAPS = K * K;
  static constexpr bool PAIR = CIN == 8;
  static constexpr int NCT = PAIR ? cdv(TAPS, 2) : TAPS * (CIN / 16);
  static constexpr int NMW = NMW_, MTW = MT / NMW, NCW = NCW_, NPW = WAVES / (NMW * NCW);
  static constexpr int NW = cdv(NCT, NCW);
  static constexpr int DYS = DYS_, XS = XS_;                 // LDS bytes per pixel
  static constexpr int SPIX = TR * WO, NPIX = NSS * SPIX, KST = cdv(NPIX, 128), DYP = KST * 128;
  static constexpr int DY_T = NSS * TR * WO * (COUT / 8), X_T = NSS * XR * XW * (CIN / 8);
  static constexpr int SLOTS = cdv(DY_T + X_T, NTHR);
  static constexpr int DY_BYTES = DYP * DYS, X_BYTES = NSS * XR * XW * XS;
  static constexpr int RED = NPW > 1 ? (NPW - 1) * NCW * NMW * MTW * NW * 64 : 0;   // f4
  static constexpr int PER_CO = CIN * TAPS;
  static constexpr int SMEM0 = DY_BYTES + X_BYTES;
  static constexpr int SMEM1 = RED * 16 > 16 * PER_CO * 4 ? RED * 16 : 16 * PER_CO * 4;
  static constexpr int SMEM = SMEM0 > SMEM1 ? SMEM0 : SMEM1;
  static_assert(HO % TR == 0 && (NSS == 1 || SPS == 1), "strips tile the map");
  static_assert(COUT % 16 == 0 && (CIN == 8 || CIN % 16 == 0), "channel tiles");
  static_assert(DYS % 8 == 0 && XS % 8 == 0 && DYS >= COUT && XS >= CIN, "strides");
  static_assert(WAVES % (NMW * NCW) == 0 && MT % NMW == 0, "wave split");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

typedef __attribute__((ext_vector_type(2))) int i2v;
__device__ __forceinline__ i2v tr8(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (__attribute__((address_space(3))) i2v*)(reinterpret_cast<uintptr_t>(p)));
}

template <class L>
__global__ __launch_bounds__(L::NTHR, L::OCC) void wgrad_ws8_kernel(const bf16* __restrict__ x,
                                                                const bf16* __restrict__ dy,
                                                                float* __restrict__ parts, int N,
                                                                int chunks) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[L::SMEM];
  __shared__ unsigned amx[2][L::WAVES];
  unsigned char* dys = smem;                   // [DYP][DYS]: strip pixel (s * TR + r) * WO + ox
  unsigned char* xs = smem + L::DY_BYTES;      // [NSS][XR][XW][XS]: X[y0 - PAD + r][c - PAD]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15, qr = r16 >> 1, p2 = r16 & 1;
  const int wm = wave % L::NMW, wc = (wave / L::NMW) % L::NCW, wp = wave / (L::NMW * L::NCW);

  const int ngrp = N / L::NSS;
  const int g0 = (int)(((long long)blockIdx.x * ngrp) / chunks);
  const int g1 = (int)(((long long)(blockIdx.x + 1) * ngrp) / chunks);
  const int st0 = g0 * L::SPS, st1 = g1 * L::SPS;

  // this lane's address part for column tile j: (tap of its 8-byte half, channel offset)
  int xo[L::NW];
  bool cv[L::NW];
#pragma unroll
  for (int j = 0; j < L::NW; ++j) {
    const int ct = wc * L::NW + j;
    int tap, ch;
    if constexpr (L::PAIR) { tap = 2 * ct + p2; ch = 0; }
    else { tap = ct / (L::CIN / 16); ch = 16 * (ct % (L::CIN / 16)) + 8 * p2; }
    cv[j] = ct < L::NCT;
    if (!cv[j] || tap >= L::TAPS) tap = 0;
    xo[j] = ((tap / L::K) * L::XW + tap % L::K) * L::XS + ch;
  }

  f4 acc[L::MTW][L::NW];
#pragma unroll
  for (int m = 0; m < L::MTW; ++m)
#pragma unroll
    for (int j = 0; j < L::NW; ++j) acc[m][j] = f4{0.f, 0.f, 0.f, 0.f};

  // the k-step tail of the dY image (pixels >= NPIX) stays zero for the whole launch
  for (int i = tid; i < (L::DYP - L::NPIX) * L::DYS / 8; i += L::NTHR)
    *reinterpret_cast<uint2*>(dys + (size_t)L::NPIX * L::DYS + 8 * i) = make_uint2(0u, 0u);

  struct Slot { int goff, loff, xrow; };   // xrow < 0: a dY task
  auto slot = [&](int i) -> Slot {
    const int task = tid + L::NTHR * i;
    if (task < L::DY_T) {
      constexpr int V = L::COUT / 8;
      const int q = task % V, pix = task / V;
      const int rs = pix / L::WO, ox = pix - rs * L::WO;
      const int sm = rs / L::TR, r = rs - sm * L::TR;
      return Slot{((sm * L::HO + r) * L::WO + ox) * L::COUT + 8 * q, pix * L::DYS + 8 * q, -1};
    }
    constexpr int V = L::CIN / 8;
    const int t = task - L::DY_T;
    const int q = t % V, pix = t / V;
    const int rs = pix / L::XW, c = pix - rs * L::XW;
    const int sm = rs / L::XR, r = rs - sm * L::XR;
    const int ix = c - L::PAD;
    return Slot{(task < L::DY_T + L::X_T && ix >= 0 && ix < L::W) ? ((sm * L::H + r) * L::W + ix) * L::CIN + 8 * q : -1,
                L::DY_BYTES + pix * L::XS + 8 * q, r};
  };
  u4 pre[L::SLOTS];
  auto load_strip = [&](int st) {
    const int sg = st / L::SPS, y0 = (st - sg * L::SPS) * L::TR;
    const int n = sg * L::NSS;
    const bf16* bdy = dy + ((size_t)n * L::HO + y0) * L::WO * L::COUT;
    const bf16* bx = x + ((long long)n * L::H + y0 - L::PAD) * L::W * L::CIN;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) {
      const Slot sl = slot(i);
      const void* src = &kZero8;
      if (tid + L::NTHR * i < L::DY_T) src = bdy + sl.goff;
      else if (sl.goff >= 0 && (unsigned)(y0 - L::PAD + sl.xrow) < (unsigned)L::H) src = bx + sl.goff;
      pre[i] = ldg16(src);
    }
  };

  if (st0 < st1) load_strip(st0);
  for (int st = st0; st < st1; ++st) {
    // the strip's max |dY| and max |X|: per wave, then through LDS
    unsigned md = 0u, mx = 0u;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) {
      if (tid + L::NTHR * i < L::DY_T) md = absmax_bf16x8(pre[i], md);
      else mx = absmax_bf16x8(pre[i], mx);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      md = max(md, (unsigned)__shfl_xor((int)md, o, 64));
      mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if (lane == 0) { amx[0][wave] = md; amx[1][wave] = mx; }
    __syncthreads();   // every wave is done with the previous strip; amx complete
    md = amx[0][0];
    mx = amx[1][0];
#pragma unroll
    for (int w = 1; w < L::WAVES; ++w) { md = max(md, amx[0][w]); mx = max(mx, amx[1][w]); }
    const int shd = mx_shift(__uint_as_float(md << 16)), shx = mx_shift(__uint_as_float(mx << 16));
    const float muld = ldexpf(1.f, shd), mulx = ldexpf(1.f, shx);
    const int sbd = 127 - shd, sbx = 127 - shx;
#pragma unroll
    for (int i = 0; i < L::SLOTS; ++i) {
      const int task = tid + L::NTHR * i;
      if (task < L::DY_T + L::X_T)
        *reinterpret_cast<uint2*>(smem + slot(i).loff) = q8(pre[i], task < L::DY_T ? muld : mulx);
    }
    __syncthreads();
    if (st + 1 < st1) load_strip(st + 1);

    for (int ks = wp; ks < L::KST; ks += L::NPW) {
      // this lane's 4 rows (pixels) of the k-step: piece pc, transposed read h, row q8
      int xb[2][2];
      i8v a[L::MTW];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int P = 128 * ks + 64 * pc + 16 * g + 8 * h + qr;
          const int Pc = min(P, L::NPIX - 1);                 // tail pixels: dY is 0 there
          const int sm = Pc / L::SPIX, rem = Pc - sm * L::SPIX;
          const int r = rem / L::WO, ox = rem - r * L::WO;
          xb[pc][h] = ((sm * L::XR + r) * L::XW + ox) * L::XS;
#pragma unroll
          for (int m = 0; m < L::MTW; ++m) {
            const i2v v = tr8(dys + P * L::DYS + 16 * (wm * L::MTW + m) + 8 * p2);
            a[m][4 * pc + 2 * h] = v.x;
            a[m][4 * pc + 2 * h + 1] = v.y;
          }
        }
      constexpr int PF = L::PF;
      i8v bq[PF + 1];
      auto ldb = [&](i8v& d, int j) {
#pragma unroll
        for (int pc = 0; pc < 2; ++pc)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const i2v v = tr8(xs + xb[pc][h] + xo[j]);
            d[4 * pc + 2 * h] = v.x;
            d[4 * pc + 2 * h + 1] = v.y;
          }
      };
#pragma unroll
      for (int j = 0; j < PF && j < L::NW; ++j) ldb(bq[j], j);
#pragma unroll
      for (int j = 0; j < L::NW; ++j) {
        if (j + PF < L::NW) ldb(bq[(j + PF) % (PF + 1)], j + PF);
#pragma unroll
        for (int m = 0; m < L::MTW; ++m)
          acc[m][j] = mxmma_<0>(a[m], bq[j % (PF + 1)], acc[m][j], sbd, sbx);
      }
    }
  }

  // pixel-split partials -> wave wp = 0 (fixed order), then the slab write (as wgrad_ws_kernel)
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
  float* tb = reinterpret_cast<float*>(smem);
  float* out = parts + (size_t)blockIdx.x * L::COUT * L::PER_CO;
  for (int mt = 0; mt < L::MT; ++mt) {
    __syncthreads();
    if (wp == 0) {
#pragma unroll
      for (int m = 0; m < L::MTW; ++m) {
        if (wm * L::MTW + m != mt) continue;
#pragma unroll
        for (int j = 0; j < L::NW; ++j) {
          if (!cv[j]) continue;
          const int ct = wc * L::NW + j;
          int tap, ci;
          if constexpr (L::PAIR) { tap = 2 * ct + (r16 >> 3); ci = r16 & 7; }
          else { tap = ct / (L::CIN / 16); ci = 16 * (ct % (L::CIN / 16)) + r16; }
          if (tap >= L::TAPS) continue;
#pragma unroll
          for (int i = 0; i < 4; ++i) tb[(4 * g + i) * L::PER_CO + ci * L::TAPS + tap] = acc[m][j][i];
        }
      }
    }
    __syncthreads();
    float4* o4 = reinterpret_cast<float4*>(out + (size_t)mt * 16 * L::PER_CO);
    const float4* t4 = reinterpret_cast<const float4*>(tb);
    for (int e = tid; e < 16 * L::PER_CO / 4; e += L::NTHR) o4[e] = t4[e];
  }
}

//          CIN COUT K PAD  H   W  TR NCW OCC NSS DYS XS
typedef G8<8, 16, 5, 2, 56, 56, 8, 1, 2, 1, 16, 8> G8A2;     // audio conv2
typedef G8<16, 32, 5, 2, 28, 28, 14, 4, 2, 1, 32, 16> G8A3;  // audio conv3
typedef G8<32, 64, 5, 2, 14, 14, 7, 4, 1, 1, 64, 32, 512, 2, 1> G8A4;   // audio conv4
typedef G8<32, 64, 5, 0, 14, 14, 10, 4, 1, 1, 64, 32, 512, 2, 1> G8I2;  // image conv2

template <class L>
bool g8_is(int Cin, int H, int Cout, int K, int pad) {
  return Cin == L::CIN && Cout == L::COUT && K == L::K && pad == L::PAD && H == L::H;
}

template <class L>
int g8_chunks(int N) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, wgrad_ws8_kernel<L>, L::NTHR, 0) != hipSuccess || occ <= 0)
      occ = 1;
  }
  // one resident wave of blocks, one slab each (every slab is a [Cout][Cin][K][K] f32 partial the
  // fixed-order reduce reads back)
  return std::max(1, grid_cap(std::min(N / L::NSS, num_cus8() * occ)));
}

}  // namespace

extern "C" {

// slabs of avd_mx_conv_wgrad for the conv Cin -> Cout over H x H (0: not served)
int avd_mx_wgrad_chunks(int N, int Cin, int H, int Cout, int K, int pad) {
#define AVD_G8(LL) if (g8_is<LL>(Cin, H, Cout, K, pad)) return N % LL::NSS ? 0 : g8_chunks<LL>(N);
  AVD_G8(G8A2) AVD_G8(G8A3) AVD_G8(G8A4) AVD_G8(G8I2)
#undef AVD_G8
  return 0;
}

// per-slab weight gradients parts [chunks][Cout][Cin][K][K] (sum them: avd_sum_rows)
int avd_mx_conv_wgrad(const void* x, const void* dy, float* parts, int N, int Cin, int H, int W,
                      int Cout, int K, int pad, void* stream) {
  if (!x || !dy || !parts) return AVD_ERR_ARG;
  if (H != W) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
#define AVD_G8(LL)                                                                               \
  if (g8_is<LL>(Cin, H, Cout, K, pad)) {                                                        \
    if (N % LL::NSS) return AVD_ERR_SHAPE;                                                      \
    const int chunks = g8_chunks<LL>(N);                                                        \
    wgrad_ws8_kernel<LL><<<chunks, LL::NTHR, 0, st>>>((const bf16*)x, (const bf16*)dy, parts, N, chunks); \
    AVD_CHECK_LAUNCH();                                                                         \
    return AVD_OK;                                                                              \
  }
  AVD_G8(G8A2) AVD_G8(G8A3) AVD_G8(G8A4) AVD_G8(G8I2)
#undef AVD_G8
  return AVD_ERR_SHAPE;
}



long long avd_mx_weight_bytes(int Cout, int Cin, int K, int dgrad) {
  const int O = dgrad ? Cin : Cout, C = dgrad ? Cout : Cin;
  return (long long)mx_rows(O) * mx_kpad(C, K);
}

long long avd_mx_scale_bytes(int Cout, int Cin, int K, int dgrad) {
  return avd_mx_weight_bytes(Cout, Cin, K, dgrad) / 32;
}

int avd_mx_weight_layout(const float* w, void* wq, void* wsc, int Cout, int Cin, int K, int dgrad,
                         void* stream) {
  if (!w || !wq || !wsc) return AVD_ERR_ARG;
  if (Cout <= 0 || Cin <= 0 || K <= 0) return AVD_ERR_SHAPE;
  const int O = dgrad ? Cin : Cout, C = dgrad ? Cout : Cin;
  const int rows = mx_rows(O), kpad = mx_kpad(C, K);
  const int n = rows * (kpad / 32);
  mx_weight_layout_kernel<<<avd_cdiv(n, 128), 128, 0, avd_stream(stream)>>>(
      w, (unsigned char*)wq, (unsigned char*)wsc, Cout, Cin, K * K, dgrad ? 1 : 0, rows, kpad);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// n layouts (<= 16) in one launch: the arguments of avd_mx_weight_layout as arrays
int avd_mx_weight_layout_batch(int n, const float* const* w, void* const* wq, void* const* wsc,
                               const int* cout, const int* cin, const int* k, const int* dgrad,
                               void* stream) {
  if (n <= 0 || n > MXB_MAX) return AVD_ERR_ARG;
  MXBatch b{};
  int most = 1;
  for (int e = 0; e < n; ++e) {
    if (!w[e] || !wq[e] || !wsc[e]) return AVD_ERR_ARG;
    if (cout[e] <= 0 || cin[e] <= 0 || k[e] <= 0) return AVD_ERR_SHAPE;
    const int O = dgrad[e] ? cin[e] : cout[e], C = dgrad[e] ? cout[e] : cin[e];
    b.w[e] = w[e];
    b.wq[e] = (unsigned char*)wq[e];
    b.wsc[e] = (unsigned char*)wsc[e];
    b.cout[e] = cout[e]; b.cin[e] = cin[e]; b.kk[e] = k[e] * k[e]; b.dgrad[e] = dgrad[e] ? 1 : 0;
    b.kpad[e] = mx_kpad(C, k[e]);
    b.n[e] = mx_rows(O) * (b.kpad[e] / 32);
    most = std::max(most, b.n[e]);
  }
  mx_weight_layout_batch_kernel<<<dim3(avd_cdiv(most, 128), n), 128, 0, avd_stream(stream)>>>(b);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// 1 if the forward (dgrad = 0) or input gradient (dgrad = 1) of the conv Cin -> Cout over an
// H x W input has an MX kernel
int avd_mx_conv_serves(int Cin, int H, int W, int Cout, int K, int pad, int dgrad) {
  if (!dgrad)
    return is8<F8A2>(Cin, H, W, Cout, K, pad) || is8<F8A3>(Cin, H, W, Cout, K, pad) ||
           is8<F8A4>(Cin, H, W, Cout, K, pad) || is8<F8I2>(Cin, H, W, Cout, K, pad);
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1, dp = K - 1 - pad;
  return is8<D8A2>(Cout, Ho, Wo, Cin, K, dp) || is8<D8A3>(Cout, Ho, Wo, Cin, K, dp) ||
         is8<D8A4>(Cout, Ho, Wo, Cin, K, dp) || is8<D8I2>(Cout, Ho, Wo, Cin, K, dp);
}

// samples per strip (NS) of the MX kernel serving the forward (dgrad = 0) or input gradient
// (dgrad = 1) of the conv Cin -> Cout over H x W (0: not served); the launch needs N % NS == 0,
// and a forward that writes BN partials also B % NS == 0
int avd_mx_conv_ns(int Cin, int H, int W, int Cout, int K, int pad, int dgrad) {
  if (!dgrad) {
    if (is8<F8A2>(Cin, H, W, Cout, K, pad)) return F8A2::NS;
    if (is8<F8A3>(Cin, H, W, Cout, K, pad)) return F8A3::NS;
    if (is8<F8A4>(Cin, H, W, Cout, K, pad)) return F8A4::NS;
    if (is8<F8I2>(Cin, H, W, Cout, K, pad)) return F8I2::NS;
    return 0;
  }
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1, dp = K - 1 - pad;
  if (is8<D8A2>(Cout, Ho, Wo, Cin, K, dp)) return D8A2::NS;
  if (is8<D8A3>(Cout, Ho, Wo, Cin, K, dp)) return D8A3::NS;
  if (is8<D8A4>(Cout, Ho, Wo, Cin, K, dp)) return D8A4::NS;
  if (is8<D8I2>(Cout, Ho, Wo, Cin, K, dp)) return D8I2::NS;
  return 0;
}

// BN partial rows per group written by avd_mx_conv_fwd (0: not served)
int avd_mx_stat_rows(int H, int W, int B, int K, int Cin, int Cout, int pad) {
  auto rows = [&](auto l) -> int {
    typedef decltype(l) L;
    return B % L::NS ? 0 : stat_grid8<L>() * L::NPW;
  };
  if (is8<F8A2>(Cin, H, W, Cout, K, pad)) return rows(F8A2{});
  if (is8<F8A3>(Cin, H, W, Cout, K, pad)) return rows(F8A3{});
  if (is8<F8A4>(Cin, H, W, Cout, K, pad)) return rows(F8A4{});
  if (is8<F8I2>(Cin, H, W, Cout, K, pad)) return rows(F8I2{});
  return 0;
}

int avd_mx_conv_fwd(const void* x, const void* wq, const void* wsc, const float* bias,
                    const float* pivot, void* y, float* stats, int N, int B, int Cin, int H, int W,
                    int Cout, int K, int pad, void* stream) {
  if (!x || !wq || !wsc || !y) return AVD_ERR_ARG;
  hipStream_t st = avd_stream(stream);
#define AVD_F8(LL) \
  if (is8<LL>(Cin, H, W, Cout, K, pad)) return launch8<LL, true>(x, wq, wsc, bias, y, stats, N, B, st, pivot);
  AVD_F8(F8A2) AVD_F8(F8A3) AVD_F8(F8A4) AVD_F8(F8I2)
#undef AVD_F8
  return AVD_ERR_SHAPE;
}

int avd_mx_conv_dgrad(const void* dy, const void* wq_d, const void* wsc_d, void* dx, int N, int Cin,
                      int H, int W, int Cout, int K, int pad, void* stream) {
  if (!dy || !wq_d || !wsc_d || !dx) return AVD_ERR_ARG;
  hipStream_t st = avd_stream(stream);
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1, dp = K - 1 - pad;
#define AVD_D8(LL) \
  if (is8<LL>(Cout, Ho, Wo, Cin, K, dp)) return launch8<LL, false>(dy, wq_d, wsc_d, nullptr, dx, nullptr, N, N, st, nullptr);
  AVD_D8(D8A2) AVD_D8(D8A3) AVD_D8(D8A4) AVD_D8(D8I2)
#undef AVD_D8
  return AVD_ERR_SHAPE;
}

}  // extern "C"
