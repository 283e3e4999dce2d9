// fp8 (OCP e4m3fn) MFMA forward convolution for the mid-layer convs of the CentralNet / 3x3
// encoders (BASELINE config 5, "fp8 MFMA conv path").  Inputs stay bf16 in
// HBM (the BatchNorm / pooling chain and the backward read them); the kernel quantises while
// staging, so only the MFMA operands are fp8:
//   * x:  per-tensor scale sx (post-BN/ReLU/pool maps are O(1); the caller passes 1 by default),
//         q = e4m3(clamp(x / sx, +-448)), round to nearest even (v_cvt_pk_fp8_f32);
//   * W:  per-output-channel scale sw[o] = max|W[o]| / 448 (avd_fp8_weight_quant), tap-major
//         rows [O][KP] with K index tap * C + c, zero-padded to KP = 32 * ceil(K*K*C / 32);
//   * y = bf16(acc * sx * sw[o] + bias[o]) NHWC, + BatchNorm partial sums of the stored values.
// The backward (dgrad / wgrad) stays bf16 on the stored bf16 maps: fp8 forward, bf16 backward.
//
// Implicit GEMM on v_mfma_f32_16x16x32_fp8_fp8 (8 fp8 per lane per operand, the bf16 16x16x32
// layout): A = weights [16 out channels][32 k], B = input [32 k][16 output pixels]; a lane's k
// run 8g..8g+7 is 8 consecutive channels of one tap (C % 8 == 0), one ds_read_b64 from the
// staged tile + halo.  The block owns a tile of <= GPW*64 output pixels x all O channels;
// input tile and the fp8 weight rows sit in LDS for the whole tile.
#include <algorithm>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

__device__ const u4 kZero8 = {0u, 0u, 0u, 0u};
constexpr float kE4M3Max = 448.f;

__device__ __forceinline__ float clampq(float v) { return fminf(fmaxf(v, -kE4M3Max), kE4M3Max); }

// 8 bf16 (one u4) * inv -> 8 e4m3 bytes (two dwords, element 0 in the low byte)
__device__ __forceinline__ uint2 q8(u4 v, float inv) {
  float f[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = clampq(__uint_as_float(v[i] << 16) * inv);
    f[2 * i + 1] = clampq(__uint_as_float(v[i] & 0xffff0000u) * inv);
  }
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}

__device__ __forceinline__ int fdiv_i(int a, int b, float rb) {
  int q = (int)((float)a * rb);
  const int r = a - q * b;
  return q + (r >= b) - (r < 0);
}

template <int C, int NT, int K, int GPW>
__global__ __launch_bounds__(256, 2) void conv8_kernel(
    const bf16* __restrict__ x, float xscale, const unsigned char* __restrict__ wq,
    const float* __restrict__ wscale, const float* __restrict__ bias, bf16* __restrict__ y,
    float* __restrict__ stats, int N, int H, int W, int pad, int TR, int NS, int tilesPS,
    int nrows) {
  constexpr int O = NT * 16;
  constexpr int KK = K * K * C, KP = (KK + 31) / 32 * 32, KS = KP / 32;
  constexpr int PSB = C + 8;                 // LDS bytes per staged pixel
  constexpr int KPS = KP + 8;                // LDS bytes per weight row
  extern __shared__ __attribute__((aligned(16))) unsigned char smem8[];
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  const int IW = Wo + K - 1, IR = TR + K - 1;
  const int npix = NS * IR * IW;
  unsigned char* xs = smem8;                             // [npix][PSB]
  unsigned char* ws = smem8 + ((npix * PSB + 15) & ~15); // [O][KPS]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int TRW = TR * Wo, TP = NS * TRW;
  const float rIW = 1.f / IW, rIR = 1.f / IR, rWo = 1.f / Wo, rTRW = 1.f / TRW;
  const int ntiles = (N / NS) * tilesPS;

  // ---- the weight rows (fp8 bytes, 16 per task) stay in LDS for all of the block's tiles
  for (int t = tid; t < O * (KP / 16); t += 256) {
    const int o = t / (KP / 16), q = t - o * (KP / 16);
    *reinterpret_cast<u4*>(ws + o * KPS + 16 * q) =
        *reinterpret_cast<const u4*>(wq + (size_t)o * KP + 16 * q);
  }
  const float inv = 1.f / xscale;
  constexpr int VPP = C / 8;                 // 16-byte bf16 loads per pixel
  const int ntask = npix * VPP;
  constexpr int U = 4;
  auto stage = [&](int n0, int y0) {         // the quantised input tile + halo
    for (int b0 = tid; b0 < ntask; b0 += 256 * U) {
      u4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = b0 + 256 * u;
        const int pix = t / VPP, q = t - pix * VPP;
        const int row = fdiv_i(pix, IW, rIW), col = pix - row * IW;
        const int s = fdiv_i(row, IR, rIR), iy = y0 + row - s * IR - pad, ix = col - pad;
        const int n = n0 + s;
        const bool ok = t < ntask && n < N && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        v[u] = ldg16(ok ? (const void*)(x + (((size_t)n * H + iy) * W + ix) * C + 8 * q)
                        : (const void*)&kZero8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = b0 + 256 * u;
        if (t < ntask) {
          const int pix = t / VPP, q = t - pix * VPP;
          *reinterpret_cast<uint2*>(xs + pix * PSB + 8 * q) = q8(v[u], inv);
        }
      }
    }
  };

  // ---- lane geometry: pixel bases, per-k-step tap offsets
  int base[GPW];
  bool pv[GPW];
  int gp[GPW], prow[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int p = (wave + 4 * j) * 16 + r16;
    const int s = fdiv_i(p, TRW, rTRW), rem = p - s * TRW;
    const int r = fdiv_i(rem, Wo, rWo), xx = rem - r * Wo;
    pv[j] = p < TP;
    prow[j] = r;
    base[j] = pv[j] ? ((s * IR + r) * IW + xx) * PSB : 0;
    gp[j] = (s * Ho + r) * Wo + xx;            // + the tile's (n0, y0) offset
  }
  int toff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 32 * ks + 8 * g;
    int tap = k / C;
    const int c0 = k - tap * C;
    if (tap >= K * K) tap = 0;               // zero weights there
    toff[ks] = ((tap / K) * IW + tap % K) * PSB + c0;
  }
  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  for (int ti = t0; ti < t1; ++ti) {
    const int sg = ti / tilesPS, tt = ti - sg * tilesPS;
    const int n0 = sg * NS, y0 = tt * TR;
    const size_t tb = ((size_t)n0 * Ho + y0) * Wo;
    __syncthreads();                           // the previous tile's reads are done
    stage(n0, y0);
    __syncthreads();
    f4 acc[GPW][NT];
#pragma unroll
    for (int j = 0; j < GPW; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      long a[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        a[t] = *reinterpret_cast<const long*>(ws + (16 * t + r16) * KPS + 32 * ks + 8 * g);
#pragma unroll
      for (int j = 0; j < GPW; ++j) {
        const long bv = *reinterpret_cast<const long*>(xs + base[j] + toff[ks]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a[t], bv, acc[j][t], 0, 0, 0);
      }
    }

    // ---- epilogue: dequantise, bias, bf16 rounding, NHWC store, BN partial sums
    float sc[NT][4], bb[NT][4], ss[NT][4], sq[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = 16 * t + 4 * g + i;
        sc[t][i] = xscale * wscale[co];
        bb[t][i] = bias ? bias[co] : 0.f;
        ss[t][i] = 0.f;
        sq[t][i] = 0.f;
      }
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      if (!pv[j] || y0 + prow[j] >= Ho) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int co = 16 * t + 4 * g;
        const uint32_t lo = pack_bf16x2(fmaf(acc[j][t][0], sc[t][0], bb[t][0]),
                                        fmaf(acc[j][t][1], sc[t][1], bb[t][1]));
        const uint32_t hi = pack_bf16x2(fmaf(acc[j][t][2], sc[t][2], bb[t][2]),
                                        fmaf(acc[j][t][3], sc[t][3], bb[t][3]));
        const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                            __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ss[t][i] += v[i];
          sq[t][i] = fmaf(v[i], v[i], sq[t][i]);
        }
        *reinterpret_cast<uint2*>(y + ((size_t)gp[j] + tb) * O + co) = make_uint2(lo, hi);
      }
    }
    if (!stats) continue;
    const int row = ti * 4 + wave;             // one partial row per (tile, wave)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = row16_sum(ss[t][i]), q = row16_sum(sq[t][i]);
        if (r16 == 0)
          *reinterpret_cast<float2*>(stats + ((size_t)(16 * t + 4 * g + i) * nrows + row) * 2) =
              make_float2(a, q);
      }
  }
}

// W [O][C][K][K] f32 -> e4m3 rows [O][KP] (k = tap * C + c, zero pad) and sw[o] = max|W[o]|/448
__global__ __launch_bounds__(256) void fp8_wquant_kernel(const float* __restrict__ w, int C, int K,
                                                         int KP, unsigned char* __restrict__ wq,
                                                         float* __restrict__ ws) {
  __shared__ float red[4];
  const int o = blockIdx.x, KK = C * K * K;
  const float* wo = w + (size_t)o * KK;
  float m = 0.f;
  for (int i = threadIdx.x; i < KK; i += 256) m = fmaxf(m, fabsf(wo[i]));
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = m > 0.f ? __fdiv_rn(m, kE4M3Max) : 1.f;   // correctly rounded, as torch
  if (threadIdx.x == 0) ws[o] = s;
  for (int k = threadIdx.x; k < KP; k += 256) {
    float v = 0.f;
    if (k < KK) {
      const int tap = k / C, c = k - tap * C;
      v = clampq(__fdiv_rn(wo[(size_t)c * K * K + tap], s));
    }
    wq[(size_t)o * KP + k] = (unsigned char)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
  }
}

struct Plan8 { int TR, NS, GPW, tilesPS; };

int num_cus8() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// tile: best utilisation of GPW*64 pixel slots, NS | B, LDS (input + weights) <= 60 KB
template <int C, int NT, int K>
Plan8 plan8(int Ho, int Wo, int B) {
  constexpr int KP = (K * K * C + 31) / 32 * 32;
  const size_t wbytes = (size_t)NT * 16 * (KP + 8);
  Plan8 best{0, 0, 0, 0};
  double bu = -1;
  for (int gpw : {4, 7}) {
    const int cap = gpw * 64;
    auto consider = [&](int TR, int NS) {
      if (TR <= 0 || NS <= 0 || TR * Wo * NS > cap) return;
      const size_t xb = (size_t)NS * (TR + K - 1) * (Wo + K - 1) * (C + 8);
      if (((xb + 15) & ~(size_t)15) + wbytes > 60 * 1024) return;
      const int tps = avd_cdiv(Ho, TR);
      const double u = (double)Ho * Wo * NS / ((double)tps * cap);
      if (u > bu + 1e-9 || (u > bu - 1e-9 && TR * NS > best.TR * best.NS)) {
        bu = u;
        best = Plan8{TR, NS, gpw, tps};
      }
    };
    if (Ho * Wo <= cap)
      for (int ns = cap / (Ho * Wo); ns >= 1; --ns)
        if (B % ns == 0) consider(Ho, ns);
    for (int tr = 1; tr <= Ho && tr * Wo <= cap; ++tr) consider(tr, 1);
  }
  return best;
}

template <int C, int NT, int K>
int launch8(const void* x, float xs, const void* wq, const float* wsc, const float* bias, void* y,
            float* stats, int N, int B, int H, int W, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  const Plan8 p = plan8<C, NT, K>(Ho, Wo, B);
  if (!p.NS || N % p.NS || B % p.NS) return AVD_ERR_SHAPE;
  constexpr int KP = (K * K * C + 31) / 32 * 32;
  const size_t xb = (size_t)p.NS * (p.TR + K - 1) * (Wo + K - 1) * (C + 8);
  const size_t lds = ((xb + 15) & ~(size_t)15) + (size_t)NT * 16 * (KP + 8);
  const int tiles = (N / p.NS) * p.tilesPS;
  const int grid = grid_cap(std::min(tiles, 3 * num_cus8()));
#define AVD_G(G)                                                                                 \
  if (p.GPW == G)                                                                                \
    conv8_kernel<C, NT, K, G><<<grid, 256, lds, st>>>((const bf16*)x, xs, (const unsigned char*)wq, \
                                                       wsc, bias, (bf16*)y, stats, N, H, W, pad,  \
                                                       p.TR, p.NS, p.tilesPS, tiles * 4);
  AVD_G(4) else AVD_G(7) else return AVD_ERR_SHAPE;
#undef AVD_G
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

template <int C, int NT, int K>
int rows8(int Ho, int Wo, int B) {
  const Plan8 p = plan8<C, NT, K>(Ho, Wo, B);
  return p.NS ? (B / p.NS) * p.tilesPS * 4 : 0;
}

// the served (C, O, K) set: the CentralNet mid layers and the 3x3 encoders' layers
#define AVD_FP8_SHAPES(X)                                                                        \
  X(8, 1, 5) X(16, 2, 5) X(32, 4, 5) X(8, 2, 5) X(16, 4, 5) X(32, 2, 3) X(32, 4, 3) X(64, 4, 3)  \
  X(16, 1, 5) X(32, 2, 5)

}  // namespace

extern "C" {

int avd_fp8_weight_elems(int Cout, int Cin, int K) {
  return Cout * ((K * K * Cin + 31) / 32 * 32);
}

int avd_fp8_weight_quant(const float* w, int Cout, int Cin, int K, void* wq, float* wscale,
                         void* stream) {
  if (!w || !wq || !wscale) return AVD_ERR_ARG;
  if (Cout <= 0 || Cin <= 0 || K <= 0) return AVD_ERR_SHAPE;
  const int KP = (K * K * Cin + 31) / 32 * 32;
  fp8_wquant_kernel<<<Cout, 256, 0, avd_stream(stream)>>>(w, Cin, K, KP, (unsigned char*)wq, wscale);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_fp8_conv_serves(int Cin, int Cout, int K) {
#define AVD_S(C_, NT_, K_) if (Cin == C_ && Cout == 16 * NT_ && K == K_) return 1;
  AVD_FP8_SHAPES(AVD_S)
#undef AVD_S
  return 0;
}

int avd_fp8_stat_rows(int Ho, int Wo, int B, int K, int Cin, int Cout) {
#define AVD_R(C_, NT_, K_) if (Cin == C_ && Cout == 16 * NT_ && K == K_) return rows8<C_, NT_, K_>(Ho, Wo, B);
  AVD_FP8_SHAPES(AVD_R)
#undef AVD_R
  return 0;
}

int avd_fp8_conv_fwd(const void* x, float xscale, const void* wq, const float* wscale,
                     const float* bias, void* y, float* stats, int N, int B, int Cin, int H,
                     int W, int Cout, int K, int pad, void* stream) {
  if (!x || !wq || !wscale || !y) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || N % B || !(xscale > 0.f)) return AVD_ERR_SHAPE;
  if (H + 2 * pad < K || W + 2 * pad < K) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
#define AVD_F(C_, NT_, K_)                                                                     \
  if (Cin == C_ && Cout == 16 * NT_ && K == K_)                                                \
    return launch8<C_, NT_, K_>(x, xscale, wq, wscale, bias, y, stats, N, B, H, W, pad, st);
  AVD_FP8_SHAPES(AVD_F)
#undef AVD_F
  return AVD_ERR_SHAPE;
}

}  // extern "C"
