// Convolution kernels of the conv -> BN -> ReLU -> maxpool2 blocks (CentralNet LeNets,
// reference models/unimodal.py:105-221; 3x3 CNNs, models/dino.py:18-73).
//
// v1 design (direct convolution, fp32 accumulate, activations f32 or bf16 in HBM):
//  * forward / input-grad: one workgroup = 16x16 output pixels of one sample x CO output
//    channels.  The input tile (+halo) for a chunk of input channels is staged in LDS; the
//    weights are pre-laid-out as [cin][tap][cout] so that, for a tap, the CO weights the
//    whole workgroup needs are contiguous and wave-uniform -> they arrive through the
//    scalar unit (s_load_dwordx16) and feed v_fma_f32 as SGPR operands: one LDS read per
//    CO FMAs.  The forward epilogue emits per-(sample, tile, channel) partial BN sums of the
//    stored (rounded) value, so BatchNorm statistics cost no extra pass over y.
//  * weight-grad: split over sample chunks (deterministic partial slabs, reduced by
//    avd_sum_rows); per chunk the X rows and dY rows of a row-tile sit in LDS and each thread
//    owns (cin, tap) entries x 8 output channels.
#include "common.h"

using namespace avd;

namespace {

constexpr int TS = 16;   // output tile edge
constexpr int CIC = 8;   // input channels staged per LDS pass

template <typename TI, typename TO, int K, int CO, bool STATS>
__global__ __launch_bounds__(256) void conv_direct_kernel(
    const TI* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ bias,
    TO* __restrict__ y, float* __restrict__ stats, int Cin, int H, int W, int Cout, int Ho,
    int Wo, int pad, int tilesX, int tiles) {
  constexpr int IT = TS + K - 1;
  __shared__ float xs[CIC][IT][IT + 1];
  __shared__ float red[4][2 * CO];
  const int n = blockIdx.y;
  const int tile = blockIdx.x;
  const int co0 = blockIdx.z * CO;
  const int ty0 = (tile / tilesX) * TS, tx0 = (tile % tilesX) * TS;
  const int tid = threadIdx.x;
  const int ly = tid / TS, lx = tid % TS;
  const int oy = ty0 + ly, ox = tx0 + lx;
  const bool valid = (oy < Ho) && (ox < Wo);

  float acc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) acc[c] = 0.f;

  const size_t xbase = (size_t)n * Cin * H * W;
  for (int ci0 = 0; ci0 < Cin; ci0 += CIC) {
    const int nc = min(CIC, Cin - ci0);
    __syncthreads();
    for (int i = tid; i < nc * IT * IT; i += 256) {
      const int c = i / (IT * IT), r = (i / IT) % IT, q = i % IT;
      const int iy = ty0 - pad + r, ix = tx0 - pad + q;
      float v = 0.f;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W)
        v = io<TI>::ld(x, xbase + (size_t)(ci0 + c) * H * W + (size_t)iy * W + ix);
      xs[c][r][q] = v;
    }
    __syncthreads();
    for (int c = 0; c < nc; ++c) {
      const float* wc = wt + ((size_t)(ci0 + c) * K * K) * Cout + co0;  // [tap][cout]
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          const float xv = xs[c][ly + kh][lx + kw];
          const float* wk = wc + (kh * K + kw) * Cout;
#pragma unroll
          for (int o = 0; o < CO; ++o) acc[o] = fmaf(xv, wk[o], acc[o]);
        }
      }
    }
  }

  // epilogue: bias, store, BN partial statistics of the stored value
  const size_t ybase = (size_t)n * Cout * Ho * Wo + (size_t)oy * Wo + ox;
  const int w = tid >> 6, l = tid & 63;
#pragma unroll
  for (int o = 0; o < CO; ++o) {
    float v = acc[o] + (bias ? bias[co0 + o] : 0.f);
    v = io<TO>::rnd(v);
    if (valid) io<TO>::st(y, ybase + (size_t)(co0 + o) * Ho * Wo, v);
    if (STATS) {
      float s = valid ? v : 0.f, q = s * s;
      s = wave_sum(s);
      q = wave_sum(q);
      if (l == 0) { red[w][2 * o] = s; red[w][2 * o + 1] = q; }
    }
  }
  if (STATS) {
    __syncthreads();
    if (tid < 2 * CO) {  // channel-major partials: stats[co][n][tile][2]
      const float r = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      const int o = tid >> 1, k = tid & 1;
      stats[(((size_t)(co0 + o) * gridDim.y + n) * tiles + tile) * 2 + k] = r;
    }
  }
}

// wt[ci][t][co] = w[co][ci][t]            (mode 0, forward)
// wt[co][t][ci] = w[co][ci][K*K-1-t]      (mode 1, input-grad = conv with flipped taps)
__global__ void weight_layout_kernel(const float* __restrict__ w, float* __restrict__ wt, int Cout,
                                     int Cin, int KK, int mode) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Cout * Cin * KK) return;
  const int co = i / (Cin * KK), ci = (i / KK) % Cin, t = i % KK;
  const float v = w[i];
  if (mode == 0) wt[((size_t)ci * KK + t) * Cout + co] = v;
  else wt[((size_t)co * KK + (KK - 1 - t)) * Cin + ci] = v;
}

template <typename TI, typename TO, int K, int CO, bool STATS>
int launch_direct(const void* x, const float* wt, const float* bias, void* y, float* stats,
                  int N, int Cin, int H, int W, int Cout, int Ho, int Wo, int pad, hipStream_t st) {
  const int tilesX = avd_cdiv(Wo, TS), tilesY = avd_cdiv(Ho, TS);
  dim3 grid(tilesX * tilesY, N, Cout / CO);
  conv_direct_kernel<TI, TO, K, CO, STATS><<<grid, 256, 0, st>>>(
      (const TI*)x, wt, bias, (TO*)y, stats, Cin, H, W, Cout, Ho, Wo, pad, tilesX,
      tilesX * tilesY);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

template <typename TI, typename TO, bool STATS>
int dispatch_direct(const void* x, const float* wt, const float* bias, void* y, float* stats,
                    int N, int Cin, int H, int W, int Cout, int K, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  int co = Cout % 64 == 0 ? 64 : Cout % 32 == 0 ? 32 : Cout % 16 == 0 ? 16 : Cout % 8 == 0 ? 8 : 0;
  if (co == 0) return AVD_ERR_SHAPE;
#define AVD_DD(KK, CC)                                                                          \
  if (K == KK && co == CC)                                                                      \
    return launch_direct<TI, TO, KK, CC, STATS>(x, wt, bias, y, stats, N, Cin, H, W, Cout, Ho,  \
                                                 Wo, pad, st);
  AVD_DD(5, 8) AVD_DD(5, 16) AVD_DD(5, 32) AVD_DD(5, 64)
  AVD_DD(3, 8) AVD_DD(3, 16) AVD_DD(3, 32) AVD_DD(3, 64)
#undef AVD_DD
  return AVD_ERR_SHAPE;
}

// ----------------------------------------------------------------------------- weight grad
constexpr int WG_COB = 8;
constexpr int WG_JMAX = 5;

template <typename TX, typename TD, int K>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(
    const TX* __restrict__ x, const TD* __restrict__ dy, float* __restrict__ dw_parts, int N,
    int Cin, int H, int W, int Cout, int Ho, int Wo, int pad, int spc, int TR) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Wp = W + 2 * pad;
  const int XR = TR + K - 1;
  float* xs = smem;                          // [Cin][XR][Wp]
  float* ds = smem + (size_t)Cin * XR * Wp;  // [TR*Wo][COB]
  float* red = smem;                         // reused (after the last tile) for the pixel-group reduction
  const int co0 = blockIdx.x * WG_COB;
  const int chunk = blockIdx.y;
  const int n0 = chunk * spc, n1 = min(N, n0 + spc);
  const int E = Cin * K * K;
  const int tid = threadIdx.x;
  const int PG = E >= 256 ? 1 : 256 / E;
  const int pg = tid / (E >= 256 ? 256 : E);
  const int e0 = tid % (E >= 256 ? 256 : E);
  const bool active = pg < PG;
  const int ncob = min(WG_COB, Cout - co0);

  float acc[WG_JMAX][WG_COB];
#pragma unroll
  for (int j = 0; j < WG_JMAX; ++j)
#pragma unroll
    for (int o = 0; o < WG_COB; ++o) acc[j][o] = 0.f;

  int eci[WG_JMAX], ekh[WG_JMAX], ekw[WG_JMAX];
#pragma unroll
  for (int j = 0; j < WG_JMAX; ++j) {
    const int e = e0 + j * 256;
    eci[j] = e / (K * K);
    ekh[j] = (e % (K * K)) / K;
    ekw[j] = e % K;
  }

  for (int n = n0; n < n1; ++n) {
    for (int r0 = 0; r0 < Ho; r0 += TR) {
      const int tr = min(TR, Ho - r0);
      __syncthreads();
      // X rows r0-pad .. r0-pad+tr+K-2, zero padded
      const int xr = tr + K - 1;
      for (int i = tid; i < Cin * xr * Wp; i += 256) {
        const int c = i / (xr * Wp), r = (i / Wp) % xr, q = i % Wp;
        const int iy = r0 - pad + r, ix = q - pad;
        float v = 0.f;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W)
          v = io<TX>::ld(x, (((size_t)n * Cin + c) * H + iy) * W + ix);
        xs[((size_t)c * XR + r) * Wp + q] = v;
      }
      for (int i = tid; i < WG_COB * tr * Wo; i += 256) {
        const int o = i / (tr * Wo), p = i % (tr * Wo);
        float v = 0.f;
        if (o < ncob) v = io<TD>::ld(dy, (((size_t)n * Cout + co0 + o) * Ho + r0) * Wo + p);
        ds[p * WG_COB + o] = v;
      }
      __syncthreads();
      if (active) {
        for (int p = pg; p < tr * Wo; p += PG) {
          const int py = p / Wo, px = p % Wo;
          float d[WG_COB];
#pragma unroll
          for (int o = 0; o < WG_COB; ++o) d[o] = ds[p * WG_COB + o];
#pragma unroll
          for (int j = 0; j < WG_JMAX; ++j) {
            if (e0 + j * 256 < E) {
              const float xv = xs[((size_t)eci[j] * XR + py + ekh[j]) * Wp + px + ekw[j]];
#pragma unroll
              for (int o = 0; o < WG_COB; ++o) acc[j][o] = fmaf(xv, d[o], acc[j][o]);
            }
          }
        }
      }
    }
  }

  // reduce over pixel groups (fixed order) and write this chunk's partial slab
  float* out = dw_parts + (size_t)chunk * Cout * E;
  if (PG == 1) {
#pragma unroll
    for (int j = 0; j < WG_JMAX; ++j) {
      const int e = e0 + j * 256;
      if (active && e < E)
        for (int o = 0; o < ncob; ++o) out[(size_t)(co0 + o) * E + e] = acc[j][o];
    }
  } else {
    __syncthreads();
    if (active)
      for (int o = 0; o < WG_COB; ++o) red[(pg * E + e0) * WG_COB + o] = acc[0][o];
    __syncthreads();
    for (int i = tid; i < E * WG_COB; i += 256) {
      const int e = i / WG_COB, o = i % WG_COB;
      float s = 0.f;
      for (int g = 0; g < PG; ++g) s += red[(g * E + e) * WG_COB + o];
      if (o < ncob) out[(size_t)(co0 + o) * E + e] = s;
    }
  }
}

template <typename TX, typename TD>
int launch_wgrad(const void* x, const void* dy, float* dw_parts, int N, int Cin, int H, int W,
                 int Cout, int K, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  const int E = Cin * K * K;
  if (E > 256 * WG_JMAX) return AVD_ERR_SHAPE;
  const int chunks = avd_conv2d_wgrad_chunks(N, Cout, Cin, K);
  const int spc = avd_cdiv(N, chunks);
  const int Wp = W + 2 * pad;
  // rows per tile: keep LDS <= 48 KB, and the reduction buffer (PG*E*8 floats) must fit.
  const size_t budget = 12288;
  int TR = Ho;
  while (TR > 1 && (size_t)Cin * (TR + K - 1) * Wp + (size_t)WG_COB * TR * Wo > budget) --TR;
  const int PG = E >= 256 ? 1 : 256 / E;
  size_t fl = (size_t)Cin * (TR + K - 1) * Wp + (size_t)WG_COB * TR * Wo;
  const size_t redfl = PG > 1 ? (size_t)PG * E * WG_COB : 0;
  if (fl < redfl) fl = redfl;
  dim3 grid(avd_cdiv(Cout, WG_COB), chunks);
  if (K == 5)
    conv_wgrad_kernel<TX, TD, 5><<<grid, 256, fl * sizeof(float), st>>>(
        (const TX*)x, (const TD*)dy, dw_parts, N, Cin, H, W, Cout, Ho, Wo, pad, spc, TR);
  else if (K == 3)
    conv_wgrad_kernel<TX, TD, 3><<<grid, 256, fl * sizeof(float), st>>>(
        (const TX*)x, (const TD*)dy, dw_parts, N, Cin, H, W, Cout, Ho, Wo, pad, spc, TR);
  else
    return AVD_ERR_SHAPE;
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // namespace

int avd_wgrad_mfma_bf16(const void* x, const void* dy, float* parts, int N, int Cin, int H, int W,
                        int Cout, int K, int pad, hipStream_t st);
int avd_conv_mfma_bf16(const void* x, const void* wk, const float* bias, void* y, float* stats,
                       int N, int Cin, int H, int W, int Cout, int K, int pad, hipStream_t st);
int avd_weight_layout_mfma(const float* w, void* wk, int Cout, int Cin, int K, int mode,
                           hipStream_t st);
int avd_mfma_layout_size(int Cout, int Cin, int K, int mode);

// MFMA path for bf16 activations when the conv's input channels are a multiple of 8
static bool use_mfma(int dt_in, int dt_out, int cin) {
  return dt_in == AVD_BF16 && dt_out == AVD_BF16 && cin % 8 == 0 && cin <= 256;
}

extern "C" {

int avd_conv2d_stat_tiles(int Ho, int Wo) { return avd_cdiv(Ho, TS) * avd_cdiv(Wo, TS); }

int avd_conv_weight_layout_elems(int Cout, int Cin, int K, int mode) {
  if (mode == 0 || mode == 1) return Cout * Cin * K * K;
  if (mode == 2 || mode == 3) return avd_mfma_layout_size(Cout, Cin, K, mode);
  return AVD_ERR_ARG;
}

int avd_conv_weight_layout(const float* w, void* wt, int Cout, int Cin, int K, int mode,
                           void* stream) {
  if (!w || !wt || mode < 0 || mode > 3) return AVD_ERR_ARG;
  if (mode >= 2) return avd_weight_layout_mfma(w, wt, Cout, Cin, K, mode, avd_stream(stream));
  const int n = Cout * Cin * K * K;
  weight_layout_kernel<<<avd_cdiv(n, 256), 256, 0, avd_stream(stream)>>>(w, (float*)wt, Cout, Cin,
                                                                          K * K, mode);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_conv2d_fwd(const void* x, int xdt, const void* wt_, const float* bias, void* y, int ydt,
                   float* stats, int N, int Cin, int H, int W, int Cout, int K, int pad,
                   void* stream) {
  if (!x || !wt_ || !y) return AVD_ERR_ARG;
  if (N <= 0 || Cin <= 0 || Cout <= 0 || (K != 3 && K != 5) || H + 2 * pad < K) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
  if (use_mfma(xdt, ydt, Cin))
    return avd_conv_mfma_bf16(x, wt_, bias, y, stats, N, Cin, H, W, Cout, K, pad, st);
  const float* wt = (const float*)wt_;
#define AVD_F(TI, TO)                                                                          \
  return stats ? dispatch_direct<TI, TO, true>(x, wt, bias, y, stats, N, Cin, H, W, Cout, K,   \
                                               pad, st)                                        \
               : dispatch_direct<TI, TO, false>(x, wt, bias, y, stats, N, Cin, H, W, Cout, K,  \
                                                pad, st);
  if (xdt == AVD_F32 && ydt == AVD_F32) { AVD_F(float, float) }
  if (xdt == AVD_F32 && ydt == AVD_BF16) { AVD_F(float, bf16) }
  if (xdt == AVD_BF16 && ydt == AVD_BF16) { AVD_F(bf16, bf16) }
  if (xdt == AVD_BF16 && ydt == AVD_F32) { AVD_F(bf16, float) }
#undef AVD_F
  return AVD_ERR_DTYPE;
}

int avd_conv2d_dgrad(const void* dy, const void* wt_d, void* dx, int dt, int N, int Cin,
                     int H, int W, int Cout, int K, int pad, void* stream) {
  // input-grad = forward conv of dy with flipped taps, channels swapped, pad' = K-1-pad
  if (!dy || !wt_d || !dx) return AVD_ERR_ARG;
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  if (Ho <= 0 || Wo <= 0) return AVD_ERR_SHAPE;
  const int padT = K - 1 - pad;
  hipStream_t st = avd_stream(stream);
  if (use_mfma(dt, dt, Cout))
    return avd_conv_mfma_bf16(dy, wt_d, nullptr, dx, nullptr, N, Cout, Ho, Wo, Cin, K, padT, st);
  const float* wt_dgrad = (const float*)wt_d;
  if (dt == AVD_F32)
    return dispatch_direct<float, float, false>(dy, wt_dgrad, nullptr, dx, nullptr, N, Cout, Ho,
                                                Wo, Cin, K, padT, st);
  if (dt == AVD_BF16)
    return dispatch_direct<bf16, bf16, false>(dy, wt_dgrad, nullptr, dx, nullptr, N, Cout, Ho,
                                              Wo, Cin, K, padT, st);
  return AVD_ERR_DTYPE;
}

int avd_conv2d_wgrad_chunks(int N, int Cout, int Cin, int K) {
  // enough sample chunks to fill the chip, partial slabs capped at ~64 MB
  long long per = (long long)Cout * Cin * K * K;
  long long c = (1ll << 24) / (per > 0 ? per : 1);
  if (c > 1024) c = 1024;
  if (c < 128) c = 128;
  if (c > N) c = N;
  return (int)c;
}

int avd_conv2d_wgrad(const void* x, int xdt, const void* dy, int dydt, float* dw_parts, int N,
                     int Cin, int H, int W, int Cout, int K, int pad, void* stream) {
  if (!x || !dy || !dw_parts) return AVD_ERR_ARG;
  hipStream_t st = avd_stream(stream);
  if (xdt == AVD_F32 && dydt == AVD_F32)
    return launch_wgrad<float, float>(x, dy, dw_parts, N, Cin, H, W, Cout, K, pad, st);
  if (xdt == AVD_BF16 && dydt == AVD_BF16)
    return avd_wgrad_mfma_bf16(x, dy, dw_parts, N, Cin, H, W, Cout, K, pad, st);
  if (xdt == AVD_F32 && dydt == AVD_BF16)
    return launch_wgrad<float, bf16>(x, dy, dw_parts, N, Cin, H, W, Cout, K, pad, st);
  if (xdt == AVD_BF16 && dydt == AVD_F32)
    return launch_wgrad<bf16, float>(x, dy, dw_parts, N, Cin, H, W, Cout, K, pad, st);
  return AVD_ERR_DTYPE;
}

}  // extern "C"
