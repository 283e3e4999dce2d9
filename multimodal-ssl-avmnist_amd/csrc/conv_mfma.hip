// MFMA (v_mfma_f32_16x16x32_bf16) kernels for the bf16 conv layers of the CentralNet / CNN
// encoders (reference models/unimodal.py:105-221, models/dino.py:18-73).
//
// Weight gradient, as a GEMM with the pixels as the reduction axis:
//     dW^T[(ci,kh,kw)][co] = sum_{n,y,x} X[n][ci][y+kh-p][x+kw-p] * dY[n][co][y][x]
//   M = (ci, kh, kw) of a group of CIB input channels, N = co, K = output pixels.
//   An MFMA k-group is 8 consecutive output pixels of one row.  For the A operand those are
//   8 consecutive input pixels shifted by kw, which would be a misaligned 16-byte LDS read.
//   The input rows are therefore staged once per shift s = kw (K copies, each row 16-byte
//   aligned): xs[ci][s][r][c] = Xpad[ci][r][c + s].  Every A and B fragment is then a single
//   aligned ds_read_b128, and kh is only a row offset.  Output rows are padded to Wo8 = 8*ceil(Wo/8)
//   with zero dY so partial groups contribute nothing.
//   Deterministic: each block writes one partial slab per sample chunk (no atomics), reduced
//   by avd_sum_rows in fixed order.
#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

__device__ __forceinline__ bf16x8 as_frag(u4 v) { return __builtin_bit_cast(bf16x8, v); }

// Pack 8 consecutive bf16 starting at element offset o (0..) of a dword window w[].
template <int NW>
__device__ __forceinline__ u4 window8(const unsigned (&w)[NW], int o) {
  u4 r;
  const int d = o >> 1;
  if ((o & 1) == 0) {
    r.x = w[d]; r.y = w[d + 1]; r.z = w[d + 2]; r.w = w[d + 3];
  } else {
    r.x = __builtin_amdgcn_alignbyte(w[d + 1], w[d], 2);
    r.y = __builtin_amdgcn_alignbyte(w[d + 2], w[d + 1], 2);
    r.z = __builtin_amdgcn_alignbyte(w[d + 3], w[d + 2], 2);
    r.w = __builtin_amdgcn_alignbyte(w[d + 4], w[d + 3], 2);
  }
  return r;
}

template <int K, int NT, int MTW, int WK>
__global__ __launch_bounds__(256) void wgrad_mfma_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ dw_parts, int N,
    int Cin, int H, int W, int Cout, int Ho, int Wo, int pad, int spc, int TR, int Wo8, int CIB) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int WT = 4 / WK;
  const int QW = Wo8 >> 3;
  const int XR = TR + K - 1;
  bf16* xs = reinterpret_cast<bf16*>(smem);          // [CIB][K][XR][Wo8]
  bf16* ds = xs + (size_t)CIB * K * XR * Wo8;        // [NT*16][TR][Wo8]
  const int ci0 = blockIdx.x * CIB;
  const int co0 = blockIdx.z * NT * 16;
  const int chunk = blockIdx.y;
  const int n0 = chunk * spc, n1 = min(N, n0 + spc);
  const int M = CIB * K * K;
  const int Mt = (M + 15) >> 4;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wt = wave % WT, wk = wave / WT;
  const int g = lane >> 4, r16 = lane & 15;
  const int E = Cin * K * K;

  f4 acc[MTW][NT];
#pragma unroll
  for (int j = 0; j < MTW; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};

  int a_off[MTW];
  bool a_ok[MTW];
#pragma unroll
  for (int j = 0; j < MTW; ++j) {
    const int mt = wt + j * WT;
    const int m = mt * 16 + r16;
    a_ok[j] = (mt < Mt) && (m < M);
    const int mm = a_ok[j] ? m : 0;
    const int cl = mm / (K * K), t = mm % (K * K), kh = t / K, kw = t % K;
    a_off[j] = ((cl * K + kw) * XR + kh) * Wo8;
  }
  int b_off[NT];
  bool b_ok[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int co = co0 + t * 16 + r16;
    b_ok[t] = co < Cout;
    b_off[t] = (t * 16 + r16) * TR * Wo8;
  }
  const bool vec_dy = (Wo & 7) == 0;
  const int sh = (pad & 1);  // window start parity (8q - pad) & 1

  for (int n = n0; n < n1; ++n) {
    for (int y0 = 0; y0 < Ho; y0 += TR) {
      const int tr = min(TR, Ho - y0);
      const int xr = tr + K - 1;
      __syncthreads();
      // ---- stage the K shifted copies of the input rows y0-pad .. y0-pad+xr-1
      const int nxt = CIB * xr * QW;
      for (int task = tid; task < nxt; task += 256) {
        const int cl = task / (xr * QW);
        const int rem = task - cl * xr * QW;
        const int r = rem / QW, q = rem - (rem / QW) * QW;
        const int iy = y0 - pad + r;
        const int cs = 8 * q - pad - sh;  // even window start
        unsigned w[8];
        const bool row_ok = (iy >= 0) && (iy < H) && (ci0 + cl < Cin);
        const unsigned* src = reinterpret_cast<const unsigned*>(
            x + (((size_t)n * Cin + ci0 + cl) * H + (row_ok ? iy : 0)) * W);
        if (!(W & 1)) {
#pragma unroll
          for (int d = 0; d < 8; ++d) {
            const int c = cs + 2 * d;
            w[d] = (row_ok && c >= 0 && c < W) ? src[c >> 1] : 0u;  // W even: both halves in/out together
          }
        } else {  // odd width (e.g. 7x7 maps): rows are not dword aligned, gather elements
          const unsigned short* e16 = reinterpret_cast<const unsigned short*>(src);
#pragma unroll
          for (int d = 0; d < 8; ++d) {
            const int c = cs + 2 * d;
            const unsigned lo = (row_ok && c >= 0 && c < W) ? e16[c] : 0u;
            const unsigned hi = (row_ok && c + 1 >= 0 && c + 1 < W) ? e16[c + 1] : 0u;
            w[d] = lo | (hi << 16);
          }
        }
#pragma unroll
        for (int s = 0; s < K; ++s) {
          const u4 v = window8(w, sh + s);
          *reinterpret_cast<u4*>(xs + ((size_t)(cl * K + s) * XR + r) * Wo8 + 8 * q) = v;
        }
      }
      // ---- stage dY rows y0 .. y0+tr-1 for NT*16 output channels (zero beyond Cout / Wo)
      const int ndt = NT * 16 * tr * QW;
      for (int task = tid; task < ndt; task += 256) {
        const int co = task / (tr * QW);
        const int rem = task - co * tr * QW;
        const int r = rem / QW, q = rem - (rem / QW) * QW;
        u4 v = u4{0u, 0u, 0u, 0u};
        if (co0 + co < Cout) {
          const bf16* row = dy + (((size_t)n * Cout + co0 + co) * Ho + y0 + r) * Wo;
          if (vec_dy) {
            v = *reinterpret_cast<const u4*>(row + 8 * q);
          } else {
            const unsigned short* e16 = reinterpret_cast<const unsigned short*>(row);
            unsigned t4[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const int c = 8 * q + 2 * d;
              const unsigned lo = c < Wo ? e16[c] : 0u;
              const unsigned hi = c + 1 < Wo ? e16[c + 1] : 0u;
              t4[d] = lo | (hi << 16);
            }
            v = u4{t4[0], t4[1], t4[2], t4[3]};
          }
        }
        *reinterpret_cast<u4*>(ds + ((size_t)co * TR + r) * Wo8 + 8 * q) = v;
      }
      __syncthreads();
      // ---- MFMA over the strip's pixel groups
      const int GS = tr * QW;
      const int KS = (GS + 3) >> 2;
      for (int ks = wk; ks < KS; ks += WK) {
        const int gi = 4 * ks + g;
        const bool kok = gi < GS;
        const int r = kok ? gi / QW : 0, q = kok ? gi % QW : 0;
        const int rq = r * Wo8 + 8 * q;
        bf16x8 b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          u4 v = u4{0u, 0u, 0u, 0u};
          if (kok && b_ok[t]) v = *reinterpret_cast<const u4*>(ds + b_off[t] + rq);
          b[t] = as_frag(v);
        }
#pragma unroll
        for (int j = 0; j < MTW; ++j) {
          if (wt + j * WT >= Mt) continue;  // wave-uniform
          u4 v = u4{0u, 0u, 0u, 0u};
          if (kok && a_ok[j]) v = *reinterpret_cast<const u4*>(xs + a_off[j] + rq);
          const bf16x8 a = as_frag(v);
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[t], acc[j][t], 0, 0, 0);
        }
      }
    }
  }

  // ---- reduce the WK k-split waves (fixed order) and write the chunk's partial slab
  float* red = reinterpret_cast<float*>(smem);
  if (WK > 1) {
    __syncthreads();
    if (wk > 0) {
#pragma unroll
      for (int j = 0; j < MTW; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          *reinterpret_cast<f4*>(red + ((((wk - 1) * WT + wt) * MTW + j) * NT + t) * 256 + lane * 4) =
              acc[j][t];
    }
    __syncthreads();
    if (wk == 0) {
      for (int k2 = 1; k2 < WK; ++k2)
#pragma unroll
        for (int j = 0; j < MTW; ++j)
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[j][t] += *reinterpret_cast<const f4*>(
                red + ((((k2 - 1) * WT + wt) * MTW + j) * NT + t) * 256 + lane * 4);
    }
  }
  if (wk == 0) {
    float* out = dw_parts + (size_t)chunk * Cout * E;
#pragma unroll
    for (int j = 0; j < MTW; ++j) {
      const int mt = wt + j * WT;
      if (mt >= Mt) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int co = co0 + t * 16 + r16;
        if (co >= Cout) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mt * 16 + 4 * g + i;
          if (m < M) out[(size_t)co * E + (size_t)ci0 * K * K + m] = acc[j][t][i];
        }
      }
    }
  }
}

template <int K, int NT, int MTW, int WK>
int launch_wgrad_mfma(const bf16* x, const bf16* dy, float* parts, int N, int Cin, int H, int W,
                      int Cout, int Ho, int Wo, int pad, int CIB, int TR, int Wo8, size_t lds,
                      hipStream_t st) {
  const int chunks = avd_conv2d_wgrad_chunks(N, Cout, Cin, K);
  const int spc = avd_cdiv(N, chunks);
  dim3 grid(Cin / CIB, chunks, avd_cdiv(Cout, NT * 16));
  wgrad_mfma_kernel<K, NT, MTW, WK><<<grid, 256, lds, st>>>(x, dy, parts, N, Cin, H, W, Cout, Ho,
                                                            Wo, pad, spc, TR, Wo8, CIB);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // namespace

// bf16 weight-gradient entry used by avd_conv2d_wgrad (conv.hip) for bf16 x/dy.
int avd_wgrad_mfma_bf16(const void* x, const void* dy, float* parts, int N, int Cin, int H, int W,
                        int Cout, int K, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  if (K != 3 && K != 5) return AVD_ERR_SHAPE;
  const int CIB = Cin < 8 ? Cin : 8;
  if (Cin % CIB) return AVD_ERR_SHAPE;
  const int M = CIB * K * K;
  const int Mt = (M + 15) / 16;
  int WK, MTW;
  if (Mt >= 4) { WK = 1; MTW = (Mt + 3) / 4; }
  else if (Mt >= 2) { WK = 2; MTW = (Mt + 1) / 2; }
  else { WK = 4; MTW = 1; }
  if (MTW > 4) return AVD_ERR_SHAPE;
  if (MTW == 3) MTW = 4;
  const int NT = Cout <= 16 ? 1 : Cout <= 32 ? 2 : 4;
  const int Wo8 = (Wo + 7) & ~7;
  // rows per strip: LDS (shift copies + dY tile) <= 64 KB
  const size_t budget = 64 * 1024;
  int TR = Ho;
  auto need = [&](int tr) {
    return ((size_t)CIB * K * (tr + K - 1) * Wo8 + (size_t)NT * 16 * tr * Wo8) * 2;
  };
  while (TR > 1 && need(TR) > budget) --TR;
  size_t lds = need(TR);
  const size_t red = (size_t)(WK - 1) * (4 / WK) * MTW * NT * 256 * 4;
  if (lds < red) lds = red;
  const bf16* xb = (const bf16*)x;
  const bf16* db = (const bf16*)dy;
#define AVD_W(KK, NTT, MW, WKK)                                                                  \
  if (K == KK && NT == NTT && MTW == MW && WK == WKK)                                           \
    return launch_wgrad_mfma<KK, NTT, MW, WKK>(xb, db, parts, N, Cin, H, W, Cout, Ho, Wo, pad,  \
                                                CIB, TR, Wo8, lds, st);
#define AVD_WN(KK, MW, WKK) AVD_W(KK, 1, MW, WKK) AVD_W(KK, 2, MW, WKK) AVD_W(KK, 4, MW, WKK)
  AVD_WN(5, 4, 1) AVD_WN(5, 2, 1) AVD_WN(5, 1, 1) AVD_WN(5, 1, 2) AVD_WN(5, 2, 2) AVD_WN(5, 1, 4)
  AVD_WN(3, 4, 1) AVD_WN(3, 2, 1) AVD_WN(3, 1, 1) AVD_WN(3, 1, 2) AVD_WN(3, 2, 2) AVD_WN(3, 1, 4)
#undef AVD_WN
#undef AVD_W
  return AVD_ERR_SHAPE;
}

// ============================================================================================
// Forward / input-grad convolution as an implicit GEMM on MFMA (bf16 in, fp32 accumulate):
//     y[n][co][oy][ox] = bias[co] + sum_{tap, ci} X[n][ci][oy+kh-p][ox+kw-p] * W[co][ci][tap]
//   M = 16x16 output pixels of one sample (16 M-tiles, one per tile row; 4 waves x 4 rows),
//   N = NT*16 output channels, K = (tap, ci) with ci fastest, padded to a multiple of 32.
//   The input tile (+halo) is staged channels-last in LDS ([r][c][ci], pixel stride padded to
//   an odd multiple of 16 B for Cin >= 16 so the 16 lanes of a fragment hit distinct banks), so
//   an A fragment (8 consecutive ci of one pixel and tap) is one aligned ds_read_b128.  B
//   fragments come pre-laid-out from global memory (avd_conv_weight_layout modes 2/3).
//   The forward epilogue adds the bias, rounds to bf16 and emits the per-(channel, sample,
//   tile) BatchNorm partial sums of the stored values (same layout as the VALU kernel).
//   The input gradient is the same kernel on dY with flipped taps and swapped channels.
namespace {

constexpr int FT = 16;  // output tile edge

template <int K, int CIN, int NT, bool STATS>
__global__ __launch_bounds__(256) void conv_fwd_mfma_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    bf16* __restrict__ y, float* __restrict__ stats, int H, int W, int Cout, int Ho, int Wo,
    int pad, int tilesX, int tiles, int Kpad) {
  constexpr int IT = FT + K - 1;
  constexpr int CC = CIN < 64 ? CIN : 64;     // input channels per LDS chunk
  constexpr int PS = CC == 8 ? 8 : CC + 8;    // LDS pixel stride (elements), odd multiple of 16 B
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = reinterpret_cast<bf16*>(smem);  // [IT][IT][PS]
  __shared__ float red[4][NT * 16][2];
  const int n = blockIdx.y;
  const int tile = blockIdx.x;
  const int co0 = blockIdx.z * NT * 16;
  const int ty0 = (tile / tilesX) * FT, tx0 = (tile % tilesX) * FT;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;

  f4 acc[4][NT];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};

  // Input channels are processed in chunks of CC (<= 64) so the LDS tile stays <= ~58 KB.
  const bf16* xn = x + (size_t)n * CIN * H * W;
  constexpr int GPT = CC / 8;                    // 8-channel k-groups per tap in a chunk
  constexpr int KSC = (K * K * GPT + 3) / 4;     // k-steps (4 groups each) per chunk
  for (int c0 = 0; c0 < CIN; c0 += CC) {
    if (c0) __syncthreads();
    // ---- stage the chunk's input tile channels-last (pairs of channels per dword write)
    for (int task = tid; task < (CC / 2) * IT * IT; task += 256) {
      const int cp = task / (IT * IT);
      const int pix = task - cp * IT * IT;
      const int r = pix / IT, c = pix - (pix / IT) * IT;
      const int iy = ty0 - pad + r, ix = tx0 - pad + c;
      unsigned v = 0u;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
        const size_t o = ((size_t)(c0 + 2 * cp) * H + iy) * W + ix;
        const unsigned lo = reinterpret_cast<const unsigned short*>(xn)[o];
        const unsigned hi = reinterpret_cast<const unsigned short*>(xn)[o + (size_t)H * W];
        v = lo | (hi << 16);
      }
      *reinterpret_cast<unsigned*>(xs + (r * IT + c) * PS + 2 * cp) = v;
    }
    __syncthreads();
    for (int s = 0; s < KSC; ++s) {
      const int kg = 4 * s + g;               // this lane's k-group within the chunk
      const bool kok = kg < K * K * GPT;
      const int tap = kok ? kg / GPT : 0, cig = kg % GPT;
      const int kh = tap / K, kw = tap % K;
      const int kw_off = tap * CIN + c0 + 8 * cig;  // column in the [o][tap*Cin + ci] layout
      bf16x8 b[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        u4 v = u4{0u, 0u, 0u, 0u};
        if (kok) v = *reinterpret_cast<const u4*>(wk + (size_t)(co0 + t * 16 + r16) * Kpad + kw_off);
        b[t] = as_frag(v);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ly = 4 * wave + j;
        u4 v = u4{0u, 0u, 0u, 0u};
        if (kok) v = *reinterpret_cast<const u4*>(xs + ((ly + kh) * IT + r16 + kw) * PS + 8 * cig);
        const bf16x8 a = as_frag(v);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[t], acc[j][t], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: C[row = pixel 4g+i of tile row ly][col = co]
  float ssum[NT], ssq[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { ssum[t] = 0.f; ssq[t] = 0.f; }
  const bool even = (Wo & 1) == 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int co = co0 + t * 16 + r16;
    const bool cok = co < Cout;
    const float bv = (bias && cok) ? bias[co] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oy = ty0 + 4 * wave + j;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ox = tx0 + 4 * g + i;
        v[i] = io<bf16>::rnd(acc[j][t][i] + bv);
        const bool ok = cok && oy < Ho && ox < Wo;
        if (STATS && ok) { ssum[t] += v[i]; ssq[t] += v[i] * v[i]; }
      }
      if (cok && oy < Ho) {
        bf16* row = y + (((size_t)n * Cout + co) * Ho + oy) * Wo;
        const int ox0 = tx0 + 4 * g;
        if (even && ox0 + 3 < Wo) {
          const unsigned p0 = pack_bf16x2(v[0], v[1]);
          const unsigned p1 = pack_bf16x2(v[2], v[3]);
          reinterpret_cast<unsigned*>(row + ox0)[0] = p0;
          reinterpret_cast<unsigned*>(row + ox0)[1] = p1;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (ox0 + i < Wo) row[ox0 + i] = f2bf(v[i]);
        }
      }
    }
  }
  if (STATS) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float a = ssum[t], q = ssq[t];
      a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (g == 0) { red[wave][t * 16 + r16][0] = a; red[wave][t * 16 + r16][1] = q; }
    }
    __syncthreads();
    if (tid < NT * 16 * 2) {
      const int cl = tid >> 1, k = tid & 1;
      const int co = co0 + cl;
      if (co < Cout) {
        const float r = red[0][cl][k] + red[1][cl][k] + red[2][cl][k] + red[3][cl][k];
        stats[(((size_t)co * gridDim.y + n) * tiles + tile) * 2 + k] = r;
      }
    }
  }
}

// wk[o][tap*C + c] (bf16, rows padded to Kpad, o padded to a multiple of 16, zeros elsewhere)
//   mode 2 (forward):    o = co, c = ci, value w[co][ci][tap]
//   mode 3 (input-grad): o = ci, c = co, value w[co][ci][K*K-1-tap]
__global__ void weight_layout_mfma_kernel(const float* __restrict__ w, bf16* __restrict__ wk,
                                          int Cout, int Cin, int KK, int mode, int O, int C,
                                          int Kpad, int Opad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Opad * Kpad) return;
  const int o = i / Kpad, k = i % Kpad;
  float v = 0.f;
  if (o < O && k < KK * C) {
    const int tap = k / C, c = k % C;
    if (mode == 2) v = w[((size_t)o * Cin + c) * KK + tap];
    else v = w[((size_t)c * Cin + o) * KK + (KK - 1 - tap)];
  }
  wk[i] = f2bf(v);
}

template <int K, int CIN, int NT, bool STATS>
int launch_fwd_mfma(const bf16* x, const bf16* wk, const float* bias, bf16* y, float* stats, int N,
                    int H, int W, int Cout, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  const int tilesX = avd_cdiv(Wo, FT), tilesY = avd_cdiv(Ho, FT);
  constexpr int IT = FT + K - 1;
  constexpr int CC = CIN < 64 ? CIN : 64;
  constexpr int PS = CC == 8 ? 8 : CC + 8;
  const size_t lds = (size_t)IT * IT * PS * 2;
  const int Kpad = avd_cdiv(K * K * CIN, 32) * 32;
  dim3 grid(tilesX * tilesY, N, avd_cdiv(Cout, NT * 16));
  conv_fwd_mfma_kernel<K, CIN, NT, STATS><<<grid, 256, lds, st>>>(
      x, wk, bias, y, stats, H, W, Cout, Ho, Wo, pad, tilesX, tilesX * tilesY, Kpad);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // namespace

int avd_mfma_layout_size(int Cout, int Cin, int K, int mode) {
  const int O = mode == 2 ? Cout : Cin, C = mode == 2 ? Cin : Cout;
  const int Opad = (O + 15) / 16 * 16;
  // rows padded to the largest NT*16 block so blockIdx.z tiles never read past the end
  const int Opad64 = O > 32 ? (O + 63) / 64 * 64 : Opad;
  return Opad64 * avd_cdiv(K * K * C, 32) * 32;
}

int avd_weight_layout_mfma(const float* w, void* wk, int Cout, int Cin, int K, int mode,
                           hipStream_t st) {
  const int O = mode == 2 ? Cout : Cin, C = mode == 2 ? Cin : Cout;
  const int Kpad = avd_cdiv(K * K * C, 32) * 32;
  const int rows = avd_mfma_layout_size(Cout, Cin, K, mode) / Kpad;
  const int n = rows * Kpad;
  weight_layout_mfma_kernel<<<avd_cdiv(n, 256), 256, 0, st>>>(w, (bf16*)wk, Cout, Cin, K * K, mode,
                                                              O, C, Kpad, rows);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// Forward (STATS as requested) / input-grad convolution on MFMA; Cin % 8 == 0, Cin <= 256.
int avd_conv_mfma_bf16(const void* x, const void* wk, const float* bias, void* y, float* stats,
                       int N, int Cin, int H, int W, int Cout, int K, int pad, hipStream_t st) {
  const int NT = Cout <= 16 ? 1 : Cout <= 32 ? 2 : 4;
  const bf16* xb = (const bf16*)x;
  const bf16* wb = (const bf16*)wk;
  bf16* yb = (bf16*)y;
#define AVD_F(KK, CI, NTT)                                                                      \
  if (K == KK && Cin == CI && NT == NTT)                                                       \
    return stats ? launch_fwd_mfma<KK, CI, NTT, true>(xb, wb, bias, yb, stats, N, H, W, Cout,   \
                                                        pad, st)                                \
                 : launch_fwd_mfma<KK, CI, NTT, false>(xb, wb, bias, yb, stats, N, H, W, Cout,  \
                                                         pad, st);
#define AVD_FN(KK, CI) AVD_F(KK, CI, 1) AVD_F(KK, CI, 2) AVD_F(KK, CI, 4)
  AVD_FN(5, 8) AVD_FN(5, 16) AVD_FN(5, 32) AVD_FN(5, 64)
  AVD_FN(3, 8) AVD_FN(3, 16) AVD_FN(3, 32) AVD_FN(3, 64) AVD_FN(3, 128) AVD_FN(3, 256)
#undef AVD_FN
#undef AVD_F
  return AVD_ERR_SHAPE;
}
