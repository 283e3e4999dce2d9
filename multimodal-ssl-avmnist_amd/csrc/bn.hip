// BatchNorm (train mode, per-(group, channel) statistics), ReLU, maxpool2 / global-average
// pool, GELU and dropout kernels, forward and backward, plus deterministic reductions.
//
// Reference semantics:
//  * BatchNorm2d/1d train mode, eps 1e-5, momentum 0.1, biased variance for normalisation,
//    unbiased for running_var (nn.BatchNorm, unimodal.py:114,130; dino.py:1245);
//  * one BN "group" per encoder call: the reference runs each view separately
//    (dino.py:680-704), so statistics are per (view, channel);
//  * F.max_pool2d(2) floor mode with first-max tie-break (ATen CPU scan order);
//  * nn.GELU() erf form; nn.Dropout inverted scaling.
//
// Partial-statistic layout everywhere: channel-major parts [C][G][R][2] so the finaliser
// reads contiguous rows.  All reductions are fixed-order (f64 in the finalisers).
#include <algorithm>

#include "common.h"

using namespace avd;

namespace {

// ----------------------------------------------------------------------------- helpers
template <int NT>
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += sh[i];
  return r;
}

// Sum of rows [r0, r0+R) of a channel-major (sum, sumsq)-pair array, block of 256, f64.
__device__ __forceinline__ void reduce_pairs(const float* __restrict__ p, long long R, double* sh,
                                             double& a, double& b) {
  double s = 0.0, q = 0.0;
  for (long long r = threadIdx.x; r < R; r += 256) {
    const float2 v = reinterpret_cast<const float2*>(p)[r];
    s += v.x;
    q += v.y;
  }
  a = block_sum_d<256>(s, sh);
  b = block_sum_d<256>(q, sh);
}

// ----------------------------------------------------------------------------- forward stats
// Two passes.  (1) grid (S, G, C): block (s, g, c) sums rows [s*chunk, ...) of the (g, c)
// partial-pair list in f64 and, once every thread has read its rows, stores the two doubles
// over the first rows of its own chunk (disjoint per block, so the in-place write is safe:
// parts is consumed).  (2) one thread per channel folds the S chunk sums of every group in
// fixed order and applies the running-stat updates sequentially over g.
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(float* __restrict__ parts, int G,
                                                               int R, int S, int chunk) {
  __shared__ double sh[4];
  const int s = blockIdx.x, g = blockIdx.y, c = blockIdx.z;
  float* p = parts + (((size_t)c * G + g) * R + (size_t)s * chunk) * 2;
  // the last chunk takes the remainder, so every chunk has >= 2 rows = room for 2 doubles
  const int rows = s == S - 1 ? R - s * chunk : chunk;
  double a, q;
  reduce_pairs(p, rows, sh, a, q);   // ends with a barrier after all reads
  if (threadIdx.x == 0) {
    double* d = reinterpret_cast<double*>(p);   // 8-byte aligned: even float offset
    d[0] = a;
    d[1] = q;
  }
}

__global__ __launch_bounds__(64) void bn_finalize_kernel(
    const float* __restrict__ parts, int G, int R, int C, int S, int chunk, long long count,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* mean_o, float* invstd_o, float* scale_o, float* shift_o, float* rm, float* rv,
    const float* __restrict__ pivot) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  double rmean = rm ? (double)rm[c] : 0.0, rvar = rv ? (double)rv[c] : 0.0;
  const double n = (double)count;
  for (int g = 0; g < G; ++g) {
    double sum = 0.0, sq = 0.0;
    if (S == 0) {   // R == 1: the single partial row as is
      sum = parts[((size_t)c * G + g) * 2];
      sq = parts[((size_t)c * G + g) * 2 + 1];
    }
    for (int s = 0; s < S; ++s) {
      const double* d =
          reinterpret_cast<const double*>(parts + (((size_t)c * G + g) * R + (size_t)s * chunk) * 2);
      sum += d[0];
      sq += d[1];
    }
    const double ms = sum / n;                       // mean of (x - K)
    const double mean = (pivot ? (double)pivot[(size_t)g * C + c] : 0.0) + ms;
    double var = sq / n - ms * ms;
    if (var < 0) var = 0;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const double sc = (double)gamma[c] * invstd;
    mean_o[g * C + c] = (float)mean;
    invstd_o[g * C + c] = (float)invstd;
    scale_o[g * C + c] = (float)sc;
    shift_o[g * C + c] = (float)((double)beta[c] - mean * sc);
    rmean = (1.0 - momentum) * rmean + momentum * mean;
    rvar = (1.0 - momentum) * rvar + momentum * var * n / (n - 1.0);
  }
  if (rm) {
    rm[c] = (float)rmean;
    rv[c] = (float)rvar;
  }
}

// Single pass, one block per channel, for partial lists up to FIN1_MAXROWS rows per group:
// thread t sums rows t / G, t / G + 256 / G, ... of group t % G (every group's loads in flight
// together), the per-thread partials of a group are then folded in fixed order by thread g.
constexpr int FIN1_MAXROWS = 8192;

__device__ __forceinline__ void group_sums(const float* __restrict__ parts, int G, int R, int c,
                                           double* sh1, double* sh2) {
  const int tid = threadIdx.x, per = 256 / G, gq = tid % G, j = tid / G;
  double s1 = 0.0, s2 = 0.0;
  if (j < per) {
    const float2* p = reinterpret_cast<const float2*>(parts) + ((size_t)c * G + gq) * R;
    for (int r = j; r < R; r += per) {
      const float2 v = p[r];
      s1 += v.x;
      s2 += v.y;
    }
  }
  sh1[tid] = s1;
  sh2[tid] = s2;
  __syncthreads();
  if (tid < G) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < per; ++k) {
      a += sh1[k * G + tid];
      b += sh2[k * G + tid];
    }
    sh1[256 + tid] = a;
    sh2[256 + tid] = b;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void bn_finalize1_kernel(
    const float* __restrict__ parts, int G, int R, int C, long long count,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* mean_o, float* invstd_o, float* scale_o, float* shift_o, float* rm, float* rv,
    const float* __restrict__ pivot) {
  __shared__ double sh1[512], sh2[512];
  const int c = blockIdx.x;
  group_sums(parts, G, R, c, sh1, sh2);
  if (threadIdx.x != 0) return;
  double rmean = rm ? (double)rm[c] : 0.0, rvar = rv ? (double)rv[c] : 0.0;
  const double n = (double)count;
  for (int g = 0; g < G; ++g) {
    const double ms = sh1[256 + g] / n;
    const double mean = (pivot ? (double)pivot[(size_t)g * C + c] : 0.0) + ms;
    double var = sh2[256 + g] / n - ms * ms;
    if (var < 0) var = 0;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const double sc = (double)gamma[c] * invstd;
    mean_o[g * C + c] = (float)mean;
    invstd_o[g * C + c] = (float)invstd;
    scale_o[g * C + c] = (float)sc;
    shift_o[g * C + c] = (float)((double)beta[c] - mean * sc);
    rmean = (1.0 - momentum) * rmean + momentum * mean;
    rvar = (1.0 - momentum) * rvar + momentum * var * n / (n - 1.0);
  }
  if (rm) {
    rm[c] = (float)rmean;
    rv[c] = (float)rvar;
  }
}

// ----------------------------------------------------------------------------- relu + pool
template <typename TY, typename TO>
__global__ __launch_bounds__(256) void bn_relu_pool_kernel(
    const TY* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    TO* __restrict__ out, long long total, int B, int C, int H, int W) {
  const int Hp = H / 2, Wp = W / 2;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int wp = (int)(i % Wp);
    const int hp = (int)((i / Wp) % Hp);
    const long long nc = i / ((long long)Hp * Wp);
    const int c = (int)(nc % C);
    const int n = (int)(nc / C);
    const int g = n / B;
    const float sc = scale[g * C + c], sf = shift[g * C + c];
    const size_t base = ((size_t)nc * H + 2 * hp) * W + 2 * wp;
    float m = 0.f;  // relu output >= 0
    m = fmaxf(m, fmaf(io<TY>::ld(y, base), sc, sf));
    m = fmaxf(m, fmaf(io<TY>::ld(y, base + 1), sc, sf));
    m = fmaxf(m, fmaf(io<TY>::ld(y, base + W), sc, sf));
    m = fmaxf(m, fmaf(io<TY>::ld(y, base + W + 1), sc, sf));
    io<TO>::st(out, i, m);
  }
}

template <typename TY>
__global__ __launch_bounds__(256) void bn_relu_pool_gap_kernel(
    const TY* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    float* __restrict__ out, long long total, int B, int C, int H, int W) {
  const int Hp = H / 2, Wp = W / 2;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int n = (int)(i / C);
    const int g = n / B;
    const float sc = scale[g * C + c], sf = shift[g * C + c];
    float acc = 0.f;
    for (int hp = 0; hp < Hp; ++hp)
      for (int wp = 0; wp < Wp; ++wp) {
        const size_t base = ((size_t)i * H + 2 * hp) * W + 2 * wp;
        float m = 0.f;
        m = fmaxf(m, fmaf(io<TY>::ld(y, base), sc, sf));
        m = fmaxf(m, fmaf(io<TY>::ld(y, base + 1), sc, sf));
        m = fmaxf(m, fmaf(io<TY>::ld(y, base + W), sc, sf));
        m = fmaxf(m, fmaf(io<TY>::ld(y, base + W + 1), sc, sf));
        acc += m;
      }
    out[i] = acc / (float)(Hp * Wp);
  }
}

// Window helper: z values of the 2x2 window, first-max argmax and the max of relu(z).
struct Win {
  float y[4];
  int arg;
  float zmax;
};
template <typename TY>
__device__ __forceinline__ Win load_win(const TY* y, size_t base, int W, float sc, float sf) {
  Win w;
  w.y[0] = io<TY>::ld(y, base);
  w.y[1] = io<TY>::ld(y, base + 1);
  w.y[2] = io<TY>::ld(y, base + W);
  w.y[3] = io<TY>::ld(y, base + W + 1);
  // max over relu(z) with first-max tie-break in row-major window order (scan with '>')
  float best = fmaxf(fmaf(w.y[0], sc, sf), 0.f);
  int arg = 0;
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const float r = fmaxf(fmaf(w.y[k], sc, sf), 0.f);
    if (r > best) { best = r; arg = k; }
  }
  w.arg = arg;
  w.zmax = best;
  return w;
}

template <typename TG>
__device__ __forceinline__ float gout_at(const TG* gout, int pool_mode, long long nc, int q, int HpWp) {
  if (pool_mode == 0) return io<TG>::ld(gout, (size_t)nc * HpWp + q);
  return reinterpret_cast<const float*>(gout)[nc] / (float)HpWp;
}

// ----------------------------------------------------------------------------- backward reduce
template <typename TY, typename TG>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const TY* __restrict__ y, const TG* __restrict__ gout, int pool_mode,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ parts,
    int N, int B, int C, int H, int W) {
  const int Hp = H / 2, Wp = W / 2, HpWp = Hp * Wp;
  const long long nc = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (nc >= (long long)N * C) return;
  const int c = (int)(nc % C), n = (int)(nc / C), g = n / B;
  const float sc = scale[g * C + c], sf = shift[g * C + c];
  const float mu = mean[g * C + c], is = invstd[g * C + c];
  float s1 = 0.f, s2 = 0.f;
  for (int q = lane; q < HpWp; q += 64) {
    const int hp = q / Wp, wp = q % Wp;
    const Win w = load_win<TY>(y, ((size_t)nc * H + 2 * hp) * W + 2 * wp, W, sc, sf);
    if (w.zmax > 0.f) {
      const float d = gout_at<TG>(gout, pool_mode, nc, q, HpWp);
      s1 += d;
      s2 += d * (w.y[w.arg] - mu) * is;
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    parts[((size_t)c * N + n) * 2] = s1;
    parts[((size_t)c * N + n) * 2 + 1] = s2;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(
    const float* __restrict__ parts, int G, int R, int C, long long count,
    const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ invstd, float* coef, float* dgamma, float* dbeta, float* dbias,
    int accumulate) {
  __shared__ double sh1[512], sh2[512];
  const int c = blockIdx.x;
  group_sums(parts, G, R, c, sh1, sh2);
  if (threadIdx.x != 0) return;
  double dg = 0.0, db = 0.0, dbi = 0.0;
  const double n = (double)count;
  for (int g = 0; g < G; ++g) {
    const double s1 = sh1[256 + g], s2 = sh2[256 + g];
    const double is = invstd[g * C + c], mu = mean[g * C + c], ga = gamma[c];
    const double k1 = ga * is;
    const double kx = -ga * is * is * s2 / n;
    const double k0 = -ga * is * s1 / n + ga * is * is * mu * s2 / n;
    coef[(g * C + c) * 3 + 0] = (float)k1;
    coef[(g * C + c) * 3 + 1] = (float)kx;
    coef[(g * C + c) * 3 + 2] = (float)k0;
    dg += s2;
    db += s1;
    dbi += k1 * s1 + kx * mu * n + k0 * n;  // = sum of dy over the group (analytically 0)
  }
  if (dgamma) dgamma[c] = (float)(accumulate ? dgamma[c] + dg : dg);
  if (dbeta) dbeta[c] = (float)(accumulate ? dbeta[c] + db : db);
  if (dbias) dbias[c] = (float)(accumulate ? dbias[c] + dbi : dbi);
}

template <typename TY, typename TG, typename TD>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const TY* __restrict__ y, const TG* __restrict__ gout, int pool_mode,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ coef, TD* __restrict__ dy, long long total, int B, int C, int H,
    int W) {
  const int Hp = H / 2, Wp = W / 2, HpWp = Hp * Wp;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;  // windows incl. floor-mode leftovers
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int wc = (int)(i % Wc);
    const int hc = (int)((i / Wc) % Hc);
    const long long nc = i / ((long long)Hc * Wc);
    const int c = (int)(nc % C), n = (int)(nc / C), g = n / B;
    const float sc = scale[g * C + c], sf = shift[g * C + c];
    const float k1 = coef[(g * C + c) * 3], kx = coef[(g * C + c) * 3 + 1],
                k0 = coef[(g * C + c) * 3 + 2];
    const int h0 = 2 * hc, w0 = 2 * wc;
    const size_t base = ((size_t)nc * H + h0) * W + w0;
    if (hc < Hp && wc < Wp) {
      const Win w = load_win<TY>(y, base, W, sc, sf);
      const float d = w.zmax > 0.f ? gout_at<TG>(gout, pool_mode, nc, hc * Wp + wc, HpWp) : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float dz = (k == w.arg) ? d : 0.f;
        const size_t o = base + (k >> 1) * W + (k & 1);
        io<TD>::st(dy, o, fmaf(k1, dz, fmaf(kx, w.y[k], k0)));
      }
    } else {  // incomplete window (odd H/W): no gradient flows through pooling
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
          if (h0 + a < H && w0 + b < W) {
            const size_t o = base + a * W + b;
            io<TD>::st(dy, o, fmaf(kx, io<TY>::ld(y, o), k0));
          }
    }
  }
}

// ----------------------------------------------------------------------------- bf16 x4 paths
// bf16 maps whose row width is a multiple of 8: one thread handles 4 consecutive pooling
// windows of an output row -> two 16-byte loads of y (the two input rows), 8-byte gradient
// loads/stores.  (f32 maps and other widths take the scalar kernels above.)
typedef __attribute__((ext_vector_type(4))) unsigned u4v;
typedef __attribute__((ext_vector_type(2))) unsigned u2v;

__device__ __forceinline__ void unpack8(u4v v, float (&f)[8]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return pack_bf16x2(a, b);
}

// per window k = 0..3 of the quad: first-max argmax over relu(z) and the max
__device__ __forceinline__ void quad_windows(const float (&r0)[8], const float (&r1)[8], float sc,
                                             float sf, int (&arg)[4], float (&mx)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v[4] = {r0[2 * k], r0[2 * k + 1], r1[2 * k], r1[2 * k + 1]};
    float best = fmaxf(fmaf(v[0], sc, sf), 0.f);
    int a = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const float r = fmaxf(fmaf(v[j], sc, sf), 0.f);
      if (r > best) { best = r; a = j; }
    }
    arg[k] = a;
    mx[k] = best;
  }
}

__global__ __launch_bounds__(256) void bn_relu_pool_q4_kernel(
    const bf16* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    bf16* __restrict__ out, long long total4, int B, int C, int H, int W) {
  const int Hp = H / 2, Wp = W / 2, Q = Wp / 4;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const int q = (int)(i % Q);
    const int hp = (int)((i / Q) % Hp);
    const long long nc = i / ((long long)Q * Hp);
    const int c = (int)(nc % C), g = (int)(nc / C) / B;
    const float sc = scale[g * C + c], sf = shift[g * C + c];
    const size_t base = ((size_t)nc * H + 2 * hp) * W + 8 * q;
    float r0[8], r1[8];
    unpack8(*reinterpret_cast<const u4v*>(y + base), r0);
    unpack8(*reinterpret_cast<const u4v*>(y + base + W), r1);
    int arg[4];
    float mx[4];
    quad_windows(r0, r1, sc, sf, arg, mx);
    *reinterpret_cast<u2v*>(out + ((size_t)nc * Hp + hp) * Wp + 4 * q) =
        u2v{pack2(mx[0], mx[1]), pack2(mx[2], mx[3])};
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_q4_kernel(
    const bf16* __restrict__ y, const bf16* __restrict__ gout, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, float* __restrict__ parts, int N, int B, int C, int H, int W) {
  const int Hp = H / 2, Wp = W / 2, Q = Wp / 4, HQ = Hp * Q;
  const long long nc = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (nc >= (long long)N * C) return;
  const int c = (int)(nc % C), n = (int)(nc / C), g = n / B;
  const float sc = scale[g * C + c], sf = shift[g * C + c];
  const float mu = mean[g * C + c], is = invstd[g * C + c];
  float s1 = 0.f, s2 = 0.f;
  const bf16* yp = y + (size_t)nc * H * W;
  const bf16* gp = gout + (size_t)nc * Hp * Wp;
  // 4 quads per lane per pass with every load issued before any math: a wave-per-plane
  // reduction is bound by load latency, not bandwidth
  for (int t0 = lane; t0 < HQ; t0 += 256) {
    u4v a0[4], a1[4];
    u2v gv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 64 * u;
      if (t < HQ) {
        const int hp = t / Q, q = t - hp * Q;
        const size_t base = (size_t)(2 * hp) * W + 8 * q;
        a0[u] = *reinterpret_cast<const u4v*>(yp + base);
        a1[u] = *reinterpret_cast<const u4v*>(yp + base + W);
        gv[u] = *reinterpret_cast<const u2v*>(gp + (size_t)hp * Wp + 4 * q);
      } else {   // zero gradient: contributes nothing
        a0[u] = u4v{0u, 0u, 0u, 0u};
        a1[u] = u4v{0u, 0u, 0u, 0u};
        gv[u] = u2v{0u, 0u};
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float r0[8], r1[8];
      unpack8(a0[u], r0);
      unpack8(a1[u], r1);
      const float gg[4] = {__uint_as_float(gv[u].x << 16), __uint_as_float(gv[u].x & 0xffff0000u),
                           __uint_as_float(gv[u].y << 16), __uint_as_float(gv[u].y & 0xffff0000u)};
      int arg[4];
      float mx[4];
      quad_windows(r0, r1, sc, sf, arg, mx);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int a = arg[k];   // selects, not a runtime register index
        const float ya = a == 0 ? r0[2 * k] : a == 1 ? r0[2 * k + 1] : a == 2 ? r1[2 * k] : r1[2 * k + 1];
        const float gk = mx[k] > 0.f ? gg[k] : 0.f;
        s1 += gk;
        s2 += gk * (ya - mu) * is;
      }
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    parts[((size_t)c * N + n) * 2] = s1;
    parts[((size_t)c * N + n) * 2 + 1] = s2;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_q4_kernel(
    const bf16* __restrict__ y, const bf16* __restrict__ gout, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, bf16* __restrict__ dy,
    long long total4, int B, int C, int H, int W) {
  const int Hp = H / 2, Wp = W / 2, Q = Wp / 4;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const int q = (int)(i % Q);
    const int hp = (int)((i / Q) % Hp);
    const long long nc = i / ((long long)Q * Hp);
    const int c = (int)(nc % C), g = (int)(nc / C) / B;
    const float sc = scale[g * C + c], sf = shift[g * C + c];
    const float k1 = coef[(g * C + c) * 3], kx = coef[(g * C + c) * 3 + 1],
                k0 = coef[(g * C + c) * 3 + 2];
    const size_t base = ((size_t)nc * H + 2 * hp) * W + 8 * q;
    float r0[8], r1[8];
    unpack8(*reinterpret_cast<const u4v*>(y + base), r0);
    unpack8(*reinterpret_cast<const u4v*>(y + base + W), r1);
    const u2v gv = *reinterpret_cast<const u2v*>(gout + ((size_t)nc * Hp + hp) * Wp + 4 * q);
    const float gg[4] = {__uint_as_float(gv.x << 16), __uint_as_float(gv.x & 0xffff0000u),
                         __uint_as_float(gv.y << 16), __uint_as_float(gv.y & 0xffff0000u)};
    int arg[4];
    float mx[4];
    quad_windows(r0, r1, sc, sf, arg, mx);
    float d0[8], d1[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = mx[k] > 0.f ? gg[k] : 0.f;
      d0[2 * k] = fmaf(k1, arg[k] == 0 ? d : 0.f, fmaf(kx, r0[2 * k], k0));
      d0[2 * k + 1] = fmaf(k1, arg[k] == 1 ? d : 0.f, fmaf(kx, r0[2 * k + 1], k0));
      d1[2 * k] = fmaf(k1, arg[k] == 2 ? d : 0.f, fmaf(kx, r1[2 * k], k0));
      d1[2 * k + 1] = fmaf(k1, arg[k] == 3 ? d : 0.f, fmaf(kx, r1[2 * k + 1], k0));
    }
    *reinterpret_cast<u4v*>(dy + base) =
        u4v{pack2(d0[0], d0[1]), pack2(d0[2], d0[3]), pack2(d0[4], d0[5]), pack2(d0[6], d0[7])};
    *reinterpret_cast<u4v*>(dy + base + W) =
        u4v{pack2(d1[0], d1[1]), pack2(d1[2], d1[3]), pack2(d1[4], d1[5]), pack2(d1[6], d1[7])};
  }
}

// ----------------------------------------------------------------------------- BN1d / dense
constexpr int CS_ROWS = 64;

// Shifted sums: every partial is taken about the pivot K = x[first row of the group][c]
// (stored in pivot[g, c] for avd_bn_finalize), so var = E[(x-K)^2] - E[x-K]^2 does not cancel
// when |mean| >> std (BatchNorm1d over ReLU'd, pooled encoder features).
__global__ __launch_bounds__(256) void colstats_kernel(const float* __restrict__ x, int rpg, int G,
                                                       int C, int R, float* __restrict__ parts,
                                                       float* __restrict__ pivot) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y, g = blockIdx.z;
  if (c >= C) return;
  const int r0 = r * CS_ROWS, r1 = min(rpg, r0 + CS_ROWS);
  const float K = pivot ? x[(size_t)g * rpg * C + c] : 0.f;
  if (pivot && r == 0) pivot[(size_t)g * C + c] = K;
  float s = 0.f, q = 0.f;
  for (int row = r0; row < r1; ++row) {
    const float v = x[((size_t)g * rpg + row) * C + c] - K;
    s += v;
    q += v * v;
  }
  float* p = parts + (((size_t)c * G + g) * R + r) * 2;
  p[0] = s;
  p[1] = q;
}

__global__ __launch_bounds__(256) void bn1d_bwd_reduce_kernel(
    const float* __restrict__ x, const float* __restrict__ dz, const float* __restrict__ mean,
    const float* __restrict__ invstd, int rpg, int G, int C, int R, float* __restrict__ parts) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y, g = blockIdx.z;
  if (c >= C) return;
  const float mu = mean[g * C + c], is = invstd[g * C + c];
  const int r0 = r * CS_ROWS, r1 = min(rpg, r0 + CS_ROWS);
  float s1 = 0.f, s2 = 0.f;
  for (int row = r0; row < r1; ++row) {
    const size_t o = ((size_t)g * rpg + row) * C + c;
    const float d = dz[o];
    s1 += d;
    s2 += d * (x[o] - mu) * is;
  }
  float* p = parts + (((size_t)c * G + g) * R + r) * 2;
  p[0] = s1;
  p[1] = s2;
}

__global__ __launch_bounds__(256) void bn1d_bwd_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ dz, const float* __restrict__ coef,
    float* __restrict__ dx, long long total, int rpg, int C) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int g = (int)(i / C / rpg);
    const float* k = coef + (g * C + c) * 3;
    dx[i] = fmaf(k[0], dz[i], fmaf(k[1], x[i], k[2]));
  }
}

__device__ __forceinline__ float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_d(float z) {
  return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * expf(-0.5f * z * z);
}

__global__ __launch_bounds__(256) void act_fwd_kernel(
    const float* __restrict__ x, float* __restrict__ out, int act, const float* __restrict__ scale,
    const float* __restrict__ shift, long long total, int rpg, int C, float p,
    unsigned long long seed, const unsigned long long* __restrict__ seed_off) {
  if (seed_off) seed += seed_off[0];
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    float v = x[i];
    if (act == 0) {
      v = fmaxf(v, 0.f);
    } else {
      const int c = (int)(i % C);
      const int g = (int)(i / C / rpg);
      v = gelu_f(fmaf(v, scale[g * C + c], shift[g * C + c]));
    }
    out[i] = v * dropout_scale(seed, (unsigned long long)i, p);
  }
}

__global__ __launch_bounds__(256) void act_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ dout, float* __restrict__ dx, int act,
    const float* __restrict__ scale, const float* __restrict__ shift, long long total, int rpg,
    int C, float p, unsigned long long seed, const unsigned long long* __restrict__ seed_off) {
  if (seed_off) seed += seed_off[0];
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const float d = dout[i] * dropout_scale(seed, (unsigned long long)i, p);
    const float v = x[i];
    if (act == 0) {
      dx[i] = v > 0.f ? d : 0.f;
    } else {
      const int c = (int)(i % C);
      const int g = (int)(i / C / rpg);
      dx[i] = d * gelu_d(fmaf(v, scale[g * C + c], shift[g * C + c]));
    }
  }
}

// ----------------------------------------------------------------------------- reductions
// out[col] (+)= sum_rows in[row, col]; CW columns x (1024/CW) row phases per block, fixed order.
// Narrow matrices (Linear bias gradients: 256 columns x thousands of rows) use CW = 16 so 64
// phases share the rows; wide ones (conv weight-grad slabs) CW = 64.
template <int CW>
__global__ __launch_bounds__(1024) void sum_rows_kernel(const float* __restrict__ in, int rows,
                                                        int cols, long long ld,
                                                        float* __restrict__ out, int accumulate,
                                                        int rows_per_chunk) {
  // block (x, y) sums rows [y * rows_per_chunk, +rows_per_chunk) of its CW columns into row y
  // of out (leading dimension cols); a single chunk is the whole reduction
  constexpr int PH = 1024 / CW;
  __shared__ double sh[PH][CW];
  const int lc = threadIdx.x % CW, ph = threadIdx.x / CW;
  const int col = blockIdx.x * CW + lc;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(rows, r0 + rows_per_chunk);
  out += (size_t)blockIdx.y * cols;
  double s = 0.0;
  if (col < cols) {
    int r = r0 + ph;
    for (; r + 3 * PH < r1; r += 4 * PH) {
      const float a = in[(size_t)r * ld + col], b = in[(size_t)(r + PH) * ld + col];
      const float c = in[(size_t)(r + 2 * PH) * ld + col], d = in[(size_t)(r + 3 * PH) * ld + col];
      s += (double)a + (double)b + (double)c + (double)d;
    }
    for (; r < r1; r += PH) s += in[(size_t)r * ld + col];
  }
  sh[ph][lc] = s;
  __syncthreads();
  if (ph == 0 && col < cols) {
    double t = 0.0;
    for (int k = 0; k < PH; ++k) t += sh[k][lc];
    out[col] = (float)(accumulate ? out[col] + t : t);
  }
}

__global__ __launch_bounds__(1024) void sum_kernel(const float* __restrict__ in, int n, float scale,
                                                   float* out) {
  __shared__ double sh[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) s += in[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += sh[k];
    *out = (float)(t * scale);
  }
}

inline int grid_for(long long total) {
  long long b = (total + 255) / 256;
  if (b > 65536) b = 65536;
  if (b < 1) b = 1;
  return (int)b;
}

// Eval-mode BatchNorm (running statistics) as the per-channel affine the BN/ReLU/pool kernels
// apply: scale = gamma / sqrt(rv + eps), shift = beta - rm * scale (nn.BatchNorm eval mode; the
// linear probe's evaluate(), dino.py:913-947).
__global__ void bn_eval_coef_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                    const float* __restrict__ rm, const float* __restrict__ rv,
                                    float eps, int C, float* __restrict__ scale,
                                    float* __restrict__ shift) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const double sc = (double)gamma[c] / sqrt((double)rv[c] + (double)eps);
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - (double)rm[c] * sc);
}

}  // namespace

extern "C" {

int avd_bn_finalize(float* parts, int G, int R, int C, long long count, const float* gamma,
                    const float* beta, float eps, float momentum, float* mean, float* invstd,
                    float* scale, float* shift, float* running_mean, float* running_var,
                    const float* pivot, void* stream) {
  if (!parts || !gamma || !beta || !mean || !invstd || !scale || !shift) return AVD_ERR_ARG;
  if (G <= 0 || R <= 0 || C <= 0 || count <= 1) return AVD_ERR_SHAPE;
  if ((running_mean == nullptr) != (running_var == nullptr)) return AVD_ERR_ARG;
  hipStream_t st = avd_stream(stream);
  // single pass (one block per channel reads all G*R rows of its channel) only on request
  // (AVDINO_FIN1_ROWS = max G*R): A/B on the config-2 step, 2048 vs 0 (two-pass always) was
  // within noise with two-pass ahead (6.42-6.46 vs 6.46-6.48 ms), so two-pass is the default
  static const long long fin1_rows =
      getenv("AVDINO_FIN1_ROWS") ? atoll(getenv("AVDINO_FIN1_ROWS")) : 0;
  if (G <= 256 && R <= FIN1_MAXROWS && (long long)G * R <= fin1_rows) {
    bn_finalize1_kernel<<<C, 256, 0, st>>>(parts, G, R, C, count, gamma, beta, eps, momentum, mean,
                                           invstd, scale, shift, running_mean, running_var, pivot);
    AVD_CHECK_LAUNCH();
    return AVD_OK;
  }
  // ~2048 partial rows per block, >= 2 rows per chunk (room for the in-place doubles)
  int S = 0, chunk = 1;
  if (R >= 2) {
    chunk = std::max(2, avd_cdiv(R, std::min(avd_cdiv(R, 2048), 1024)));
    S = R / chunk;
    bn_stats_partial_kernel<<<dim3(S, G, C), 256, 0, st>>>(parts, G, R, S, chunk);
  }
  bn_finalize_kernel<<<avd_cdiv(C, 64), 64, 0, st>>>(parts, G, R, C, S, chunk, count, gamma, beta,
                                                    eps, momentum, mean, invstd, scale, shift,
                                                    running_mean, running_var, pivot);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_bn_relu_pool(const void* y, int ydt, const float* scale, const float* shift, void* out,
                     int odt, int pool_mode, int N, int B, int C, int H, int W, void* stream) {
  if (!y || !scale || !shift || !out) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || N % B || H < 2 || W < 2) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
  if (pool_mode == 0 && ydt == AVD_BF16 && odt == AVD_BF16 && W % 8 == 0 && H % 2 == 0) {
    const long long total4 = (long long)N * C * (H / 2) * (W / 8);
    bn_relu_pool_q4_kernel<<<grid_for(total4), 256, 0, st>>>((const bf16*)y, scale, shift,
                                                             (bf16*)out, total4, B, C, H, W);
  } else if (pool_mode == 0) {
    const long long total = (long long)N * C * (H / 2) * (W / 2);
#define AVD_P(TY, TO)                                                                     \
  bn_relu_pool_kernel<TY, TO><<<grid_for(total), 256, 0, st>>>((const TY*)y, scale, shift, \
                                                              (TO*)out, total, B, C, H, W);
    if (ydt == AVD_F32 && odt == AVD_F32) { AVD_P(float, float) }
    else if (ydt == AVD_F32 && odt == AVD_BF16) { AVD_P(float, bf16) }
    else if (ydt == AVD_BF16 && odt == AVD_BF16) { AVD_P(bf16, bf16) }
    else if (ydt == AVD_BF16 && odt == AVD_F32) { AVD_P(bf16, float) }
    else return AVD_ERR_DTYPE;
#undef AVD_P
  } else if (pool_mode == 1) {
    if (odt != AVD_F32) return AVD_ERR_DTYPE;
    const long long total = (long long)N * C;
    if (ydt == AVD_F32)
      bn_relu_pool_gap_kernel<float><<<grid_for(total), 256, 0, st>>>((const float*)y, scale, shift,
                                                                      (float*)out, total, B, C, H, W);
    else if (ydt == AVD_BF16)
      bn_relu_pool_gap_kernel<bf16><<<grid_for(total), 256, 0, st>>>((const bf16*)y, scale, shift,
                                                                     (float*)out, total, B, C, H, W);
    else return AVD_ERR_DTYPE;
  } else {
    return AVD_ERR_ARG;
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_bn_bwd_reduce(const void* y, int ydt, const void* gout, int gdt, int pool_mode,
                      const float* scale, const float* shift, const float* mean,
                      const float* invstd, float* parts, int N, int B, int C, int H, int W,
                      void* stream) {
  if (!y || !gout || !scale || !shift || !mean || !invstd || !parts) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || N % B || (pool_mode != 0 && pool_mode != 1)) return AVD_ERR_SHAPE;
  if (pool_mode == 1 && gdt != AVD_F32) return AVD_ERR_DTYPE;
  hipStream_t st = avd_stream(stream);
  const int grid = avd_cdiv((long long)N * C, 4);
  if (pool_mode == 0 && ydt == AVD_BF16 && gdt == AVD_BF16 && W % 8 == 0 && H % 2 == 0) {
    bn_bwd_reduce_q4_kernel<<<grid, 256, 0, st>>>((const bf16*)y, (const bf16*)gout, scale, shift,
                                                  mean, invstd, parts, N, B, C, H, W);
    AVD_CHECK_LAUNCH();
    return AVD_OK;
  }
#define AVD_R(TY, TG)                                                                         \
  bn_bwd_reduce_kernel<TY, TG><<<grid, 256, 0, st>>>((const TY*)y, (const TG*)gout, pool_mode, \
                                                     scale, shift, mean, invstd, parts, N, B,  \
                                                     C, H, W);
  if (ydt == AVD_F32 && gdt == AVD_F32) { AVD_R(float, float) }
  else if (ydt == AVD_BF16 && gdt == AVD_BF16) { AVD_R(bf16, bf16) }
  else if (ydt == AVD_BF16 && gdt == AVD_F32) { AVD_R(bf16, float) }
  else if (ydt == AVD_F32 && gdt == AVD_BF16) { AVD_R(float, bf16) }
  else return AVD_ERR_DTYPE;
#undef AVD_R
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_bn_bwd_finalize(const float* parts, int G, int R, int C, long long count,
                        const float* gamma, const float* mean, const float* invstd, float* coef,
                        float* dgamma, float* dbeta, float* dbias, int accumulate, void* stream) {
  if (!parts || !gamma || !mean || !invstd || !coef) return AVD_ERR_ARG;
  if (G <= 0 || G > 256 || R <= 0 || C <= 0 || count <= 0) return AVD_ERR_SHAPE;
  bn_bwd_finalize_kernel<<<C, 256, 0, avd_stream(stream)>>>(parts, G, R, C, count, gamma, mean,
                                                             invstd, coef, dgamma, dbeta, dbias,
                                                             accumulate);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_bn_bwd_apply(const void* y, int ydt, const void* gout, int gdt, int pool_mode,
                     const float* scale, const float* shift, const float* coef, void* dy, int dt,
                     int N, int B, int C, int H, int W, void* stream) {
  if (!y || !gout || !scale || !shift || !coef || !dy) return AVD_ERR_ARG;
  if (N <= 0 || B <= 0 || N % B || (pool_mode != 0 && pool_mode != 1)) return AVD_ERR_SHAPE;
  if (pool_mode == 1 && gdt != AVD_F32) return AVD_ERR_DTYPE;
  hipStream_t st = avd_stream(stream);
  if (pool_mode == 0 && ydt == AVD_BF16 && gdt == AVD_BF16 && dt == AVD_BF16 && W % 8 == 0 &&
      H % 2 == 0) {
    const long long total4 = (long long)N * C * (H / 2) * (W / 8);
    bn_bwd_apply_q4_kernel<<<grid_for(total4), 256, 0, st>>>((const bf16*)y, (const bf16*)gout, scale,
                                                             shift, coef, (bf16*)dy, total4, B, C, H,
                                                             W);
    AVD_CHECK_LAUNCH();
    return AVD_OK;
  }
  const long long total = (long long)N * C * ((H + 1) / 2) * ((W + 1) / 2);
#define AVD_A(TY, TG, TD)                                                                       \
  bn_bwd_apply_kernel<TY, TG, TD><<<grid_for(total), 256, 0, st>>>(                            \
      (const TY*)y, (const TG*)gout, pool_mode, scale, shift, coef, (TD*)dy, total, B, C, H, W);
  if (ydt == AVD_F32 && gdt == AVD_F32 && dt == AVD_F32) { AVD_A(float, float, float) }
  else if (ydt == AVD_BF16 && gdt == AVD_BF16 && dt == AVD_BF16) { AVD_A(bf16, bf16, bf16) }
  else if (ydt == AVD_BF16 && gdt == AVD_F32 && dt == AVD_BF16) { AVD_A(bf16, float, bf16) }
  else if (ydt == AVD_F32 && gdt == AVD_BF16 && dt == AVD_F32) { AVD_A(float, bf16, float) }
  else return AVD_ERR_DTYPE;
#undef AVD_A
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_colstats_parts(int rows_per_group) { return avd_cdiv(rows_per_group, CS_ROWS); }

int avd_colstats(const float* x, int rows, int G, int C, float* parts, float* pivot,
                 void* stream) {
  if (!x || !parts) return AVD_ERR_ARG;
  if (rows <= 0 || G <= 0 || rows % G || C <= 0) return AVD_ERR_SHAPE;
  const int rpg = rows / G, R = avd_colstats_parts(rpg);
  dim3 grid(avd_cdiv(C, 256), R, G);
  colstats_kernel<<<grid, 256, 0, avd_stream(stream)>>>(x, rpg, G, C, R, parts, pivot);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_act_fwd_dev(const float* x, float* out, int act, const float* scale, const float* shift,
                    int rows, int G, int C, float p, unsigned long long seed,
                    const unsigned long long* seed_off, void* stream) {
  if (!x || !out || (act == 1 && (!scale || !shift)) || (act != 0 && act != 1)) return AVD_ERR_ARG;
  if (rows <= 0 || G <= 0 || rows % G || p < 0.f || p >= 1.f) return AVD_ERR_SHAPE;
  const long long total = (long long)rows * C;
  act_fwd_kernel<<<grid_for(total), 256, 0, avd_stream(stream)>>>(x, out, act, scale, shift, total,
                                                                  rows / G, C, p, seed, seed_off);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_act_fwd(const float* x, float* out, int act, const float* scale, const float* shift,
                int rows, int G, int C, float p, unsigned long long seed, void* stream) {
  return avd_act_fwd_dev(x, out, act, scale, shift, rows, G, C, p, seed, nullptr, stream);
}

int avd_act_bwd_dev(const float* x, const float* dout, float* dx, int act, const float* scale,
                    const float* shift, int rows, int G, int C, float p, unsigned long long seed,
                    const unsigned long long* seed_off, void* stream) {
  if (!x || !dout || !dx || (act == 1 && (!scale || !shift)) || (act != 0 && act != 1))
    return AVD_ERR_ARG;
  if (rows <= 0 || G <= 0 || rows % G || p < 0.f || p >= 1.f) return AVD_ERR_SHAPE;
  const long long total = (long long)rows * C;
  act_bwd_kernel<<<grid_for(total), 256, 0, avd_stream(stream)>>>(x, dout, dx, act, scale, shift,
                                                                  total, rows / G, C, p, seed,
                                                                  seed_off);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_act_bwd(const float* x, const float* dout, float* dx, int act, const float* scale,
                const float* shift, int rows, int G, int C, float p, unsigned long long seed,
                void* stream) {
  return avd_act_bwd_dev(x, dout, dx, act, scale, shift, rows, G, C, p, seed, nullptr, stream);
}

int avd_bn1d_bwd_reduce(const float* x, const float* dz, const float* mean, const float* invstd,
                        int rows, int G, int C, float* parts, void* stream) {
  if (!x || !dz || !mean || !invstd || !parts) return AVD_ERR_ARG;
  if (rows <= 0 || G <= 0 || rows % G) return AVD_ERR_SHAPE;
  const int rpg = rows / G, R = avd_colstats_parts(rpg);
  dim3 grid(avd_cdiv(C, 256), R, G);
  bn1d_bwd_reduce_kernel<<<grid, 256, 0, avd_stream(stream)>>>(x, dz, mean, invstd, rpg, G, C, R,
                                                               parts);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_bn1d_bwd_apply(const float* x, const float* dz, const float* coef, float* dx, int rows,
                       int G, int C, void* stream) {
  if (!x || !dz || !coef || !dx) return AVD_ERR_ARG;
  if (rows <= 0 || G <= 0 || rows % G) return AVD_ERR_SHAPE;
  const long long total = (long long)rows * C;
  bn1d_bwd_apply_kernel<<<grid_for(total), 256, 0, avd_stream(stream)>>>(x, dz, coef, dx, total,
                                                                         rows / G, C);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

static void launch_sum_rows(const float* in, int rows, int cols, long long ld, float* out,
                            int accumulate, int chunks, hipStream_t st) {
  const int rpc = avd_cdiv(rows, chunks);
  if (cols <= 2048)
    sum_rows_kernel<16><<<dim3(avd_cdiv(cols, 16), chunks), 1024, 0, st>>>(in, rows, cols, ld, out,
                                                                          accumulate, rpc);
  else
    sum_rows_kernel<64><<<dim3(avd_cdiv(cols, 64), chunks), 1024, 0, st>>>(in, rows, cols, ld, out,
                                                                          accumulate, rpc);
}

int avd_sum_rows(const float* in, int rows, int cols, long long ld, float* out, int accumulate,
                 void* stream) {
  if (!in || !out) return AVD_ERR_ARG;
  if (rows <= 0 || cols <= 0 || ld < cols) return AVD_ERR_SHAPE;
  launch_sum_rows(in, rows, cols, ld, out, accumulate, 1, avd_stream(stream));
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// Row chunks for avd_sum_rows_split (inputs of >= 2^20 elements): enough blocks to cover the
// chip (>= 1024) with >= 4 row phases of work per thread; 1 = no split.  A function of the shape only, so the summation
// order (and the result) is the same on every device.
int avd_sum_rows_chunks(int rows, int cols) {
  // small inputs: one launch (a second one costs more than the single pass takes)
  if (rows <= 0 || cols <= 0 || (long long)rows * cols < (1ll << 20)) return 1;
  const int cw = cols <= 2048 ? 16 : 64, ph = 1024 / cw;
  const int cb = avd_cdiv(cols, cw);
  const int want = avd_cdiv(1024, cb), most = rows / (4 * ph);
  const int c = want < most ? want : most;
  return c > 1 ? c : 1;
}

int avd_sum_rows_split(const float* in, int rows, int cols, long long ld, float* out,
                       int accumulate, float* work, long long work_elems, void* stream) {
  if (!in || !out) return AVD_ERR_ARG;
  if (rows <= 0 || cols <= 0 || ld < cols) return AVD_ERR_SHAPE;
  const int chunks = avd_sum_rows_chunks(rows, cols);
  hipStream_t st = avd_stream(stream);
  if (chunks == 1) {
    launch_sum_rows(in, rows, cols, ld, out, accumulate, 1, st);
  } else {
    if (!work || work_elems < (long long)chunks * cols) return AVD_ERR_ARG;
    launch_sum_rows(in, rows, cols, ld, work, 0, chunks, st);        // chunk partials
    launch_sum_rows(work, chunks, cols, cols, out, accumulate, 1, st);   // fixed-order total
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_bn_eval_coef(const float* gamma, const float* beta, const float* running_mean,
                     const float* running_var, float eps, int C, float* scale, float* shift,
                     void* stream) {
  if (!gamma || !beta || !running_mean || !running_var || !scale || !shift) return AVD_ERR_ARG;
  if (C <= 0) return AVD_ERR_SHAPE;
  bn_eval_coef_kernel<<<avd_cdiv(C, 256), 256, 0, avd_stream(stream)>>>(
      gamma, beta, running_mean, running_var, eps, C, scale, shift);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_sum(const float* in, int n, float scale, float* out, void* stream) {
  if (!in || !out) return AVD_ERR_ARG;
  if (n <= 0) return AVD_ERR_SHAPE;
  sum_kernel<<<1, 1024, 0, avd_stream(stream)>>>(in, n, scale, out);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
