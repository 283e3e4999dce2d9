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
#include <cstdlib>

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

// the pivot a producer subtracted (non-finite pivots are taken as 0 there, conv_ws.hip)
__device__ __forceinline__ float pivot_of(const float* pivot, size_t i) {
  const float k = pivot[i];
  return isfinite(k) ? k : 0.f;
}

__global__ __launch_bounds__(64) void bn_finalize_kernel(
    const float* __restrict__ parts, int G, int R, int C, int S, int chunk, long long count,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* mean_o, float* invstd_o, float* scale_o, float* shift_o, float* rm, float* rv,
    const float* pivot, int pivot_gs) {
  // pivot may alias rm (the running mean as the pivot): every element is read by the thread that
  // writes it, before the write -- hence no __restrict__ on either
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
    const double mean = (pivot ? (double)pivot_of(pivot, (size_t)g * pivot_gs + c) : 0.0) + ms;
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
    const float* pivot, int pivot_gs) {
  __shared__ double sh1[512], sh2[512];
  const int c = blockIdx.x;
  group_sums(parts, G, R, c, sh1, sh2);
  if (threadIdx.x != 0) return;
  double rmean = rm ? (double)rm[c] : 0.0, rvar = rv ? (double)rv[c] : 0.0;
  const double n = (double)count;
  for (int g = 0; g < G; ++g) {
    const double ms = sh1[256 + g] / n;
    const double mean = (pivot ? (double)pivot_of(pivot, (size_t)g * pivot_gs + c) : 0.0) + ms;
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

// ----------------------------------------------------------------------------- BN1d / dense
// rows per partial of the column reductions: 16 keeps ~4 blocks per CU busy at the heads' shapes
// ([6144, 512] per call; 64 rows per thread left the loop latency-bound, ~20 us per launch)
constexpr int CS_ROWS = 16;

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
#pragma unroll 16
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
#pragma unroll 16
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

__device__ __forceinline__ float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_d(float z) {
  return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * expf(-0.5f * z * z);
}

// act_bwd_kernel (act 1) + bn1d_bwd_reduce_kernel in one pass over the same grid as the reduce:
// a thread owns column c of a CS_ROWS row chunk, forms dz exactly as act_bwd_kernel does (same
// dropout hash of the flat index, same GELU derivative), stores it and folds it into the
// chunk's partials in row order as bn1d_bwd_reduce_kernel does.
__global__ __launch_bounds__(256) void bn1d_act_bwd_reduce_kernel(
    const float* __restrict__ x, const float* __restrict__ dout, float* __restrict__ dz,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd, int rpg, int G, int C, int R,
    float p, unsigned long long seed, const unsigned long long* __restrict__ seed_off,
    float* __restrict__ parts) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y, g = blockIdx.z;
  if (c >= C) return;
  if (seed_off) seed += seed_off[0];
  const float sc = scale[g * C + c], sf = shift[g * C + c];
  const float mu = mean[g * C + c], is = invstd[g * C + c];
  const int r0 = r * CS_ROWS, r1 = min(rpg, r0 + CS_ROWS);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int row = r0; row < r1; ++row) {
    const size_t o = ((size_t)g * rpg + row) * C + c;
    const float v = x[o];
    const float d = dout[o] * dropout_scale(seed, (unsigned long long)o, p) * gelu_d(fmaf(v, sc, sf));
    dz[o] = d;
    s1 += d;
    s2 += d * (v - mu) * is;
  }
  float* q = parts + (((size_t)c * G + g) * R + r) * 2;
  q[0] = s1;
  q[1] = s2;
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

// The 16-byte path of sum_rows_kernel (cols and ld multiples of 4, 16-byte aligned in / out):
// each lane owns 4 consecutive columns (one global_load_dwordx4 per row), CQ lanes per row phase
// and 256 / CQ phases per block; a phase sums its rows in double, row order, 4 rows' loads in
// flight, then thread (0, lane) folds the phases in phase order.  Fixed order, deterministic.
// 256-thread blocks: the slab reductions run beside the other streams' kernels, and a
// 1024-thread block waits for a CU with 16 free wave slots (the round-4 form took 50-60 us in
// the step for 6.5-52 MB)
template <int CQ>
__global__ __launch_bounds__(256) void sum_rows4_kernel(const float* __restrict__ in, int rows,
                                                        int cols, long long ld,
                                                        float* __restrict__ out, int accumulate,
                                                        int rows_per_chunk) {
  constexpr int PH = 256 / CQ;
  __shared__ double sh[PH][CQ][4];
  const int lq = threadIdx.x % CQ, ph = threadIdx.x / CQ;
  const int c = 4 * (blockIdx.x * CQ + lq);
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(rows, r0 + rows_per_chunk);
  out += (size_t)blockIdx.y * cols;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < cols) {
    const float* base = in + c;
    int r = r0 + ph;
    for (; r + 3 * PH < r1; r += 4 * PH) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(base + (size_t)(r + u * PH) * ld);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s0 += (double)v[u].x; s1 += (double)v[u].y; s2 += (double)v[u].z; s3 += (double)v[u].w;
      }
    }
    for (; r < r1; r += PH) {
      const float4 v = *reinterpret_cast<const float4*>(base + (size_t)r * ld);
      s0 += (double)v.x; s1 += (double)v.y; s2 += (double)v.z; s3 += (double)v.w;
    }
  }
  sh[ph][lq][0] = s0; sh[ph][lq][1] = s1; sh[ph][lq][2] = s2; sh[ph][lq][3] = s3;
  __syncthreads();
  if (ph == 0 && c < cols) {
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
    for (int k = 0; k < PH; ++k) {
      t0 += sh[k][lq][0]; t1 += sh[k][lq][1]; t2 += sh[k][lq][2]; t3 += sh[k][lq][3];
    }
    float4* o = reinterpret_cast<float4*>(out + c);
    if (accumulate) {
      const float4 a = *o;
      t0 += a.x; t1 += a.y; t2 += a.z; t3 += a.w;
    }
    *o = make_float4((float)t0, (float)t1, (float)t2, (float)t3);
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
                    const float* pivot, int pivot_gs, void* stream) {
  if (!parts || !gamma || !beta || !mean || !invstd || !scale || !shift) return AVD_ERR_ARG;
  if (G <= 0 || R <= 0 || C <= 0 || count <= 1) return AVD_ERR_SHAPE;
  if ((running_mean == nullptr) != (running_var == nullptr)) return AVD_ERR_ARG;
  hipStream_t st = avd_stream(stream);
  // single pass (one block per channel reads all G*R rows of its channel: one launch instead of
  // two) where it fits.  Round-4 A/B on the config-2 step (3 interleaved rounds): 5.483 vs
  // 5.516 ms for the two-pass form, which stays for larger G / R
  if (G <= 256 && R <= FIN1_MAXROWS) {
    bn_finalize1_kernel<<<C, 256, 0, st>>>(parts, G, R, C, count, gamma, beta, eps, momentum, mean,
                                           invstd, scale, shift, running_mean, running_var, pivot,
                                           pivot_gs);
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
                                                    running_mean, running_var, pivot, pivot_gs);
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

int avd_bn1d_act_bwd_reduce(const float* x, const float* dout, float* dz, const float* scale,
                            const float* shift, const float* mean, const float* invstd, int rows,
                            int G, int C, float p, unsigned long long seed,
                            const unsigned long long* seed_off, float* parts, void* stream) {
  if (!x || !dout || !dz || !scale || !shift || !mean || !invstd || !parts) return AVD_ERR_ARG;
  if (rows <= 0 || G <= 0 || rows % G || C <= 0 || p < 0.f || p >= 1.f) return AVD_ERR_SHAPE;
  const int rpg = rows / G, R = avd_colstats_parts(rpg);
  dim3 grid(avd_cdiv(C, 256), R, G);
  bn1d_act_bwd_reduce_kernel<<<grid, 256, 0, avd_stream(stream)>>>(
      x, dout, dz, scale, shift, mean, invstd, rpg, G, C, R, p, seed, seed_off, parts);
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

// columns per block of the launch sum_rows takes for this shape (the 16-byte path when cols % 4
// == 0; the chunk count, and with it the summation order, depends on the shape only)
static int sum_rows_cw(int cols) {
  if (cols % 4 == 0) return 64;            // sum_rows4_kernel<16>: 16 phases of 256 threads
  return cols <= 2048 ? 16 : 64;
}
static int sum_rows_phases(int cols) { return cols % 4 == 0 ? 16 : 1024 / sum_rows_cw(cols); }

static void launch_sum_rows(const float* in, int rows, int cols, long long ld, float* out,
                            int accumulate, int chunks, hipStream_t st) {
  const int rpc = avd_cdiv(rows, chunks);
  const bool v4 = cols % 4 == 0 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (v4)
    sum_rows4_kernel<16><<<dim3(avd_cdiv(cols, 64), chunks), 256, 0, st>>>(in, rows, cols, ld, out,
                                                                          accumulate, rpc);
  else if (cols <= 2048)
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
  const int cw = sum_rows_cw(cols), ph = sum_rows_phases(cols);
  const int cb = avd_cdiv(cols, cw);
  // >= ~512 blocks per launch: a wide slab stack (51200 columns: 800 blocks of 256 threads, 16
  // rows of 16-byte loads per thread) is one pass, narrow ones split their rows
  const int target = 512;
  const int want = avd_cdiv(target, cb), most = rows / (4 * ph);
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
