// Channels-last (NHWC) BatchNorm-apply + ReLU + 2x2 max-pool (floor mode, first-max ties) and
// its backward, for the conv blocks of CentralUnimodalImage / CentralUnimodalAudio
// (unimodal.py:127-221) and the 3x3 CNNs (dino.py:18-73, global average pool tail).
// One thread = one 16-byte channel vector (8 bf16 / 4 f32 channels) of one pooling window:
// four 16-byte loads, one 16-byte store.  Statistics are per (group = view, channel)
// (dino.py:680-704); the backward recomputes the window argmax from y, so no mask is stored.
//   mode 0: out = pooled map, NHWC, activation dtype
//   mode 1: out = global average of the pooled map, f32 [N][C]
//   mode 2: out = pooled map flattened in the reference's (c, h, w) order, f32 [N][C*Hp*Wp]
//           (the input of the encoder's Linear, dino.py:459-468)
#include <algorithm>
#include <cstdlib>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(4))) unsigned u4;

template <typename T> struct Vec;
template <> struct Vec<bf16> {
  static constexpr int V = 8;
  static __device__ __forceinline__ void ld(const bf16* p, float (&f)[8]) {
    const u4 v = *reinterpret_cast<const u4*>(p);
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void st(bf16* p, const float (&f)[8]) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
    *reinterpret_cast<u4*>(p) = u4{w[0], w[1], w[2], w[3]};
  }
};
template <> struct Vec<float> {
  static constexpr int V = 4;
  static __device__ __forceinline__ void ld(const float* p, float (&f)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  static __device__ __forceinline__ void st(float* p, const float (&f)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};

// Window (hp, wp) of sample n, channels c0..c0+V-1: the 4 pixels (0 outside the map for the
// partial windows of odd sizes), and per channel the first-max argmax of relu(z) and its value.
template <typename T>
struct Win {
  static constexpr int V = Vec<T>::V;
  float y[4][V];
  int arg[V];
  float mx[V];
  bool has[4];
};

template <typename T>
__device__ __forceinline__ void load_win(const T* __restrict__ y, size_t pix0, int W, int C,
                                         int c0, bool has_r, bool has_c, const float* sc,
                                         const float* sf, Win<T>& w) {
  constexpr int V = Vec<T>::V;
  w.has[0] = true; w.has[1] = has_c; w.has[2] = has_r; w.has[3] = has_r && has_c;
  const size_t off[4] = {pix0 * C, (pix0 + 1) * C, (pix0 + W) * C, (pix0 + W + 1) * C};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (w.has[k]) Vec<T>::ld(y + off[k] + c0, w.y[k]);
    else
#pragma unroll
      for (int e = 0; e < V; ++e) w.y[k][e] = 0.f;
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    float best = fmaxf(fmaf(w.y[0][e], sc[e], sf[e]), 0.f);
    int a = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float r = fmaxf(fmaf(w.y[k][e], sc[e], sf[e]), 0.f);
      if (w.has[k] && r > best) { best = r; a = k; }
    }
    w.arg[e] = a;
    w.mx[e] = best;
  }
}

template <int V>
__device__ __forceinline__ void load_coef(const float* __restrict__ a, int idx, float (&o)[V]) {
#pragma unroll
  for (int e = 0; e < V; ++e) o[e] = a[idx + e];
}

// ------------------------------------------------------------------------------ forward
template <typename T>
__global__ __launch_bounds__(256) void relu_pool_cl_kernel(
    const T* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    void* __restrict__ out, int mode, long long total, int B, int C, int H, int W, U32Div dcv,
    U32Div dwp, U32Div dhp) {
  constexpr int V = Vec<T>::V;
  const int Hp = H / 2, Wp = W / 2, CV = C / V;
  // total < 2^32 (host-checked): 32-bit index decomposition by exact reciprocal multiplies
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const unsigned pw = dcv.div((unsigned)i);         // pooled pixel index
    const int cv = (int)((unsigned)i - pw * CV);
    const unsigned ph = dwp.div(pw);
    const int wp = (int)(pw - ph * Wp);
    const int n = (int)dhp.div(ph), hp = (int)(ph - (unsigned)n * Hp);
    const int g = n / B, c0 = cv * V;
    float sc[V], sf[V];
    load_coef<V>(scale, g * C + c0, sc);
    load_coef<V>(shift, g * C + c0, sf);
    Win<T> w;
    load_win<T>(y, ((size_t)n * H + 2 * hp) * W + 2 * wp, W, C, c0, true, true, sc, sf, w);
    if (mode == 0) {
      Vec<T>::st(reinterpret_cast<T*>(out) + (size_t)pw * C + c0, w.mx);
    } else {   // mode 2: f32 (c, h, w) flatten
      float* o = reinterpret_cast<float*>(out) + (size_t)n * C * Hp * Wp + (size_t)hp * Wp + wp;
#pragma unroll
      for (int e = 0; e < V; ++e) o[(size_t)(c0 + e) * Hp * Wp] = w.mx[e];
    }
  }
}

// mode 1: one thread per (n, channel vector), mean over the pooled map
template <typename T>
__global__ __launch_bounds__(256) void relu_pool_gap_cl_kernel(
    const T* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    float* __restrict__ out, long long total, int B, int C, int H, int W) {
  constexpr int V = Vec<T>::V;
  const int Hp = H / 2, Wp = W / 2, CV = C / V;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cv = (int)(i % CV), n = (int)(i / CV);
    const int g = n / B, c0 = cv * V;
    float sc[V], sf[V], acc[V];
    load_coef<V>(scale, g * C + c0, sc);
    load_coef<V>(shift, g * C + c0, sf);
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int hp = 0; hp < Hp; ++hp)
      for (int wp = 0; wp < Wp; ++wp) {
        Win<T> w;
        load_win<T>(y, ((size_t)n * H + 2 * hp) * W + 2 * wp, W, C, c0, true, true, sc, sf, w);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += w.mx[e];
      }
#pragma unroll
    for (int e = 0; e < V; ++e) out[(size_t)n * C + c0 + e] = acc[e] / (float)(Hp * Wp);
  }
}

// gradient of the pooled output at window (n, hp, wp), channels c0..c0+V-1
template <typename T, int V>
__device__ __forceinline__ void load_gout(const void* __restrict__ gout, int mode, int n, int hp,
                                          int wp, int Hp, int Wp, int C, int c0, float (&gg)[V]) {
  if (mode == 0) {
    if (hp < Hp && wp < Wp) {
      Vec<T>::ld(reinterpret_cast<const T*>(gout) + (((size_t)n * Hp + hp) * Wp + wp) * C + c0, gg);
      return;
    }
  } else if (mode == 1) {
    if (hp < Hp && wp < Wp) {
      const float* p = reinterpret_cast<const float*>(gout) + (size_t)n * C + c0;
#pragma unroll
      for (int e = 0; e < V; ++e) gg[e] = p[e] / (float)(Hp * Wp);
      return;
    }
  } else {
    if (hp < Hp && wp < Wp) {
      const float* p = reinterpret_cast<const float*>(gout) + (size_t)n * C * Hp * Wp +
                       (size_t)hp * Wp + wp;
#pragma unroll
      for (int e = 0; e < V; ++e) gg[e] = p[(size_t)(c0 + e) * Hp * Wp];
      return;
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) gg[e] = 0.f;   // rows/cols the floor-mode pool never saw
}

// ------------------------------------------------------------------------------ backward
// Fixed-order fold of the block's per-thread partials sh[slot * CV + cv][2e + k] over its slots
// into parts[c][g][r][2].  When the C*2 outputs divide the block, every thread sums one
// contiguous segment of one output's slots and one thread per output adds the segments in
// order (a 32-output block used to leave 224 threads idle while 32 walked 128 slots each);
// otherwise one thread per output walks all slots.
template <int V>
__device__ __forceinline__ void fold_slots(float (*sh)[2 * V + 1], int C, int slots, float* parts,
                                           int G, int g, int R, int r) {
  const int CV = C / V, no = 2 * C;
  if (no <= 256 && 256 % no == 0) {
    __shared__ float red[256];
    const int tpo = 256 / no;
    const int o = threadIdx.x % no, q = threadIdx.x / no;
    const int c = o >> 1, k = o & 1, ocv = c / V, e = c % V;
    const int seg = (slots + tpo - 1) / tpo;
    const int s0 = q * seg, s1 = min(slots, s0 + seg);
    float t = 0.f;
    for (int s = s0; s < s1; ++s) t += sh[s * CV + ocv][2 * e + k];
    red[q * no + o] = t;
    __syncthreads();
    if ((int)threadIdx.x < no) {
      float u = 0.f;
      for (int j = 0; j < tpo; ++j) u += red[j * no + o];
      parts[(((size_t)c * G + g) * R + r) * 2 + k] = u;
    }
    return;
  }
  for (int o = threadIdx.x; o < no; o += 256) {
    const int c = o >> 1, k = o & 1;
    const int ocv = c / V, e = c % V;
    float t = 0.f;
    for (int s = 0; s < slots; ++s) t += sh[s * CV + ocv][2 * e + k];
    parts[(((size_t)c * G + g) * R + r) * 2 + k] = t;
  }
}

// Partial sums over (samples of the group, windows) per channel: parts[c][g][r][2] =
// (sum dz, sum dz * xhat) with dz the ReLU/pool-routed gradient at the window's argmax.
// Block (r, g) covers windows [r*per, (r+1)*per) of group g; thread = (window slot, vector).
template <typename T>
__global__ __launch_bounds__(256) void bwd_reduce_cl_kernel(
    const T* __restrict__ y, const void* __restrict__ gout, int mode,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ parts,
    int G, int B, int C, int H, int W, int R, long long per) {
  constexpr int V = Vec<T>::V;
  __shared__ float sh[256][2 * V + 1];
  const int Hp = H / 2, Wp = W / 2, CV = C / V;
  const int slots = 256 / CV;
  const int cv = threadIdx.x % CV, slot = threadIdx.x / CV;
  const int r = blockIdx.x, g = blockIdx.y;
  const int c0 = cv * V;
  const long long nwin = (long long)B * Hp * Wp;
  const long long w0 = r * per, w1 = std::min(nwin, w0 + per);
  float sc[V], sf[V], mu[V], is[V], s1[V], s2[V];
  load_coef<V>(scale, g * C + c0, sc);
  load_coef<V>(shift, g * C + c0, sf);
  load_coef<V>(mean, g * C + c0, mu);
  load_coef<V>(invstd, g * C + c0, is);
#pragma unroll
  for (int e = 0; e < V; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  if (slot < slots) {
    for (long long wi = w0 + slot; wi < w1; wi += slots) {
      const int wp = (int)(wi % Wp), hp = (int)((wi / Wp) % Hp);
      const int n = g * B + (int)(wi / ((long long)Wp * Hp));
      float gg[V];
      load_gout<T, V>(gout, mode, n, hp, wp, Hp, Wp, C, c0, gg);
      Win<T> w;
      load_win<T>(y, ((size_t)n * H + 2 * hp) * W + 2 * wp, W, C, c0, true, true, sc, sf, w);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int a = w.arg[e];
        const float ya = a == 0 ? w.y[0][e] : a == 1 ? w.y[1][e] : a == 2 ? w.y[2][e] : w.y[3][e];
        const float dz = w.mx[e] > 0.f ? gg[e] : 0.f;
        s1[e] += dz;
        s2[e] += dz * (ya - mu[e]) * is[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    sh[threadIdx.x][2 * e] = s1[e];
    sh[threadIdx.x][2 * e + 1] = s2[e];
  }
  __syncthreads();
  fold_slots<V>(sh, C, slots, parts, G, g, R, r);
}

// The same partial sums from the POOLED output p = max_k relu(y_k*scale + shift) (the next
// layer's input, already in memory) instead of the 4x larger conv output y: at a window's
// argmax a, z_a = gamma*xhat_a + beta = p, so where the gradient is routed (p > 0)
// xhat_a = (p - beta) / gamma.  Reads p + gout (2/4 of y's bytes) instead of y + gout.
// A channel with gamma == 0 has every z equal (= relu(beta)), so the first-max pixel is the
// window's first one: its xhat is taken from y (read only for such channels).
template <typename T>
__global__ __launch_bounds__(256) void bwd_reduce_pooled_cl_kernel(
    const T* __restrict__ y, const void* __restrict__ pooled, const void* __restrict__ gout,
    int mode, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ parts,
    int G, int B, int C, int H, int W, int R, long long per) {
  constexpr int V = Vec<T>::V;
  __shared__ float sh[256][2 * V + 1];
  const int Hp = H / 2, Wp = W / 2, CV = C / V;
  const int slots = 256 / CV;
  const int cv = threadIdx.x % CV, slot = threadIdx.x / CV;
  const int r = blockIdx.x, g = blockIdx.y;
  const int c0 = cv * V;
  const long long nwin = (long long)B * Hp * Wp;
  const long long w0 = r * per, w1 = std::min(nwin, w0 + per);
  float ig[V], be[V], mu[V], is[V], s1[V], s2[V], gs[V];
  bool any0 = false;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    // xhat = (p - beta) / gamma carries the stored p's rounding amplified by |beta / gamma|:
    // such channels (and gamma == 0) take xhat from y at the argmax instead -- bound: the
    // error stays under 8 ulps of the storage type in xhat units
    const float ga = gamma[c0 + e], bb = beta[c0 + e];
    const bool use_y = ga == 0.f || fabsf(bb) > (sizeof(T) == 2 ? 8.f : 4096.f) * fabsf(ga);
    ig[e] = use_y ? 0.f : 1.f / ga;
    gs[e] = ga > 0.f ? 1.f : (ga < 0.f ? -1.f : 0.f);
    any0 |= use_y;
    be[e] = bb;
    s1[e] = 0.f; s2[e] = 0.f;
  }
  load_coef<V>(mean, g * C + c0, mu);
  load_coef<V>(invstd, g * C + c0, is);
  if (slot < slots && mode == 0 && !any0) {
    // NHWC pooled maps: window wi of group g sits at ((g*B*Hp*Wp + wi) * C + c0) -- no index
    // division; 4 windows' loads in flight per thread, summed in the same order as below
    const size_t gbase = (size_t)g * B * Hp * Wp;
    const T* gp = reinterpret_cast<const T*>(gout) + c0;
    const T* pp = reinterpret_cast<const T*>(pooled) + c0;
    for (long long wi = w0 + slot; wi < w1; wi += 4ll * slots) {
      float gg[4][V], pv[4][V];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long long wk = wi + (long long)k * slots;
        const size_t off = (gbase + (size_t)(wk < w1 ? wk : wi)) * C;
        Vec<T>::ld(gp + off, gg[k]);
        Vec<T>::ld(pp + off, pv[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (wi + (long long)k * slots >= w1) break;
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float dz = pv[k][e] > 0.f ? gg[k][e] : 0.f;
          s1[e] += dz;
          s2[e] += dz * ((pv[k][e] - be[e]) * ig[e]);
        }
      }
    }
  } else if (slot < slots) {
    for (long long wi = w0 + slot; wi < w1; wi += slots) {
      const int wp = (int)(wi % Wp), hp = (int)((wi / Wp) % Hp);
      const int n = g * B + (int)(wi / ((long long)Wp * Hp));
      float gg[V], pv[V];
      load_gout<T, V>(gout, mode, n, hp, wp, Hp, Wp, C, c0, gg);
      load_gout<T, V>(pooled, mode, n, hp, wp, Hp, Wp, C, c0, pv);
      // y-path channels: the window's argmax of gamma * xhat + beta is the max of xhat for
      // gamma > 0, its min for gamma < 0 (first of equals); gamma == 0 makes every element
      // equal, and the forward's max keeps the first (top-left) one
      float y0[V], y1[V], y2[V], y3[V];
      if (any0) {
        const T* yw = y + (((size_t)n * H + 2 * hp) * W + 2 * wp) * C + c0;
        Vec<T>::ld(yw, y0);
        Vec<T>::ld(yw + C, y1);
        Vec<T>::ld(yw + (size_t)W * C, y2);
        Vec<T>::ld(yw + (size_t)W * C + C, y3);
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float dz = pv[e] > 0.f ? gg[e] : 0.f;
        float xh = 0.f;
        if (ig[e] != 0.f) {
          xh = (pv[e] - be[e]) * ig[e];
        } else if (any0) {
          xh = (y0[e] - mu[e]) * is[e];
          if (gs[e] != 0.f) {
            const float c1 = (y1[e] - mu[e]) * is[e], c2 = (y2[e] - mu[e]) * is[e],
                        c3 = (y3[e] - mu[e]) * is[e];
            if (gs[e] * c1 > gs[e] * xh) xh = c1;
            if (gs[e] * c2 > gs[e] * xh) xh = c2;
            if (gs[e] * c3 > gs[e] * xh) xh = c3;
          }
        }
        s1[e] += dz;
        s2[e] += dz * xh;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    sh[threadIdx.x][2 * e] = s1[e];
    sh[threadIdx.x][2 * e + 1] = s2[e];
  }
  __syncthreads();
  fold_slots<V>(sh, C, slots, parts, G, g, R, r);
}

__device__ __forceinline__ float to_f(bf16 v) { return bf2f(v); }
__device__ __forceinline__ float to_f(float v) { return v; }

// Mode 2 of the kernel above (pooled map and gradient f32 in the (c, h, w) flatten order of the
// encoder Linear's input): one wave per channel, lanes over the channel's Hp*Wp <= 64 pooled
// positions -- each sample's plane is a contiguous 4*Hp*Wp-byte run, so the loads coalesce
// (the generic path reads 8 planes 4*Hp*Wp bytes apart per thread, with 64-bit index
// divisions).  Block (r, g, channel quad): samples [r*B/R, (r+1)*B/R) of group g, same rows as
// bwd_reduce_pooled_cl_kernel.  Channels whose xhat needs y take it at the window argmax of y.
template <typename T>
__global__ __launch_bounds__(256) void bwd_reduce_pooled_m2_kernel(
    const T* __restrict__ y, const float* __restrict__ pooled, const float* __restrict__ gout,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ parts,
    int G, int B, int C, int H, int W, int R) {
  const int lane = threadIdx.x & 63, c = blockIdx.z * 4 + (threadIdx.x >> 6);
  const int r = blockIdx.x, g = blockIdx.y;
  const int Hp = H / 2, Wp = W / 2, HW = Hp * Wp;
  if (c >= C) return;
  const int n0 = g * B + (int)(((long long)r * B) / R), n1 = g * B + (int)(((long long)(r + 1) * B) / R);
  const float ga = gamma[c], bb = beta[c];
  const bool use_y = ga == 0.f || fabsf(bb) > (sizeof(T) == 2 ? 8.f : 4096.f) * fabsf(ga);
  const float ig = use_y ? 0.f : 1.f / ga, gs = ga > 0.f ? 1.f : (ga < 0.f ? -1.f : 0.f);
  const float mu = mean[g * C + c], is = invstd[g * C + c];
  float s1 = 0.f, s2 = 0.f;
  for (int p0 = 0; p0 < HW; p0 += 64) {
    const int p = p0 + lane;
    if (p >= HW) continue;
    const int hp = p / Wp, wp = p - hp * Wp;
    int n = n0;
    // 4 samples' loads in flight per lane, summed in sample order
    for (; n + 4 <= n1; n += 4) {
      float pv[4], gv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const size_t o = ((size_t)(n + k) * C + c) * HW + p;
        pv[k] = pooled[o];
        gv[k] = gout[o];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float dz = pv[k] > 0.f ? gv[k] : 0.f;
        float xh = (pv[k] - bb) * ig;
        if (use_y) {
          const T* yw = y + (((size_t)(n + k) * H + 2 * hp) * W + 2 * wp) * C + c;
          float yv[4];
          yv[0] = to_f(yw[0]); yv[1] = to_f(yw[C]);
          yv[2] = to_f(yw[(size_t)W * C]); yv[3] = to_f(yw[(size_t)W * C + C]);
          xh = (yv[0] - mu) * is;
          if (gs != 0.f)
#pragma unroll
            for (int q = 1; q < 4; ++q) {
              const float cq = (yv[q] - mu) * is;
              if (gs * cq > gs * xh) xh = cq;
            }
        }
        s1 += dz;
        s2 += dz * xh;
      }
    }
    for (; n < n1; ++n) {
      const size_t o = ((size_t)n * C + c) * HW + p;
      const float pv = pooled[o], gv = gout[o];
      const float dz = pv > 0.f ? gv : 0.f;
      float xh = (pv - bb) * ig;
      if (use_y) {
        const T* yw = y + (((size_t)n * H + 2 * hp) * W + 2 * wp) * C + c;
        float yv[4];
        yv[0] = to_f(yw[0]); yv[1] = to_f(yw[C]);
        yv[2] = to_f(yw[(size_t)W * C]); yv[3] = to_f(yw[(size_t)W * C + C]);
        xh = (yv[0] - mu) * is;
        if (gs != 0.f)
#pragma unroll
          for (int q = 1; q < 4; ++q) {
            const float cq = (yv[q] - mu) * is;
            if (gs * cq > gs * xh) xh = cq;
          }
      }
      s1 += dz;
      s2 += dz * xh;
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    parts[(((size_t)c * G + g) * R + r) * 2] = s1;
    parts[(((size_t)c * G + g) * R + r) * 2 + 1] = s2;
  }
}

// dy = k1 * dz + kx * y + k0 for every pixel (incl. rows/cols outside the floor-mode windows)
template <typename T>
__global__ __launch_bounds__(256) void bwd_apply_cl_kernel(
    const T* __restrict__ y, const void* __restrict__ gout, int mode,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ coef, T* __restrict__ dy, long long total, int B, int C, int H,
    int W, U32Div dcv, U32Div dwc, U32Div dhc) {
  constexpr int V = Vec<T>::V;
  const int Hp = H / 2, Wp = W / 2, CV = C / V;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;      // windows covering every pixel
  // total < 2^32 (host-checked): 32-bit index decomposition by exact reciprocal multiplies
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const unsigned pw = dcv.div((unsigned)i);
    const int cv = (int)((unsigned)i - pw * CV);
    const unsigned ph = dwc.div(pw);
    const int wc = (int)(pw - ph * Wc);
    const int n = (int)dhc.div(ph), hc = (int)(ph - (unsigned)n * Hc);
    const int g = n / B, c0 = cv * V;
    float sc[V], sf[V], k1[V], kx[V], k0[V];
    load_coef<V>(scale, g * C + c0, sc);
    load_coef<V>(shift, g * C + c0, sf);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      k1[e] = coef[(g * C + c0 + e) * 3];
      kx[e] = coef[(g * C + c0 + e) * 3 + 1];
      k0[e] = coef[(g * C + c0 + e) * 3 + 2];
    }
    const bool has_r = 2 * hc + 1 < H, has_c = 2 * wc + 1 < W;
    const size_t pix0 = ((size_t)n * H + 2 * hc) * W + 2 * wc;
    Win<T> w;
    load_win<T>(y, pix0, W, C, c0, has_r, has_c, sc, sf, w);
    float gg[V];
    load_gout<T, V>(gout, mode, n, hc, wc, Hp, Wp, C, c0, gg);
    const size_t off[4] = {pix0 * C, (pix0 + 1) * C, (pix0 + W) * C, (pix0 + W + 1) * C};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!w.has[k]) continue;
      float d[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float dz = (w.arg[e] == k && w.mx[e] > 0.f) ? gg[e] : 0.f;
        d[e] = fmaf(k1[e], dz, fmaf(kx[e], w.y[k][e], k0[e]));
      }
      Vec<T>::st(dy + off[k] + c0, d);
    }
  }
}

int grid_for(long long total) {
  return (int)std::max(1ll, std::min<long long>((total + 255) / 256, 1ll << 20));
}

}  // namespace

// ============================================================================= entry points
int avd_cl_bn_relu_pool_impl(const void* y, int dt, const float* scale, const float* shift,
                             void* out, int mode, int N, int B, int C, int H, int W,
                             hipStream_t st) {
  const int V = dt == AVD_BF16 ? 8 : 4;
  if (C % V || N % B || H < 2 || W < 2) return AVD_ERR_SHAPE;
  if (mode == 1) {
    const long long total = (long long)N * (C / V);
    if (dt == AVD_BF16)
      relu_pool_gap_cl_kernel<bf16><<<grid_for(total), 256, 0, st>>>((const bf16*)y, scale, shift,
                                                                     (float*)out, total, B, C, H, W);
    else
      relu_pool_gap_cl_kernel<float><<<grid_for(total), 256, 0, st>>>((const float*)y, scale, shift,
                                                                      (float*)out, total, B, C, H, W);
  } else if (mode == 0 || mode == 2) {
    const long long total = (long long)N * (H / 2) * (W / 2) * (C / V);
    if (total >= (1ll << 32)) return AVD_ERR_SHAPE;
    const U32Div dcv = U32Div::make(C / V), dwp = U32Div::make(W / 2), dhp = U32Div::make(H / 2);
    if (dt == AVD_BF16)
      relu_pool_cl_kernel<bf16><<<grid_for(total), 256, 0, st>>>((const bf16*)y, scale, shift, out,
                                                                 mode, total, B, C, H, W, dcv, dwp,
                                                                 dhp);
    else
      relu_pool_cl_kernel<float><<<grid_for(total), 256, 0, st>>>((const float*)y, scale, shift, out,
                                                                  mode, total, B, C, H, W, dcv, dwp,
                                                                  dhp);
  } else {
    return AVD_ERR_ARG;
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// partial rows per group of avd_cl_bn_bwd_reduce: ~16 windows per slot
int avd_cl_bn_bwd_rows_impl(int B, int C, int H, int W, int dt) {
  const int V = dt == AVD_BF16 ? 8 : 4;
  const long long nwin = (long long)B * (H / 2) * (W / 2);
  const int slots = 256 / std::max(1, C / V);
  // windows per slot (thread) of a partial row: long enough that the block's fixed reduction is
  // amortised over several rounds of 4 in-flight windows
  constexpr int wps = 16;
  const long long r = (nwin + (long long)slots * wps - 1) / ((long long)slots * wps);
  return (int)std::max(1ll, std::min(r, 4096ll));
}

int avd_cl_bn_bwd_reduce_impl(const void* y, int dt, const void* gout, int mode,
                              const float* scale, const float* shift, const float* mean,
                              const float* invstd, float* parts, int N, int B, int C, int H,
                              int W, hipStream_t st) {
  const int V = dt == AVD_BF16 ? 8 : 4;
  if (C % V || C / V > 256 || N % B || mode < 0 || mode > 2) return AVD_ERR_SHAPE;
  const int G = N / B;
  const int R = avd_cl_bn_bwd_rows_impl(B, C, H, W, dt);
  const long long nwin = (long long)B * (H / 2) * (W / 2);
  const long long per = (nwin + R - 1) / R;
  dim3 grid(R, G);
  if (dt == AVD_BF16)
    bwd_reduce_cl_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)y, gout, mode, scale, shift, mean,
                                                     invstd, parts, G, B, C, H, W, R, per);
  else
    bwd_reduce_cl_kernel<float><<<grid, 256, 0, st>>>((const float*)y, gout, mode, scale, shift, mean,
                                                      invstd, parts, G, B, C, H, W, R, per);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_cl_bn_bwd_apply_impl(const void* y, int dt, const void* gout, int mode,
                             const float* scale, const float* shift, const float* coef, void* dy,
                             int N, int B, int C, int H, int W, hipStream_t st) {
  const int V = dt == AVD_BF16 ? 8 : 4;
  if (C % V || N % B || mode < 0 || mode > 2) return AVD_ERR_SHAPE;
  const long long total = (long long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / V);
  if (total >= (1ll << 32)) return AVD_ERR_SHAPE;
  const U32Div dcv = U32Div::make(C / V), dwc = U32Div::make((W + 1) / 2),
               dhc = U32Div::make((H + 1) / 2);
  if (dt == AVD_BF16)
    bwd_apply_cl_kernel<bf16><<<grid_for(total), 256, 0, st>>>((const bf16*)y, gout, mode, scale,
                                                               shift, coef, (bf16*)dy, total, B, C,
                                                               H, W, dcv, dwc, dhc);
  else
    bwd_apply_cl_kernel<float><<<grid_for(total), 256, 0, st>>>((const float*)y, gout, mode, scale,
                                                                shift, coef, (float*)dy, total, B,
                                                                C, H, W, dcv, dwc, dhc);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// BN-backward partial sums from the pooled output (bwd_reduce_pooled_cl_kernel); same rows as
// avd_cl_bn_bwd_reduce.  pooled has gout's layout (mode 0: NHWC dt, mode 2: f32 (c,h,w)).
int avd_cl_bn_bwd_reduce_pooled_impl(const void* y, int dt, const void* pooled, const void* gout,
                                     int mode, const float* gamma, const float* beta,
                                     const float* mean, const float* invstd, float* parts, int N,
                                     int B, int C, int H, int W, hipStream_t st) {
  const int V = dt == AVD_BF16 ? 8 : 4;
  if (C % V || C / V > 256 || N % B || (mode != 0 && mode != 2) || (H & 1) || (W & 1))
    return AVD_ERR_SHAPE;
  const int G = N / B;
  const int R = avd_cl_bn_bwd_rows_impl(B, C, H, W, dt);
  const long long nwin = (long long)B * (H / 2) * (W / 2);
  const long long per = (nwin + R - 1) / R;
  dim3 grid(R, G);
  if (mode == 2 && R <= B && !g_opts.generic_m2) {
    const dim3 g2(R, G, (C + 3) / 4);
    if (dt == AVD_BF16)
      bwd_reduce_pooled_m2_kernel<bf16><<<g2, 256, 0, st>>>((const bf16*)y, (const float*)pooled,
                                                            (const float*)gout, gamma, beta, mean,
                                                            invstd, parts, G, B, C, H, W, R);
    else
      bwd_reduce_pooled_m2_kernel<float><<<g2, 256, 0, st>>>((const float*)y, (const float*)pooled,
                                                             (const float*)gout, gamma, beta, mean,
                                                             invstd, parts, G, B, C, H, W, R);
    AVD_CHECK_LAUNCH();
    return AVD_OK;
  }
  if (dt == AVD_BF16)
    bwd_reduce_pooled_cl_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)y, pooled, gout, mode, gamma,
                                                            beta, mean, invstd, parts, G, B, C, H, W,
                                                            R, per);
  else
    bwd_reduce_pooled_cl_kernel<float><<<grid, 256, 0, st>>>((const float*)y, pooled, gout, mode, gamma,
                                                             beta, mean, invstd, parts, G, B, C, H, W,
                                                             R, per);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

