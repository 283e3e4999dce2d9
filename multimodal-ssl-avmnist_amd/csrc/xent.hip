// Fused softmax cross-entropy over a similarity matrix that is never stored: the InfoNCE
// (MultiModalDINOWithINFONCELightning.infoNCE_loss, dino.py:1091-1128) and NT-Xent
// (MultiModalSimCLRLightning.nt_xent_loss, multimodal_simclr.py:74-89) losses with their
// gradients, for this rank's rows Q [R][P] against the (gathered) columns K [C][P]:
//
//   S[i][j] = inv_t q_i . k_j          (q, k L2-normalised; j = mask(i) excluded)
//   loss_i  = logsumexp_j S[i][j] - S[i][t(i)]
//   dQ_i    = g inv_t (sum_j p_ij k_j - k_t(i))           p_ij = softmax_j S[i][j]
//   dK_j    = g inv_t (sum_i p_ij q_i - sum_{i: t(i) = j} q_i)
//
// Row i lies in half h = i / Bh (NT-Xent: [z1; z2]; InfoNCE: one half) with i' = i - h Bh:
// t(i) = tgt[h] + i', mask(i) = msk[h] + i' (msk[h] < 0: no mask).
//
// Before (contrastive.py, bf16 step): three GEMMs and a softmax pass over an f32 S and dS
// written to HBM -- 2 x 537 MB at config 4's [4096 x 32768] per rank.  Here, flash-style on the
// bf16 MFMA (v_mfma_f32_16x16x32_bf16):
//   pass A (rows): a wave owns 16 rows, streams the columns in 32-column blocks staged in LDS:
//     S^T = K Q^T (Q fragments resident), online max / sum per row, O^T += K^T P^T -- i.e.
//     sum_j p_ij k_j accumulates without S ever leaving registers.  Column splits run in
//     parallel blocks and are merged by xent_rows_combine (lse, loss, dQ).
//   pass B (columns): a wave owns 16 columns, streams the rows: S = Q K^T again, p from the
//     row lse of pass A, dK^T += Q^T P^T; row splits merged in fixed order by
//     xent_cols_combine.  No atomics: every sum has a fixed order (deterministic).
// The S^T / S accumulator layout (lane = one row / one column, 8 entries) is the B operand of
// the second MFMA as is: its 8 k values {4g..4g+3, 16+4g..16+4g+3} are matched by reading the
// A operand (K^T / Q^T) with ds_read_b64_tr_b16 in the same order (wgrad_ws.hip's kpix).
#include <algorithm>
#include <math.h>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(4))) short s4;
typedef __attribute__((ext_vector_type(2))) unsigned u2;

constexpr int XB = 32;          // rows / columns per streamed block
constexpr int XT = 256;         // threads per block (4 waves x 16 owned rows / columns)

struct XArgs {
  const float* q;               // [R][P]
  const float* k;               // [C][P]
  int R, C, Bh;
  int tgt0, tgt1, msk0, msk1;
  float inv_t, g;
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
__device__ __forceinline__ bf16x8 cvt8(float4 a, float4 b) {
  return bf16x8{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
}
__device__ __forceinline__ int xtarget(const XArgs& a, int i) {
  const int h = i >= a.Bh, ii = i - h * a.Bh;
  return (h ? a.tgt1 : a.tgt0) + ii;
}
__device__ __forceinline__ int xmask(const XArgs& a, int i) {
  const int h = i >= a.Bh, ii = i - h * a.Bh;
  const int m = h ? a.msk1 : a.msk0;
  return m < 0 ? -1 : m + ii;
}

// stage XB rows of an f32 [n][P] matrix (rows r0..) as bf16 [XB][P + 8] (16-byte row pad:
// the 16 lanes of a b128 fragment read land on distinct banks); rows >= n are zero
template <int P>
__device__ __forceinline__ void stage_block(const float* __restrict__ src, int n, int r0, bf16* lds, int tid) {
  constexpr int PP = P + 8, V = P / 8;   // 8-element vectors per row
  for (int t = tid; t < XB * V; t += XT) {
    const int r = t / V, c = (t - r * V) * 8;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (r0 + r < n) {
      const float4* s = reinterpret_cast<const float4*>(src + (size_t)(r0 + r) * P + c);
      a = s[0];
      b = s[1];
    }
    *reinterpret_cast<bf16x8*>(lds + r * PP + c) = cvt8(a, b);
  }
}

// the same staging split in two: loads into registers (issued before the current block's
// MFMAs), LDS stores after them
template <int P>
struct BlockRegs {
  static constexpr int V = P / 8, NT = (XB * V) / XT;
  float4 v[NT][2];
};
template <int P>
__device__ __forceinline__ void load_block(const float* __restrict__ src, int n, int r0, int tid, BlockRegs<P>& br) {
  constexpr int V = P / 8;
  static_assert((XB * V) % XT == 0, "whole tasks per thread");
#pragma unroll
  for (int i = 0; i < BlockRegs<P>::NT; ++i) {
    const int t = tid + XT * i, r = t / V, c = (t - r * V) * 8;
    br.v[i][0] = br.v[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < n) {
      const float4* s = reinterpret_cast<const float4*>(src + (size_t)(r0 + r) * P + c);
      br.v[i][0] = s[0];
      br.v[i][1] = s[1];
    }
  }
}
template <int P>
__device__ __forceinline__ void store_block(const BlockRegs<P>& br, bf16* lds, int tid) {
  constexpr int PP = P + 8, V = P / 8;
#pragma unroll
  for (int i = 0; i < BlockRegs<P>::NT; ++i) {
    const int t = tid + XT * i, r = t / V, c = (t - r * V) * 8;
    *reinterpret_cast<bf16x8*>(lds + r * PP + c) = cvt8(br.v[i][0], br.v[i][1]);
  }
}

// the resident B fragments (16 owned rows of src, as B^T: n = row, k = 32 features per step)
template <int P>
__device__ __forceinline__ void own_frags(const float* __restrict__ src, int n, int r0, int lane, bf16x8 (&f)[P / 32]) {
  const int r = r0 + (lane & 15), g = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < P / 32; ++ks) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (r < n) {
      const float4* s = reinterpret_cast<const float4*>(src + (size_t)r * P + 32 * ks + 8 * g);
      a = s[0];
      b = s[1];
    }
    f[ks] = cvt8(a, b);
  }
}

// 32 x 16 block of scores: st[h][e] = (block entry 16 h + 4 g + e) . (owned entry lane & 15)
template <int P>
__device__ __forceinline__ void scores(const bf16* lds, const bf16x8 (&own)[P / 32], int lane, f4 (&st)[2]) {
  constexpr int PP = P + 8;
  const int r16 = lane & 15, g = lane >> 4;
  st[0] = f4{0.f, 0.f, 0.f, 0.f};
  st[1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < P / 32; ++ks) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(lds + (16 * h + r16) * PP + 32 * ks + 8 * g);
      st[h] = mma(a, own[ks], st[h]);
    }
  }
}

// acc[t] (feature tile t: features 16 t + 4 g .. + 3, owned entry lane & 15) += block^T pv
template <int P>
__device__ __forceinline__ void accum(const bf16* lds, bf16x8 pv, int lane, f4 (&acc)[P / 16]) {
  constexpr int PP = P + 8;
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
  for (int t = 0; t < P / 16; ++t) {
    const bf16* b0 = lds + (4 * g + q4) * PP + 16 * t + 4 * p4;
    const bf16x8 a = frag8(tr4(b0), tr4(b0 + 16 * PP));
    acc[t] = mma(a, pv, acc[t]);
  }
}

__device__ __forceinline__ bf16x8 pack8(const float (&p)[8]) {
  return bf16x8{(__bf16)p[0], (__bf16)p[1], (__bf16)p[2], (__bf16)p[3],
                (__bf16)p[4], (__bf16)p[5], (__bf16)p[6], (__bf16)p[7]};
}

// ---------------------------------------------------------------- pass A: rows
// grid (ceil(R / 64), S splits); partials pm / pl [S][R], po [S][R][P]
template <int P>
__global__ __launch_bounds__(XT, 2) void xent_rows_kernel(XArgs a, int S, float* __restrict__ pm,
                                                       float* __restrict__ pl, float* __restrict__ po) {
  __shared__ __attribute__((aligned(16))) bf16 kb[2][XB * (P + 8)];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int row0 = blockIdx.x * 64 + wave * 16, row = row0 + r16;
  const int s = blockIdx.y;
  const int nblk = (a.C + XB - 1) / XB;
  const int b0 = (int)(((long long)s * nblk) / S), b1 = (int)(((long long)(s + 1) * nblk) / S);
  bf16x8 own[P / 32];
  own_frags<P>(a.q, a.R, row0, lane, own);
  const int msk = row < a.R ? xmask(a, row) : -1;
  f4 acc[P / 16];
#pragma unroll
  for (int t = 0; t < P / 16; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  BlockRegs<P> nx;
  if (b0 < b1) stage_block<P>(a.k, a.C, b0 * XB, kb[0], tid);
  for (int b = b0; b < b1; ++b) {
    __syncthreads();                          // block b staged; block b - 1 no longer read
    if (b + 1 < b1) load_block<P>(a.k, a.C, (b + 1) * XB, tid, nx);   // in flight under the MFMAs
    const bf16* lk = kb[(b - b0) & 1];
    f4 st[2];
    scores<P>(lk, own, lane, st);
    float v[8], bm = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = b * XB + 16 * h + 4 * g + e;
        const float x = (j < a.C && j != msk) ? st[h][e] * a.inv_t : -INFINITY;
        v[4 * h + e] = x;
        bm = fmaxf(bm, x);
      }
    bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    const float mn = fmaxf(m, bm);
    const float sc = mn == -INFINITY ? 1.f : __expf(m - mn);
    float p[8], ps = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      p[e] = mn == -INFINITY ? 0.f : __expf(v[e] - mn);
      ps += p[e];
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * sc + ps;
    m = mn;
#pragma unroll
    for (int t = 0; t < P / 16; ++t) acc[t] *= sc;
    accum<P>(lk, pack8(p), lane, acc);
    if (b + 1 < b1) store_block<P>(nx, kb[(b + 1 - b0) & 1], tid);
  }
  if (row < a.R) {
    if (g == 0) {
      pm[(size_t)s * a.R + row] = m;
      pl[(size_t)s * a.R + row] = l;
    }
    float* o = po + ((size_t)s * a.R + row) * P;
#pragma unroll
    for (int t = 0; t < P / 16; ++t)
      *reinterpret_cast<float4*>(o + 16 * t + 4 * g) = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
  }
}

// one wave per row: merge the S partials -> lse, loss = lse - S_target (target score from the
// f32 vectors), dQ = g inv_t (O / L - k_target); lane l owns features 4 l .. 4 l + 3 (P = 256)
// or 2 l, 2 l + 1 (P = 128), so every partial row is read once with vector loads
template <int P>
__global__ __launch_bounds__(XT) void xent_rows_combine(XArgs a, int S, const float* __restrict__ pm,
                                                        const float* __restrict__ pl,
                                                        const float* __restrict__ po, float* __restrict__ lse,
                                                        float* __restrict__ loss, float* __restrict__ dq) {
  constexpr int F = P / 64;
  const int row = blockIdx.x * (XT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= a.R) return;
  float ms[8], w[8];
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) {
    ms[s] = pm[(size_t)s * a.R + row];
    M = fmaxf(M, ms[s]);
  }
  float L = 0.f;
  for (int s = 0; s < S; ++s) {
    w[s] = ms[s] == -INFINITY ? 0.f : __expf(ms[s] - M);
    L += pl[(size_t)s * a.R + row] * w[s];
  }
  const int t = xtarget(a, row);
  const float* qi = a.q + (size_t)row * P + F * lane;
  const float* kt = a.k + (size_t)t * P + F * lane;
  float o[F], kv[F], dot = 0.f;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    kv[f] = kt[f];
    dot += qi[f] * kv[f];
    o[f] = 0.f;
  }
  for (int s = 0; s < S; ++s) {
    const float* ps = po + ((size_t)s * a.R + row) * P + F * lane;
#pragma unroll
    for (int f = 0; f < F; ++f) o[f] += ps[f] * w[s];
  }
  dot = wave_sum(dot);
  const float lz = M + logf(L);
  if (lane == 0) {
    lse[row] = lz;
    loss[row] = lz - a.inv_t * dot;
  }
  const float gs = a.g * a.inv_t, il = 1.f / L;
  float* d = dq + (size_t)row * P + F * lane;
#pragma unroll
  for (int f = 0; f < F; ++f) d[f] = gs * (o[f] * il - kv[f]);
}

// ---------------------------------------------------------------- pass B: columns
// grid (ceil(C / 64), S splits over the rows); partial sums pk [S][C][P] of sum_i p_ij q_i
template <int P>
__global__ __launch_bounds__(XT) void xent_cols_kernel(XArgs a, int S, const float* __restrict__ lse,
                                                       float* __restrict__ pk) {
  __shared__ __attribute__((aligned(16))) bf16 qb[2][XB * (P + 8)];
  __shared__ float lb[2][XB];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int col0 = blockIdx.x * 64 + wave * 16, col = col0 + r16;
  const int s = blockIdx.y;
  const int nblk = (a.R + XB - 1) / XB;
  const int b0 = (int)(((long long)s * nblk) / S), b1 = (int)(((long long)(s + 1) * nblk) / S);
  bf16x8 own[P / 32];
  own_frags<P>(a.k, a.C, col0, lane, own);
  f4 acc[P / 16];
#pragma unroll
  for (int t = 0; t < P / 16; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  auto stage_l = [&](int b, int buf) {
    if (tid < XB) {
      const int i = b * XB + tid;
      lb[buf][tid] = i < a.R ? lse[i] : INFINITY;     // rows past R: p = 0
    }
  };
  BlockRegs<P> nx;
  if (b0 < b1) {
    stage_block<P>(a.q, a.R, b0 * XB, qb[0], tid);
    stage_l(b0, 0);
  }
  for (int b = b0; b < b1; ++b) {
    __syncthreads();
    if (b + 1 < b1) load_block<P>(a.q, a.R, (b + 1) * XB, tid, nx);
    const int buf = (b - b0) & 1;
    f4 st[2];
    scores<P>(qb[buf], own, lane, st);
    float p[8];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ri = 16 * h + 4 * g + e, i = b * XB + ri;
        const bool ok = i < a.R && col < a.C && xmask(a, i) != col;
        p[4 * h + e] = ok ? __expf(st[h][e] * a.inv_t - lb[buf][ri]) : 0.f;
      }
    accum<P>(qb[buf], pack8(p), lane, acc);
    if (b + 1 < b1) {
      store_block<P>(nx, qb[buf ^ 1], tid);
      stage_l(b + 1, buf ^ 1);
    }
  }
  if (col < a.C) {
    float* o = pk + ((size_t)s * a.C + col) * P;
#pragma unroll
    for (int t = 0; t < P / 16; ++t)
      *reinterpret_cast<float4*>(o + 16 * t + 4 * g) = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
  }
}

// dK_j = g inv_t (sum_s pk[s][j] - sum_{i: t(i) = j} q_i), one thread per (column, feature)
template <int P>
__global__ __launch_bounds__(XT) void xent_cols_combine(XArgs a, int S, const float* __restrict__ pk,
                                                        float* __restrict__ dk) {
  const long long e = (long long)blockIdx.x * XT + threadIdx.x;
  if (e >= (long long)a.C * P) return;
  const int j = (int)(e / P), c = (int)(e - (long long)j * P);
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += pk[((size_t)s * a.C + j) * P + c];
  // rows whose target is column j: one per half at most (i' = j - tgt[h])
  const int halves = a.R > a.Bh ? 2 : 1;
  for (int h = 0; h < halves; ++h) {
    const int ii = j - (h ? a.tgt1 : a.tgt0);
    const int rows_h = h ? a.R - a.Bh : min(a.R, a.Bh);
    if (ii >= 0 && ii < rows_h) v -= a.q[(size_t)(h * a.Bh + ii) * P + c];
  }
  dk[e] = a.g * a.inv_t * v;
}

int xsplit(int blocks) {
  // fill ~2 waves of 256 CUs: S = ceil(512 / blocks), at most 8
  return std::max(1, std::min(8, (512 + blocks - 1) / blocks));
}

}  // namespace

int avd_xent_fused_ws(int R, int C, int P) {
  if (R <= 0 || C <= 0 || (P != 128 && P != 256)) return -1;
  const int sa = xsplit((R + 63) / 64), sb = xsplit((C + 63) / 64);
  // floats: pm + pl [sa][R], po [sa][R][P], lse [R], pk [sb][C][P]
  const long long n = 2LL * sa * R + (long long)sa * R * P + R + (long long)sb * C * P;
  return n > 0x7fffffffLL ? -1 : (int)n;
}

int avd_xent_fused(const float* q, const float* k, int R, int C, int P, int Bh, int tgt0, int tgt1,
                   int msk0, int msk1, float inv_t, float gscale, float* loss, float* dq, float* dk,
                   float* ws, long long ws_elems, void* stream) {
  if (!q || !k || !loss || !dq || !dk || !ws) return AVD_ERR_ARG;
  const int need = avd_xent_fused_ws(R, C, P);
  if (need < 0 || Bh <= 0 || Bh > R || R > 2 * Bh) return AVD_ERR_SHAPE;
  if (ws_elems < need) return AVD_ERR_ARG;
  // every target column must exist (the reference's labels index S's columns)
  const int r1 = R > Bh ? R - Bh : 0;
  if (tgt0 < 0 || tgt0 + Bh > C || (r1 && (tgt1 < 0 || tgt1 + r1 > C))) return AVD_ERR_SHAPE;
  XArgs a{q, k, R, C, Bh, tgt0, tgt1, msk0, msk1, inv_t, gscale};
  const int sa = xsplit((R + 63) / 64), sb = xsplit((C + 63) / 64);
  float* pm = ws;
  float* pl = pm + (size_t)sa * R;
  float* po = pl + (size_t)sa * R;
  float* lse = po + (size_t)sa * R * P;
  float* pk = lse + R;
  hipStream_t st = avd_stream(stream);
  const dim3 ga((R + 63) / 64, sa), gb((C + 63) / 64, sb);
  const int gr = (R + XT / 64 - 1) / (XT / 64);
  const int gc = (int)(((long long)C * P + XT - 1) / XT);
  if (P == 256) {
    xent_rows_kernel<256><<<ga, XT, 0, st>>>(a, sa, pm, pl, po);
    xent_rows_combine<256><<<gr, XT, 0, st>>>(a, sa, pm, pl, po, lse, loss, dq);
    xent_cols_kernel<256><<<gb, XT, 0, st>>>(a, sb, lse, pk);
    xent_cols_combine<256><<<gc, XT, 0, st>>>(a, sb, pk, dk);
  } else {
    xent_rows_kernel<128><<<ga, XT, 0, st>>>(a, sa, pm, pl, po);
    xent_rows_combine<128><<<gr, XT, 0, st>>>(a, sa, pm, pl, po, lse, loss, dq);
    xent_cols_kernel<128><<<gb, XT, 0, st>>>(a, sb, lse, pk);
    xent_cols_combine<128><<<gc, XT, 0, st>>>(a, sb, pk, dk);
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}
