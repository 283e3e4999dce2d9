// BN-backward apply fused with the weight gradient of the FIRST 3x3 layer (Cin = 1, pad 1) of the
// SimCLR / unimodal encoders (models/dino.py:18-73: conv(1->32) -> BN -> ReLU -> maxpool2 on the
// 112x112 spectrogram or the 28x28 image).  The layer needs no input gradient, so its dy is
// consumed only by dW: here dy is formed per 2x2 pooling window in LDS (the window's first
// argmax of relu(bn(y)) carries the pooled gradient, dy = k1 dz + kx y + k0, rounded to bf16
// exactly like bwd_apply_cl_kernel) and never written -- the unfused chain writes and re-reads
// the full-resolution dy (2 x 1.64 GB per config-4 step).
//
// dW[c][tap] = sum_p dy[p][c] * x[p + tap] as a GEMM M = c (C / 16 tiles), N = tap (9 of 16
// columns), K = pixels: A from dys [pixel][DYS] and B from an im2col tile x9 [pixel][16]
// (x9[p][t] = x[p + off(t)], zero halo), both by ds_read_b64_tr_b16 with the wgrad3 k<->pixel
// map (conflict-free strides: DYS = 48 / 80 for 32 / 64 channels, 16 for 16).  A persistent
// block walks tiles of TR rows (whole-width), its 4 waves split each tile's k-steps, and the
// block's accumulators are summed over waves in fixed order into one slab [C][9] (avd_sum_rows).
#include <algorithm>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s4w;
typedef __attribute__((ext_vector_type(2))) unsigned u2w;

__device__ __forceinline__ u2w trd(const bf16* p) {
  const s4w v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4w*)(reinterpret_cast<uintptr_t>(p)));
  return __builtin_bit_cast(u2w, v);
}
__device__ __forceinline__ bf16x8 fr8(u2w lo, u2w hi) {
  return __builtin_bit_cast(bf16x8, u4{lo.x, lo.y, hi.x, hi.y});
}
__device__ __forceinline__ int kpx(int g, int h, int q) { return 16 * (g >> 1) + 8 * h + 4 * (g & 1) + q; }

constexpr int XS9 = 16;      // x9 pixel stride (taps)
constexpr int TRW = 4;       // tile rows (two window rows)

template <int C>
__global__ __launch_bounds__(256, 2) void c1w3_kernel(
    const bf16* __restrict__ y, const bf16* __restrict__ gout, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, const bf16* __restrict__ x,
    float* __restrict__ parts, int N, int B, int H, int W) {
  constexpr int NT = C / 16;
  constexpr int DYS = C == 16 ? 16 : C + 16;
  constexpr int VQ = C / 8;                   // 8-channel groups
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  const int TP = TRW * W;                     // tile pixels
  const int KST = (TP + 31) / 32;             // k-steps; pixels TP .. 32*KST-1 stay zero
  const int TPP = KST * 32;
  bf16* dys = sm;                             // [TPP][DYS]
  bf16* x9 = dys + TPP * DYS;                 // [TPP][XS9]
  bf16* xr = x9 + TPP * XS9;                  // [TRW + 2][W + 2] x rows with halo
  const int XW = W + 2;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15, q4 = r16 >> 2, p4 = r16 & 3;
  const int Hp = H / 2, Wp = W / 2;
  const int tps = H / TRW, ntiles = N * tps;
  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  // k tail (TP % 32 != 0): zero rows, never rewritten
  for (int i = TP * (DYS / 8) + tid; i < TPP * (DYS / 8); i += 256)
    *reinterpret_cast<u4*>(dys + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};
  for (int i = TP * (XS9 / 8) + tid; i < TPP * (XS9 / 8); i += 256)
    *reinterpret_cast<u4*>(x9 + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};

  // this thread's window tasks t = tid + 256 i all have channel group q = tid % VQ; its 8
  // channels' BN coefficients are held in registers (reloaded when the BN group changes)
  constexpr int TPT = 2;                      // window tasks per thread (TRW=4: 2*Wp*VQ <= 512)
  const int q = tid % VQ, c0 = 8 * q;
  const int ntask = (TRW / 2) * Wp * VQ;
  float sc[8], sf[8], k1[8], kx[8], k0[8];
  int cur_g = -1;
  // next tile's operands, loaded while the current tile's MFMAs run
  u4 py[TPT][4], pg[TPT];
  bf16 px[3];
  auto load = [&](int ti) {
    const int n = ti / tps, y0 = (ti - n * tps) * TRW;
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int t = tid + 256 * i;
      const int w = t / VQ, wc = w % Wp, wr = w / Wp;
      const bool ok = t < ntask;
      const int yy = y0 + 2 * wr;
      const size_t pix0 = ok ? ((size_t)n * H + yy) * W + 2 * wc : 0;
      const size_t g0 = ok ? (((size_t)n * Hp + yy / 2) * Wp + wc) * C + c0 : 0;
      py[i][0] = *reinterpret_cast<const u4*>(y + pix0 * C + c0);
      py[i][1] = *reinterpret_cast<const u4*>(y + (pix0 + 1) * C + c0);
      py[i][2] = *reinterpret_cast<const u4*>(y + (pix0 + W) * C + c0);
      py[i][3] = *reinterpret_cast<const u4*>(y + (pix0 + W + 1) * C + c0);
      pg[i] = *reinterpret_cast<const u4*>(gout + g0);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = tid + 256 * i;
      const int r = e / XW, c = e - r * XW, iy = y0 - 1 + r, ix = c - 1;
      const bool ok = e < (TRW + 2) * XW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      px[i] = x[ok ? ((size_t)n * H + iy) * W + ix : 0];
    }
  };
  auto unpack = [](u4 w, float (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  };
  if (t0 < t1) load(t0);

  for (int ti = t0; ti < t1; ++ti) {
    const int n = ti / tps, y0 = (ti - n * tps) * TRW, gb = n / B;
    if (gb != cur_g) {
      cur_g = gb;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int gc = gb * C + c0 + e;
        sc[e] = scale[gc]; sf[e] = shift[gc];
        k1[e] = coef[gc * 3]; kx[e] = coef[gc * 3 + 1]; k0[e] = coef[gc * 3 + 2];
      }
    }
    __syncthreads();                          // the previous tile's reads are done
    // ---- x rows y0-1 .. y0+TRW (zero outside the image) and dy per window x 8 channels
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = tid + 256 * i;
      if (e < (TRW + 2) * XW) {
        const int r = e / XW, c = e - r * XW, iy = y0 - 1 + r, ix = c - 1;
        xr[e] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? px[i] : f2bf(0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int t = tid + 256 * i;
      if (t >= ntask) continue;
      const int w = t / VQ, wc = w % Wp, wr = w / Wp;
      float v[4][8], gg[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) unpack(py[i][k], v[k]);
      unpack(pg[i], gg);
      uint32_t o[4][4];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float best = fmaxf(fmaf(v[0][e], sc[e], sf[e]), 0.f);
        int a = 0;
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          const float r = fmaxf(fmaf(v[k][e], sc[e], sf[e]), 0.f);
          if (r > best) { best = r; a = k; }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float dz = (a == k && best > 0.f) ? gg[e] : 0.f;
          const float d = fmaf(k1[e], dz, fmaf(kx[e], v[k][e], k0[e]));
          const uint32_t bb = __builtin_bit_cast(uint16_t, f2bf(d));
          if (e & 1) o[k][e >> 1] |= bb << 16;
          else o[k][e >> 1] = bb;
        }
      }
      const int p0 = (2 * wr) * W + 2 * wc;
      const int pk[4] = {p0, p0 + 1, p0 + W, p0 + W + 1};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        *reinterpret_cast<u4*>(dys + pk[k] * DYS + c0) = u4{o[k][0], o[k][1], o[k][2], o[k][3]};
    }
    if (ti + 1 < t1) load(ti + 1);            // in flight under this tile's im2col and MFMAs
    __syncthreads();                          // xr ready
    // ---- im2col: x9[p][tap] = x[p + (ky - 1, kx - 1)], taps 9..15 zero
    for (int p = tid; p < TP; p += 256) {
      const int r = p / W, c = p - r * W;
      uint32_t w8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) w8[k] = 0u;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const uint32_t b = __builtin_bit_cast(uint16_t, xr[(r + t / 3) * XW + c + t % 3]);
        w8[t >> 1] |= (t & 1) ? b << 16 : b;
      }
      *reinterpret_cast<u4*>(x9 + p * XS9) = u4{w8[0], w8[1], w8[2], w8[3]};
      *reinterpret_cast<u4*>(x9 + p * XS9 + 8) = u4{w8[4], w8[5], w8[6], w8[7]};
    }
    __syncthreads();
    // ---- MFMAs: wave w takes k-steps w, w+4, ...
    for (int ks = wave; ks < KST; ks += 4) {
      const int P0 = 32 * ks;
      const int pa = P0 + kpx(g, 0, q4), pb = P0 + kpx(g, 1, q4);
      const bf16x8 bv = fr8(trd(x9 + pa * XS9 + 4 * p4), trd(x9 + pb * XS9 + 4 * p4));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x8 av = fr8(trd(dys + pa * DYS + 16 * t + 4 * p4), trd(dys + pb * DYS + 16 * t + 4 * p4));
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[t], 0, 0, 0);
      }
    }
  }

  // ---- the block's slab: sum of the 4 waves' partials in fixed order
  __syncthreads();
  float* red = reinterpret_cast<float*>(sm);  // [4][C][16]
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * C + 16 * t + 4 * g + i) * 16 + r16] = acc[t][i];
  __syncthreads();
  float* out = parts + (size_t)blockIdx.x * C * 9;
  for (int e = tid; e < C * 9; e += 256) {
    const int c = e / 9, tap = e - c * 9;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += red[(w * C + c) * 16 + tap];
    out[e] = s;
  }
}

int ncu_c1w3() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

size_t c1w3_lds(int C, int W) {
  const int DYS = C == 16 ? 16 : C + 16;
  const size_t tpp = (size_t)(TRW * W + 31) / 32 * 32;
  const size_t a = tpp * (DYS + XS9) * 2 + (size_t)(TRW + 2) * (W + 2) * 2;
  return std::max(a, (size_t)4 * C * 16 * 4);
}

}  // namespace

extern "C" {

// slabs of avd_c1w3_apply_wgrad (0: shape not served)
int avd_c1w3_slabs(int dt, int N, int Cin, int H, int W, int Cout, int K, int pad) {
  if (getenv("AVDINO_C1W3_OFF")) return 0;
  if (dt != AVD_BF16 || Cin != 1 || K != 3 || pad != 1) return 0;
  if (Cout != 16 && Cout != 32 && Cout != 64) return 0;
  if (H % TRW || W % 2 || W > 128 || (TRW / 2) * (W / 2) * (Cout / 8) > 512 || (TRW + 2) * (W + 2) > 768)
    return 0;
  if (c1w3_lds(Cout, W) > 80 * 1024) return 0;
  return grid_cap(std::min(N * (H / TRW), 2 * ncu_c1w3()));
}

int avd_c1w3_apply_wgrad(const void* y, const void* gout, const float* scale, const float* shift,
                         const float* coef, const void* x, float* parts, int N, int B, int H,
                         int W, int Cout, hipStream_t st) {
  const int grid = avd_c1w3_slabs(AVD_BF16, N, 1, H, W, Cout, 3, 1);
  if (!grid) return AVD_ERR_SHAPE;
  const size_t lds = c1w3_lds(Cout, W);
#define AVD_C(C_)                                                                               \
  if (Cout == C_)                                                                               \
    c1w3_kernel<C_><<<grid, 256, lds, st>>>((const bf16*)y, (const bf16*)gout, scale, shift, coef, \
                                            (const bf16*)x, parts, N, B, H, W);
  AVD_C(16) else AVD_C(32) else AVD_C(64) else return AVD_ERR_SHAPE;
#undef AVD_C
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"

// ============================================================================ recompute passes
// The same first layer WITHOUT a stored conv output (avd_cl_c1_recompute for 3x3 / Cin 1):
// every pass rebuilds y = bf16(conv(x) + b) for a tile from the staged input (x rows -> the
// im2col tile x9 in LDS -> one v_mfma_f32_16x16x32_bf16 per 16 channels x 16 pixels with the
// weight rows as A, the same code in every pass, so y is bit-identical across passes) and then
//   pass 0: BN partial sums of y (per-block running sums, rows [C][G][4 * grid][2]);
//   pass 1: z = maxpool2(relu(y * scale + shift)) NHWC bf16;
//   pass 2: BN-backward partial sums (sum dz, sum dz * xhat) like avd_cl_bn_bwd_reduce;
//   pass 3: dy in LDS and the weight gradient, as c1w3_kernel.
// A 16-pixel MFMA column group is a 2-row x 8-column patch (W % 8 == 0), so a pooling window
// is the lanes {n, n^1, n^8, n^9} of a 16-lane row: DPP quad_perm / row_ror:8 exchanges.
namespace {

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

template <int P, int C>
__global__ __launch_bounds__(256, 2) void c1r3_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coef, const bf16* __restrict__ gz, bf16* __restrict__ z,
    float* __restrict__ out, int N, int B, int H, int W) {
  constexpr int NT = C / 16;
  constexpr int DYS = C == 16 ? 16 : C + 16;
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  const int TP = TRW * W;
  const int KST = (TP + 31) / 32, TPP = KST * 32;
  bf16* x9 = sm;                              // [TPP][XS9]
  bf16* xr = x9 + TPP * XS9;                  // [TRW + 2][W + 2]
  bf16* dys = xr + (((TRW + 2) * (W + 2) + 7) & ~7);   // [TPP][DYS] (pass 3)
  const int XW = W + 2;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15, q4 = r16 >> 2, p4 = r16 & 3;
  const int Hp = H / 2, Wp = W / 2;
  const int tps = H / TRW, ntiles = N * tps, G = N / B, tilesPG = ntiles / G;
  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  const int ngroups16 = (TRW / 2) * (W / 8);  // 16-pixel column groups per tile

  // weight rows (A): lane holds w[16 t + r16][8 g .. 8 g + 7] (taps >= 9 are zero rows of wk)
  bf16x8 aw[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) aw[t] = *reinterpret_cast<const bf16x8*>(wk + (16 * t + r16) * 32 + 8 * g);
  float bv[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[t][i] = bias ? bias[16 * t + 4 * g + i] : 0.f;

  // per-block running sums (passes 0, 2): rows blockIdx*4 + wave of R = 4 * grid per group
  float rs[NT][4], rq[NT][4];
  int cur_g = -1;
  const int R = 4 * (int)gridDim.x, srow = blockIdx.x * 4 + wave;
  auto zero_run = [&]() {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) { rs[t][i] = 0.f; rq[t][i] = 0.f; }
  };
  auto flush = [&](int gp) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = row16_sum(rs[t][i]), b = row16_sum(rq[t][i]);
        if (r16 == 0)
          *reinterpret_cast<float2*>(out + (((size_t)(16 * t + 4 * g + i) * G + gp) * R + srow) * 2) =
              make_float2(a, b);
      }
  };
  zero_run();
  // BN coefficients of the current group (passes 1-3): channels 16 t + 4 g + i
  float sc[NT][4], sf[NT][4], mu[NT][4], is[NT][4], k1[NT][4], kx[NT][4], k0[NT][4];
  int cg = -1;
  f4 acc3[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc3[t] = f4{0.f, 0.f, 0.f, 0.f};
  if constexpr (P == 3) {
    for (int i = TP * (DYS / 8) + tid; i < TPP * (DYS / 8); i += 256)
      *reinterpret_cast<u4*>(dys + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};
  }
  for (int i = TP * (XS9 / 8) + tid; i < TPP * (XS9 / 8); i += 256)
    *reinterpret_cast<u4*>(x9 + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};

  for (int ti = t0; ti < t1; ++ti) {
    const int n = ti / tps, y0 = (ti - n * tps) * TRW, gb = n / B;
    if constexpr (P == 0 || P == 2) {
      const int gi = ti / tilesPG;
      if (gi != cur_g) {
        if (cur_g >= 0) flush(cur_g);
        cur_g = gi;
        zero_run();
      }
    }
    if constexpr (P != 0) {
      if (gb != cg) {
        cg = gb;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int gc = gb * C + 16 * t + 4 * g + i;
            sc[t][i] = scale[gc]; sf[t][i] = shift[gc];
            if constexpr (P == 2) { mu[t][i] = mean[gc]; is[t][i] = invstd[gc]; }
            if constexpr (P == 3) { k1[t][i] = coef[gc * 3]; kx[t][i] = coef[gc * 3 + 1]; k0[t][i] = coef[gc * 3 + 2]; }
          }
      }
    }
    __syncthreads();
    for (int i = tid; i < (TRW + 2) * XW; i += 256) {
      const int r = i / XW, c = i - r * XW, iy = y0 - 1 + r, ix = c - 1;
      xr[i] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                  ? x[((size_t)n * H + iy) * W + ix] : f2bf(0.f);
    }
    __syncthreads();
    for (int p = tid; p < TP; p += 256) {
      const int r = p / W, c = p - r * W;
      uint32_t w8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) w8[k] = 0u;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const uint32_t b = __builtin_bit_cast(uint16_t, xr[(r + t / 3) * XW + c + t % 3]);
        w8[t >> 1] |= (t & 1) ? b << 16 : b;
      }
      *reinterpret_cast<u4*>(x9 + p * XS9) = u4{w8[0], w8[1], w8[2], w8[3]};
      *reinterpret_cast<u4*>(x9 + p * XS9 + 8) = u4{w8[4], w8[5], w8[6], w8[7]};
    }
    __syncthreads();
    // ---- y for the wave's column groups, pass epilogues
    for (int q = wave; q < ngroups16; q += 4) {
      const int gr = q / (W / 8), gc8 = q - gr * (W / 8);
      const int prow = 2 * gr + (r16 >> 3), pcol = 8 * gc8 + (r16 & 7);   // pixel of this lane
      const int p = prow * W + pcol;
      const bf16x8 bx = g < 2 ? *reinterpret_cast<const bf16x8*>(x9 + p * XS9 + 8 * g)
                              : bf16x8{};
      float yv[NT][4];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f4 a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[t], bx, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) yv[t][i] = bf2f(f2bf(a[i] + bv[t][i]));
      }
      if constexpr (P == 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            rs[t][i] += yv[t][i];
            rq[t][i] = fmaf(yv[t][i], yv[t][i], rq[t][i]);
          }
      } else {
        // window = lanes {L, L^1, L^8, L^9}, L = r16 & ~9; k order (0,0),(0,1),(1,0),(1,1)
        const int mn = r16 & 9;
        const int wy = y0 / 2 + gr, wx = 4 * gc8 + ((r16 & 7) >> 1);
        const size_t wpix = ((size_t)n * Hp + wy) * Wp + wx;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          float gv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (P >= 2) {
            const uint2 w2 = *reinterpret_cast<const uint2*>(gz + wpix * C + 16 * t + 4 * g);
            gv[0] = __uint_as_float(w2.x << 16); gv[1] = __uint_as_float(w2.x & 0xffff0000u);
            gv[2] = __uint_as_float(w2.y << 16); gv[3] = __uint_as_float(w2.y & 0xffff0000u);
          }
          float zo[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float zz = fmaxf(fmaf(yv[t][i], sc[t][i], sf[t][i]), 0.f);
            const float z1 = dppf<0xB1>(zz), z8 = dppf<0x128>(zz), z9 = dppf<0x128>(z1);
            if constexpr (P == 1) {
              zo[i] = fmaxf(fmaxf(zz, z1), fmaxf(z8, z9));
            } else {
              // the window's values in k order: lane L^m holds k = (m >> 3) * 2 + (m & 1)
              float wv[4];
              wv[0] = mn == 0 ? zz : mn == 1 ? z1 : mn == 8 ? z8 : z9;   // lane L
              wv[1] = mn == 1 ? zz : mn == 0 ? z1 : mn == 9 ? z8 : z9;   // L^1
              wv[2] = mn == 8 ? zz : mn == 9 ? z1 : mn == 0 ? z8 : z9;   // L^8
              wv[3] = mn == 9 ? zz : mn == 8 ? z1 : mn == 1 ? z8 : z9;   // L^9
              float best = wv[0];
              int a = 0;
#pragma unroll
              for (int k = 1; k < 4; ++k)
                if (wv[k] > best) { best = wv[k]; a = k; }
              const int kn = (mn >> 3) * 2 + (mn & 1);
              const float dz = (a == kn && best > 0.f) ? gv[i] : 0.f;
              if constexpr (P == 2) {
                const float xh = (yv[t][i] - mu[t][i]) * is[t][i];
                rs[t][i] += dz;
                rq[t][i] = fmaf(dz, xh, rq[t][i]);
              } else {
                zo[i] = fmaf(k1[t][i], dz, fmaf(kx[t][i], yv[t][i], k0[t][i]));   // dy
              }
            }
          }
          if constexpr (P == 1) {
            if ((r16 & 9) == 0)
              *reinterpret_cast<uint2*>(z + wpix * C + 16 * t + 4 * g) =
                  make_uint2(pack_bf16x2(zo[0], zo[1]), pack_bf16x2(zo[2], zo[3]));
          } else if constexpr (P == 3) {
            *reinterpret_cast<uint2*>(dys + p * DYS + 16 * t + 4 * g) =
                make_uint2(pack_bf16x2(zo[0], zo[1]), pack_bf16x2(zo[2], zo[3]));
          }
        }
      }
    }
    if constexpr (P == 3) {
      __syncthreads();
      for (int ks = wave; ks < KST; ks += 4) {
        const int P0 = 32 * ks;
        const int pa = P0 + kpx(g, 0, q4), pb = P0 + kpx(g, 1, q4);
        const bf16x8 bvv = fr8(trd(x9 + pa * XS9 + 4 * p4), trd(x9 + pb * XS9 + 4 * p4));
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16x8 av = fr8(trd(dys + pa * DYS + 16 * t + 4 * p4), trd(dys + pb * DYS + 16 * t + 4 * p4));
          acc3[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bvv, acc3[t], 0, 0, 0);
        }
      }
    }
  }

  if constexpr (P == 0 || P == 2) {
    if (cur_g >= 0) flush(cur_g);
    const int first = t0 < t1 ? t0 / tilesPG : 0, last = t0 < t1 ? (t1 - 1) / tilesPG : -1;
    zero_run();
    for (int gp = 0; gp < G; ++gp)
      if (gp < first || gp > last) flush(gp);
  }
  if constexpr (P == 3) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(wave * C + 16 * t + 4 * g + i) * 16 + r16] = acc3[t][i];
    __syncthreads();
    float* o = out + (size_t)blockIdx.x * C * 9;
    for (int e = tid; e < C * 9; e += 256) {
      const int c = e / 9, tap = e - c * 9;
      float sacc = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) sacc += red[(w * C + c) * 16 + tap];
      o[e] = sacc;
    }
  }
}

size_t c1r3_lds(int C, int W) {
  const int DYS = C == 16 ? 16 : C + 16;
  const size_t tpp = (size_t)(TRW * W + 31) / 32 * 32;
  const size_t xrw = ((size_t)(TRW + 2) * (W + 2) + 7) & ~(size_t)7;
  const size_t a = (tpp * XS9 + xrw + tpp * DYS) * 2;
  return std::max(a, (size_t)4 * C * 16 * 4);
}

int c1r3_grid(int N, int H) {
  (void)N;
  (void)H;
  return grid_cap(2 * ncu_c1w3());
}

}  // namespace

extern "C" {

// rows / slabs of a recompute pass for a 3x3 Cin-1 first layer (0: not served)
int avd_c1r3_rows(int pass, int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad) {
  if (getenv("AVDINO_C1R3_OFF")) return 0;
  if (dt != AVD_BF16 || Cin != 1 || K != 3 || pad != 1 || B <= 0 || N % B) return 0;
  if (Cout != 16 && Cout != 32 && Cout != 64) return 0;
  if (H % TRW || W % 8 || W > 128) return 0;
  if (c1r3_lds(Cout, W) > 80 * 1024) return 0;
  const int grid = c1r3_grid(N, H);
  switch (pass) {
    case 0: case 2: return 4 * grid;
    case 1: return 1;
    case 3: return grid;
    default: return 0;
  }
}

int avd_c1r3_launch(int pass, const void* x, const void* wk, const float* bias, const float* scale,
                    const float* shift, const float* mean, const float* invstd, const float* coef,
                    const void* gz, void* z, float* out, int N, int B, int H, int W, int Cout,
                    hipStream_t st) {
  const int grid = c1r3_grid(N, H);
  const size_t lds = c1r3_lds(Cout, W);
#define AVD_P(P_, C_)                                                                          \
  if (pass == P_ && Cout == C_)                                                                \
    c1r3_kernel<P_, C_><<<grid, 256, lds, st>>>((const bf16*)x, (const bf16*)wk, bias, scale,   \
                                                shift, mean, invstd, coef, (const bf16*)gz,    \
                                                (bf16*)z, out, N, B, H, W);
#define AVD_PC(C_) AVD_P(0, C_) else AVD_P(1, C_) else AVD_P(2, C_) else AVD_P(3, C_)
  AVD_PC(16) else AVD_PC(32) else AVD_PC(64) else return AVD_ERR_SHAPE;
#undef AVD_PC
#undef AVD_P
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
