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
