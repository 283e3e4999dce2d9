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
// The same first layer WITHOUT a stored conv output (avd_cl_c1_recompute for Cin = 1, 3x3 pad 1
// -- the SimCLR / unimodal encoders' first layers -- and 5x5 pad 2 -- the CentralNet image
// conv1, unimodal.py:127-141): every pass rebuilds y = bf16(conv(x) + b) for a tile of TRW rows
// from the staged input rows (one v_mfma_f32_16x16x32_bf16 per 16 channels x 16 pixels, weights
// as A, k = tap: all 9 or 25 taps in one K = 32 step, so y is bit-identical to the stored-y
// forward and across passes) and then
//   pass 0: BN partial sums of y (per-block running sums, rows [C][G][4 * grid][2]);
//   pass 1: z = maxpool2(relu(y * scale + shift)) NHWC bf16;
//   pass 2: BN-backward partial sums (sum dz, sum dz * xhat) like avd_cl_bn_bwd_reduce;
//   pass 3: dy in LDS and the weight gradient, as c1w3_kernel (plus the im2col tile xk);
//   pass 4: pass 2's sums plus the moments dW is linear in: sum dz xk [C][KK] and the Gram rows
//           of the im2col tile [KK][KK + 1] (column KK = the ones tap: sum xk).
// A 16-pixel MFMA column group is a 2-row x 8-column patch, so a pooling window is the lanes
// {n, n^1, n^8, n^9} of a 16-lane row: DPP quad_perm / row_ror:8 exchanges.  Widths that are 4
// mod 8 (the 28-pixel image) run on WV = W + 4 virtual columns whose lanes are masked out of
// every output, sum and moment.  The next tile's input rows (and pooled gradient, passes 2-4)
// are register-prefetched into a second LDS buffer while the current tile computes: one barrier
// per tile (two in passes 3-4).
namespace {

template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
typedef __attribute__((ext_vector_type(2))) float f2;
typedef __attribute__((ext_vector_type(2))) short s2v;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;   // raw bf16 bits

constexpr int RXO = 8;                          // xr: column ix at RXO + ix, zero pads both sides

// blocks per CU (register budget: 512 / (4 x bpc) VGPRs per lane, no spills)
__host__ __device__ constexpr int c1r3_bpc(int P, int C, int K) {
  return K == 5 ? ((P >= 3 || C == 64) ? 2 : 3)
                : (P >= 3 || (P == 2 && C == 64)) ? 2 : (P == 2 || C == 64) ? 3 : 4;
}
__host__ __device__ constexpr int c1r3_ntap(int K) { return K * K + 1 <= 16 ? 1 : 2; }   // tap tiles

// the 8 taps 8 G_ .. 8 G_ + 7 of a lane's B fragment (k = tap) from the staged rows
template <int K, int G_>
__device__ __forceinline__ void btaps(us8& bs, const bf16* xp, int XS) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    constexpr int KK = K * K;
    const int t = 8 * G_ + q;
    if (t < KK) bs[q] = xp[(t / K) * XS + t % K];
  }
}

// TR: rows of one staged tile (4, or the whole sample for small maps: the 28x28 image, where a
// 4-row tile is too little work to hide the staging loads); passes 3-4 run their im2col /
// dy tiles and k-loop in chunks of TRW = 4 rows of it
template <int P, int C, int K, int TR>
__global__ __launch_bounds__(256, c1r3_bpc(P, C, K)) void c1r3_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coef, const bf16* __restrict__ gz, bf16* __restrict__ z,
    float* __restrict__ out, int N, int B, int H, int W, unsigned short* __restrict__ codes) {
  constexpr int NT = C / 16;
  constexpr int DYS = C == 16 ? 16 : C + 16;
  constexpr int KK = K * K, PADK = K / 2, NTAP = c1r3_ntap(K), XSK = 16 * NTAP;
  constexpr bool GZ = P >= 2;
  constexpr bool RED = P == 2 || P == 4;            // BN-backward partial sums
  constexpr bool WG = P >= 3;                       // im2col tile + weight-gradient MFMAs
  constexpr bool MOM = P == 4 || P == 5;            // moments: the ones tap and the Gram tiles
  constexpr bool ROUTED = P == 5;                   // dz from the forward's routing codes
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  constexpr int NGZ = TR == TRW ? NT : 4;          // pooled-gradient vectors per thread
  const int WV = (W + 7) & ~7;                      // virtual width (groups of 8 columns)
  const int TP = TRW * WV;                          // pixels of one compute chunk
  const int KST = TP / 32;                          // k-steps (TP is a multiple of 32)
  const int XS = WV + 2 * RXO;                      // xr row stride
  const int XB = (TR + K - 1) * XS;                 // one xr buffer
  const int Hp = H / 2, Wp = W / 2;
  const int GB = (TR / 2) * Wp * C;                 // one gz buffer (a tile's pooled gradient)
  const int CB = ROUTED ? (TR / 2) * Wp * (C / 4) : 0;   // one codes buffer (u16 per 4 channels)
  bf16* xr = sm;                                    // [2][TR + K - 1][XS]
  bf16* gzs = xr + 2 * XB;                          // [2][GB]
  unsigned short* cds = reinterpret_cast<unsigned short*>(gzs + (GZ ? 2 * GB : 0));   // [2][CB]
  bf16* xk = reinterpret_cast<bf16*>(cds + 2 * CB); // [TP][XSK] (passes 3-5)
  bf16* dys = xk + TP * XSK;                        // [TP][DYS] (passes 3, 4)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15, q4 = r16 >> 2, p4 = r16 & 3;
  const int tps = H / TR, ntiles = N * tps, G = N / B, tilesPG = ntiles / G;
  const int per = ntiles / (int)gridDim.x, extra = ntiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  const int gpr = WV / 8;                           // 16-pixel column groups per row pair
  // a 16-pixel column group is 2 rows x 8 columns: lane r16 -> pixel (r16 >> 3, r16 & 7)
  const int plane = (r16 >> 3) * WV + (r16 & 7);                // pixel within the group's rows
  const int xlane = (r16 >> 3) * XS + (r16 & 7) + RXO - PADK;
  const int mn = r16 & 9;                                       // position in the 2x2 window
  const int e1 = mn & 1, e8 = mn >> 3;                          // earlier-partner tie breaks
  const int wcol = (r16 & 7) >> 1;                              // window column within the group
  const int wlane = wcol * C + 4 * g;                           // window column, channel quad

  // weight rows (A): lane holds w[16 t + r16][8 g .. 8 g + 7] (taps >= KK are zero in wk)
  bf16x8 aw[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) aw[t] = *reinterpret_cast<const bf16x8*>(wk + (16 * t + r16) * 32 + 8 * g);
  f2 bv2[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      bv2[t][h] = bias ? f2{bias[16 * t + 4 * g + 2 * h], bias[16 * t + 4 * g + 2 * h + 1]} : f2{0.f, 0.f};

  // ---- staging: input rows y0-PADK .. y0+TR+PADK-1 (one vector per thread: 16 bytes, or 8
  // when W is 4 mod 8) and gz
  const bool v16 = (W & 7) == 0;
  const int cpr = v16 ? W / 8 : W / 4, nxv = (TR + K - 1) * cpr;
  const int xrow = tid / cpr, xcol = tid - xrow * cpr;
  u4 xv = u4{0u, 0u, 0u, 0u};
  u4 gv4[NGZ];
  u4 cv4 = u4{0u, 0u, 0u, 0u};                      // routed pass: one codes vector per thread
  auto load = [&](int tl) {
    const int n = tl / tps, y0 = (tl - n * tps) * TR;
    const int iy = y0 - PADK + xrow;
    if (tid < nxv) {
      const bool ok = (unsigned)iy < (unsigned)H;
      const bf16* src = x + ((size_t)n * H + iy) * W;
      if (v16) xv = ok ? *reinterpret_cast<const u4*>(src + 8 * xcol) : u4{0u, 0u, 0u, 0u};
      else {
        const uint2 v = ok ? *reinterpret_cast<const uint2*>(src + 4 * xcol) : make_uint2(0u, 0u);
        xv = u4{v.x, v.y, 0u, 0u};
      }
    }
    if constexpr (GZ) {
      const bf16* gb = gz + ((size_t)n * Hp + y0 / 2) * Wp * C;
#pragma unroll
      for (int j = 0; j < NGZ; ++j) {
        const int e = tid + 256 * j;
        if (8 * e < GB) gv4[j] = *reinterpret_cast<const u4*>(gb + 8 * e);
      }
    }
    if constexpr (ROUTED) {
      if (8 * tid < CB) cv4 = *reinterpret_cast<const u4*>(codes + ((size_t)n * Hp + y0 / 2) * Wp * (C / 4) + 8 * tid);
    }
  };
  auto put = [&](int buf) {
    if (tid < nxv) {
      bf16* d = xr + buf * XB + xrow * XS + RXO;
      if (v16) *reinterpret_cast<u4*>(d + 8 * xcol) = xv;
      else *reinterpret_cast<uint2*>(d + 4 * xcol) = make_uint2(xv.x, xv.y);
    }
    if constexpr (GZ) {
#pragma unroll
      for (int j = 0; j < NGZ; ++j) {
        const int e = tid + 256 * j;
        if (8 * e < GB) *reinterpret_cast<u4*>(gzs + buf * GB + 8 * e) = gv4[j];
      }
    }
    if constexpr (ROUTED) {
      if (8 * tid < CB) *reinterpret_cast<u4*>(cds + buf * CB + 8 * tid) = cv4;
    }
  };

  // per-block running sums (passes 0, 2, 4): rows blockIdx*4 + wave of R = 4 * grid per group
  float rs[NT][4], rq[NT][4];
  f2 rs2[NT][2], rq2[NT][2];                        // pass 0 keeps its sums packed
  int cur_g = -1;
  const int R = 4 * (int)gridDim.x, srow = blockIdx.x * 4 + wave;
  auto zero_run = [&]() {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { rs[t][i] = 0.f; rq[t][i] = 0.f; }
#pragma unroll
      for (int h = 0; h < 2; ++h) { rs2[t][h] = f2{0.f, 0.f}; rq2[t][h] = f2{0.f, 0.f}; }
    }
  };
  constexpr int NG = NTAP == 1 ? 1 : 3;             // Gram tiles (0,0) [(0,1) (1,1)]
  f4 acc3[NT][NTAP], gacc[NG];
  const int WSZ = C * KK + KK * (KK + 1);           // pass 4 moments per (row, group)
  float* wmo = out + (size_t)C * G * R * 2;         // pass 4: [R][G][WSZ] after the sums
  constexpr int MOMR = C * KK + KK * KK + KK + C;   // routed pass: M | Gram | S | sum dz
  auto flush = [&](int gp) {
    if constexpr (ROUTED) {
      float* o = out + ((size_t)srow * G + gp) * MOMR;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * t + 4 * g + i;
          if (r16 < KK) o[c * KK + r16] = acc3[t][0][i];
          else if (r16 == KK) o[C * KK + KK * KK + KK + c] = acc3[t][0][i];   // ones tap: sum dz
          acc3[t][0][i] = 0.f;
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a = 4 * g + i, c = r16;
        if (a < KK && c < KK) o[C * KK + a * KK + c] = gacc[0][i];
        else if (a < KK && c == KK) o[C * KK + KK * KK + a] = gacc[0][i];          // S
        gacc[0][i] = 0.f;
      }
      return;
    }
    if constexpr (P == 4) {
      // this wave's moments of group gp: sum dz xk [C][KK], then the Gram rows of xk
      // [KK][KK + 1] (column KK is the ones tap: sum xk); the lower tile (1,0) by symmetry
      float* o = wmo + ((size_t)srow * G + gp) * WSZ;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int nt = 0; nt < NTAP; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int tap = 16 * nt + r16;
            if (tap < KK) o[(16 * t + 4 * g + i) * KK + tap] = acc3[t][nt][i];
            acc3[t][nt][i] = 0.f;
          }
      float* gr = o + C * KK;
#pragma unroll
      for (int b = 0; b < NG; ++b) {
        const int ti = b == 2 ? 1 : 0, tj = b == 0 ? 0 : 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int a = 16 * ti + 4 * g + i, c = 16 * tj + r16;
          if (a < KK && c <= KK) gr[a * (KK + 1) + c] = gacc[b][i];
          if (b == 1 && c < KK && a < KK) gr[c * (KK + 1) + a] = gacc[b][i];
          gacc[b][i] = 0.f;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sa = P == 0 ? rs2[t][i >> 1][i & 1] : rs[t][i];
        const float sb = P == 0 ? rq2[t][i >> 1][i & 1] : rq[t][i];
        const float a = row16_sum(sa), b = row16_sum(sb);
        if (r16 == 0)
          *reinterpret_cast<float2*>(out + (((size_t)(16 * t + 4 * g + i) * G + gp) * R + srow) * 2) =
              make_float2(a, b);
      }
  };
  zero_run();
  // BN coefficients of the current group (passes 1-4): channels 16 t + 4 g + i
  f2 sc2[NT][2], sf2[NT][2];
  float c2[NT][4], c3[NT][4], c4[NT][4];
  int cg = -1;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int nt = 0; nt < NTAP; ++nt) acc3[t][nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < NG; ++b) gacc[b] = f4{0.f, 0.f, 0.f, 0.f};

  // zero both xr buffers (pads and virtual columns stay zero) and the dy tile (its virtual
  // columns stay zero: dz / dy is written for the valid lanes only)
  for (int i = tid; i < 2 * XB / 8; i += 256) reinterpret_cast<u4*>(xr)[i] = u4{0u, 0u, 0u, 0u};
  if constexpr (WG) {
    for (int i = tid; i < TP * (DYS / 8); i += 256)
      *reinterpret_cast<u4*>(dys + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};
  }
  if (t0 < t1) load(t0);
  __syncthreads();
  if (t0 < t1) put(t0 & 1);
  if (t0 + 1 < t1) load(t0 + 1);

  for (int ti = t0; ti < t1; ++ti) {
    const int n = ti / tps, y0 = (ti - n * tps) * TR, gb = n / B, buf = ti & 1;
    if constexpr (P == 0 || RED || ROUTED) {
      const int gi = ti / tilesPG;
      if (gi != cur_g) {
        if (cur_g >= 0) flush(cur_g);
        cur_g = gi;
        zero_run();
      }
    }
    if constexpr (P != 0 && !ROUTED) {
      if (gb != cg) {
        cg = gb;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int gc = gb * C + 16 * t + 4 * g + i;
            sc2[t][i >> 1][i & 1] = scale[gc]; sf2[t][i >> 1][i & 1] = shift[gc];
            if constexpr (RED) { c2[t][i] = mean[gc]; c3[t][i] = invstd[gc]; }
            if constexpr (P == 3) { c2[t][i] = coef[gc * 3]; c3[t][i] = coef[gc * 3 + 1]; c4[t][i] = coef[gc * 3 + 2]; }
          }
      }
    }
    __syncthreads();                    // buffer `buf` complete; the other one and xk/dys free
    if (ti + 1 < t1) put(buf ^ 1);
    if (ti + 2 < t1) load(ti + 2);      // in flight under this tile's work
    const bf16* xb = xr + buf * XB;
    const bf16* gzt = gzs + buf * GB;
    const size_t zt = ((size_t)n * Hp + y0 / 2) * Wp * C;            // tile's first pooled row
    // passes 0-2: the whole tile in one sweep; passes 3-4: chunks of TRW rows (im2col + dy
    // tiles, then the k-loop)
    constexpr int NCH = WG ? TR / TRW : 1;
    for (int cr = 0; cr < NCH; ++cr) {
      const int r0 = WG ? cr * TRW : 0;                                // first tile row of the sweep
      if (WG && cr > 0) __syncthreads();                               // last chunk's k-loop is done
      if constexpr (WG) {
        // im2col xk[p][tap] for the weight-gradient MFMAs (taps KK.. zero; pass 4: tap KK = 1);
        // virtual columns (c >= W) all zero
        for (int p = tid; p < TP; p += 256) {
          const int r = p / WV, c = p - r * WV;
          uint32_t w8[XSK / 2];
#pragma unroll
          for (int k = 0; k < XSK / 2; ++k) w8[k] = 0u;
          if (c < W) {
            if constexpr (MOM) w8[KK >> 1] = (KK & 1) ? 0x3F800000u : 0x3F80u;   // bf16 1.0 at tap KK
#pragma unroll
            for (int t = 0; t < KK; ++t) {
              const uint32_t b = __builtin_bit_cast(uint16_t, xb[(r0 + r + t / K) * XS + RXO - PADK + c + t % K]);
              w8[t >> 1] |= (t & 1) ? b << 16 : b;
            }
          }
#pragma unroll
          for (int v = 0; v < XSK / 8; ++v)
            *reinterpret_cast<u4*>(xk + p * XSK + 8 * v) = u4{w8[4 * v], w8[4 * v + 1], w8[4 * v + 2], w8[4 * v + 3]};
        }
      }
      // ---- y for the wave's column groups, straight from the staged rows; pass epilogues
      const int ngroups16 = ((WG ? TRW : TR) / 2) * gpr;
      for (int q = wave; q < ngroups16; q += 4) {
        const int grl = q / gpr, gc8 = q - grl * gpr;                   // wave-uniform
        const int gr = r0 / 2 + grl;                                    // row pair within the tile
        const bool vld = 8 * gc8 + (r16 & 7) < W;                       // a real (not virtual) column
        const bool wvld = 4 * gc8 + wcol < Wp;                          // its pooling window
        const bf16* xp = xb + 2 * gr * XS + 8 * gc8 + xlane;
        us8 bs = us8{};
        if (g == 0) btaps<K, 0>(bs, xp, XS);
        else if (g == 1) btaps<K, 1>(bs, xp, XS);
        else if (g == 2) btaps<K, 2>(bs, xp, XS);
        else btaps<K, 3>(bs, xp, XS);
        const bf16x8 bx = __builtin_bit_cast(bf16x8, bs);
        const int wg = wvld ? (gr * Wp + 4 * gc8) * C + wlane : 0;     // window (lane part in wlane)
        if constexpr (ROUTED) {
          // dz = the pooled gradient at the window position the forward's code names (nibble =
          // 1 + first argmax of relu(bn(y)) when > 0, else 0), 0 at the window's other pixels
          const int win = wvld ? gr * Wp + 4 * gc8 + wcol : 0;
          const unsigned me = 2u * (unsigned)e8 + (unsigned)e1 + 1u;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const uint2 gw = *reinterpret_cast<const uint2*>(gzt + wg + 16 * t);
            const unsigned cw = cds[buf * CB + win * (C / 4) + 4 * t + g];
            const unsigned gb4[4] = {gw.x & 0xffffu, gw.x >> 16, gw.y & 0xffffu, gw.y >> 16};
            unsigned d[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) d[i] = (vld && ((cw >> (4 * i)) & 0xFu) == me) ? gb4[i] : 0u;
            *reinterpret_cast<uint2*>(dys + (2 * grl * WV + 8 * gc8 + plane) * DYS + 16 * t + 4 * g) =
                make_uint2(d[0] | (d[1] << 16), d[2] | (d[3] << 16));
          }
          continue;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[t], bx, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          // y = bf16(acc + b) for the lane's 4 channels, as two packed pairs
          f2 y2[2];
          uint32_t yb[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f2 s2 = f2{acc[2 * h], acc[2 * h + 1]} + bv2[t][h];
            yb[h] = pack_bf16x2(s2.x, s2.y);
            y2[h] = f2{__uint_as_float(yb[h] << 16), __uint_as_float(yb[h] & 0xffff0000u)};
          }
          if constexpr (P == 0) {
            if (vld) {
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                rs2[t][h] += y2[h];
                rq2[t][h] = __builtin_elementwise_fma(y2[h], y2[h], rq2[t][h]);
              }
            }
          } else if constexpr (P == 1) {
            // relu(bn(y)) rounded to bf16 (monotone: the max of the rounded values is the rounded
            // max), window max over lanes ^1 then ^8 on packed non-negative bf16 as int16
            uint32_t m[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f2 v = __builtin_elementwise_fma(y2[h], sc2[t][h], sf2[t][h]);
              s2v r = __builtin_elementwise_max(__builtin_bit_cast(s2v, pack_bf16x2(v.x, v.y)), s2v{0, 0});
              r = __builtin_elementwise_max(r, __builtin_bit_cast(s2v, dppi<0xB1>(__builtin_bit_cast(int, r))));
              r = __builtin_elementwise_max(r, __builtin_bit_cast(s2v, dppi<0x128>(__builtin_bit_cast(int, r))));
              m[h] = __builtin_bit_cast(uint32_t, r);
            }
            if (mn == 0 && wvld)
              *reinterpret_cast<uint2*>(z + zt + wg + 16 * t) = make_uint2(m[0], m[1]);
            if (codes) {
              // routing codes for the backward: this lane's position (1 + k) where it is the
              // window's first argmax of bn(y) and > 0 (the tie rule of passes 2-4 below), OR-ed
              // over the window's four lanes
              unsigned cw = 0u;
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const f2 v = __builtin_elementwise_fma(y2[h], sc2[t][h], sf2[t][h]);
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                  const int vi = __float_as_int(v[e]);
                  const int u1 = dppi<0xB1>(vi) + e1, u8 = dppi<0x128>(vi) + e8,
                            u9 = dppi<0x128>(dppi<0xB1>(vi)) + e8;
                  const int thr = max(max(u1, u8), max(u9, 1));
                  cw |= (vi >= thr ? 2u * (unsigned)e8 + (unsigned)e1 + 1u : 0u) << (4 * (2 * h + e));
                }
              }
              cw |= (unsigned)dppi<0xB1>((int)cw);
              cw |= (unsigned)dppi<0x128>((int)cw);
              if (mn == 0 && wvld)
                codes[((size_t)n * Hp + y0 / 2 + gr) * Wp * (C / 4) + (4 * gc8 + wcol) * (C / 4) + 4 * t + g] =
                    (unsigned short)cw;
            }
          } else {
            // first argmax of the window (k order (0,0),(0,1),(1,0),(1,1); lane L^m holds
            // k = 2 (m >> 3) + (m & 1)) on bn(y) as signed ints: ordered like the floats wherever
            // one side is > 0, and only a positive maximum carries the gradient.  The lane wins
            // iff it beats its earlier partners strictly and its later ones or ties:
            // v > u  <=>  v >= u + 1 (ints), the +1 only toward earlier partners.
            const uint2 gw = *reinterpret_cast<const uint2*>(gzt + wg + 16 * t);
            const float gg[4] = {__uint_as_float(gw.x << 16), __uint_as_float(gw.x & 0xffff0000u),
                                 __uint_as_float(gw.y << 16), __uint_as_float(gw.y & 0xffff0000u)};
            float dz[4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f2 v = __builtin_elementwise_fma(y2[h], sc2[t][h], sf2[t][h]);
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const int vi = __float_as_int(v[e]);
                const int u1 = dppi<0xB1>(vi) + e1, u8 = dppi<0x128>(vi) + e8,
                          u9 = dppi<0x128>(dppi<0xB1>(vi)) + e8;
                const int thr = max(max(u1, u8), max(u9, 1));
                dz[2 * h + e] = (vi >= thr && vld) ? gg[2 * h + e] : 0.f;
              }
            }
            if constexpr (RED) {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float yy = y2[i >> 1][i & 1];
                const float xh = (yy - c2[t][i]) * c3[t][i];
                rs[t][i] += dz[i];
                rq[t][i] = fmaf(dz[i], xh, rq[t][i]);
              }
            }
            if constexpr (P == 4) {     // dz (exact in bf16: a pooled gradient or zero)
              *reinterpret_cast<uint2*>(dys + (2 * grl * WV + 8 * gc8 + plane) * DYS + 16 * t + 4 * g) =
                  make_uint2(pack_bf16x2(dz[0], dz[1]), pack_bf16x2(dz[2], dz[3]));
            } else if constexpr (P == 3) {
              float d[4];
#pragma unroll
              for (int i = 0; i < 4; ++i)
                d[i] = vld ? fmaf(c2[t][i], dz[i], fmaf(c3[t][i], y2[i >> 1][i & 1], c4[t][i])) : 0.f;   // dy
              *reinterpret_cast<uint2*>(dys + (2 * grl * WV + 8 * gc8 + plane) * DYS + 16 * t + 4 * g) =
                  make_uint2(pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3]));
            }
          }
        }
      }
      if constexpr (WG) {
        __syncthreads();
        for (int ks = wave; ks < KST; ks += 4) {
          const int P0 = 32 * ks;
          const int pa = P0 + kpx(g, 0, q4), pb = P0 + kpx(g, 1, q4);
          bf16x8 bvv[NTAP];
#pragma unroll
          for (int nt = 0; nt < NTAP; ++nt)
            bvv[nt] = fr8(trd(xk + pa * XSK + 16 * nt + 4 * p4), trd(xk + pb * XSK + 16 * nt + 4 * p4));
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const bf16x8 av = fr8(trd(dys + pa * DYS + 16 * t + 4 * p4), trd(dys + pb * DYS + 16 * t + 4 * p4));
#pragma unroll
            for (int nt = 0; nt < NTAP; ++nt)
              acc3[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bvv[nt], acc3[t][nt], 0, 0, 0);
          }
          // the same fragments are the A operands of the im2col Gram matrix (rows: taps, k: pixels)
          if constexpr (MOM) {
            gacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bvv[0], bvv[0], gacc[0], 0, 0, 0);
            if constexpr (NTAP == 2) {
              gacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bvv[0], bvv[NTAP - 1], gacc[1], 0, 0, 0);
              gacc[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bvv[NTAP - 1], bvv[NTAP - 1], gacc[2], 0, 0, 0);
            }
          }
        }
      }
    }
  }

  if constexpr (P == 0 || RED || ROUTED) {
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
      for (int nt = 0; nt < NTAP; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(wave * C + 16 * t + 4 * g + i) * XSK + 16 * nt + r16] = acc3[t][nt][i];
    __syncthreads();
    float* o = out + (size_t)blockIdx.x * C * KK;
    for (int e = tid; e < C * KK; e += 256) {
      const int c = e / KK, tap = e - c * KK;
      float sacc = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) sacc += red[(w * C + c) * XSK + tap];
      o[e] = sacc;
    }
  }
}

// staged tile rows: the whole 28-row sample for the small image maps, else 4
int c1r3_tr(int H, int W) { return (W <= 32 && H == 28) ? 28 : TRW; }

size_t c1r3_lds(int P, int C, int W, int K, int TR) {
  const int WV = (W + 7) & ~7;
  const size_t XB = (size_t)(TR + K - 1) * (WV + 2 * RXO);
  const size_t GB = P >= 2 ? (size_t)(TR / 2) * (W / 2) * C : 0;
  size_t e = 2 * XB + 2 * GB + (P == 5 ? 2 * (size_t)(TR / 2) * (W / 2) * (C / 4) : 0);
  const int XSK = 16 * c1r3_ntap(K);
  if (P >= 3) {
    const int DYS = C == 16 ? 16 : C + 16;
    e += (size_t)TRW * WV * (XSK + DYS);
  }
  return std::max(e * 2, P == 3 ? (size_t)4 * C * XSK * 4 : (size_t)0);
}

int c1r3_grid(int P, int C, int K) {
  const int bpc = K == 5 ? c1r3_bpc(P, C, 5) : c1r3_bpc(P, C, 3);
  return grid_cap(bpc * ncu_c1w3());
}

// dW of pass 4 from the row-summed moments m [G][C * KK + KK * (KK + 1)] and the BN-backward
// coefficients, in float64 (the kx and k0 terms are large and cancel: dy is centred):
//   dW[c][t] = sum_g k1 sum(dz xk_t) + kx sum(y xk_t) + k0 sum(xk_t),
//   sum(y xk_t) = sum_t' w[c][t'] Gram[t'][t] + b[c] sum(xk_t)   (y = w . xk + b)
__global__ void c1r3_combine_kernel(const float* __restrict__ m, const float* __restrict__ coef,
                                    const bf16* __restrict__ wk, const float* __restrict__ bias,
                                    float* __restrict__ dw, int G, int C, int KK) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= C * KK) return;
  const int c = e / KK, t = e - c * KK, WSZ = C * KK + KK * (KK + 1);
  const double b = bias ? (double)bias[c] : 0.0;
  double acc = 0.0;
  for (int g = 0; g < G; ++g) {
    const float* mg = m + (size_t)g * WSZ;
    const float* gram = mg + C * KK;
    const double sx = gram[t * (KK + 1) + KK];
    double sy = b * sx;
    for (int k = 0; k < KK; ++k) sy = fma((double)bf2f(wk[c * 32 + k]), (double)gram[k * (KK + 1) + t], sy);
    const float* k3 = coef + ((size_t)g * C + c) * 3;
    acc += (double)k3[0] * mg[e] + (double)k3[1] * sy + (double)k3[2] * sx;
  }
  dw[e] = (float)acc;
}

// BN backward + dW of a routed 3x3 first layer from the row-summed moments m [G][C*KK + KK*KK + KK
// + C] (M | Gram | S | sum dz) of pass 5, in float64 -- the c1r5 combine (c1r5.hip) for KK taps:
//   sum dz y = w . M + b sum dz;  sum dz xhat = (sum dz y - mean sum dz) invstd;
//   coef (k1, kx, k0) as avd_bn_bwd_finalize;  dW[c][t] = sum_g k1 M + kx (w Gram + b S) + k0 S;
//   dgamma / dbeta / dbias (= sum dy) summed over the groups.
constexpr int C1R3_GMAX = 32;
template <int C, int KK>
__global__ __launch_bounds__(256) void c1r3_codes_combine_kernel(
    const float* __restrict__ m, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    long long count, float* __restrict__ dw, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dbias, float* __restrict__ coef, int G) {
  constexpr int MOM = C * KK + KK * KK + KK + C;
  __shared__ double sk[C1R3_GMAX * C][3];
  __shared__ double s12[C1R3_GMAX * C][2];
  const int tid = threadIdx.x;
  const double n = (double)count;
  for (int i = tid; i < G * C; i += 256) {
    const int gq = i / C, c = i - gq * C;
    const float* mg = m + (size_t)gq * MOM;
    const double b = bias ? (double)bias[c] : 0.0;
    const double s1 = mg[C * KK + KK * KK + KK + c];
    double sy = b * s1;
    for (int t = 0; t < KK; ++t) sy = fma((double)bf2f(wk[c * 32 + t]), (double)mg[c * KK + t], sy);
    const double mu = mean[gq * C + c], is = invstd[gq * C + c], ga = gamma[c];
    const double s2 = (sy - mu * s1) * is;
    const double k1 = ga * is, kx = -ga * is * is * s2 / n, k0 = -ga * is * s1 / n + ga * is * is * mu * s2 / n;
    sk[i][0] = k1; sk[i][1] = kx; sk[i][2] = k0;
    s12[i][0] = s1; s12[i][1] = s2;
    if (coef) {
      coef[i * 3 + 0] = (float)k1;
      coef[i * 3 + 1] = (float)kx;
      coef[i * 3 + 2] = (float)k0;
    }
  }
  __syncthreads();
  if (tid < C) {
    double dg = 0.0, db = 0.0, dbi = 0.0;
    for (int gq = 0; gq < G; ++gq) {
      const int i = gq * C + tid;
      const double mu = mean[i];
      dg += s12[i][1];
      db += s12[i][0];
      dbi += sk[i][0] * s12[i][0] + sk[i][1] * mu * n + sk[i][2] * n;
    }
    if (dgamma) dgamma[tid] = (float)dg;
    if (dbeta) dbeta[tid] = (float)db;
    if (dbias) dbias[tid] = (float)dbi;
  }
  for (int e = tid; e < C * KK; e += 256) {
    const int c = e / KK, t = e - c * KK;
    double wr[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) wr[k] = (double)bf2f(wk[c * 32 + k]);
    const double b = bias ? (double)bias[c] : 0.0;
    double acc = 0.0;
    for (int gq = 0; gq < G; ++gq) {
      const float* mg = m + (size_t)gq * MOM;
      const float* gram = mg + C * KK;
      const double sx = gram[KK * KK + t];
      double sy = b * sx;
#pragma unroll
      for (int k = 0; k < KK; ++k) sy = fma(wr[k], (double)gram[k * KK + t], sy);
      const int i = gq * C + c;
      acc += sk[i][0] * mg[e] + sk[i][1] * sy + sk[i][2] * sx;
    }
    dw[e] = (float)acc;
  }
}

}  // namespace

namespace avd {
// the pixel-major forward passes of the 3x3 1 -> 32 layer (c1s3.hip)
bool c1s3_serves(int N, int B, int H, int W, int Cout);
int c1s3_stats_rows(int N, int B, int W);
int c1s3_stats(const void* x, const void* wk, const float* bias, float* out, int N, int B, int W,
               hipStream_t st);
int c1s3_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                     const float* shift, void* z, unsigned short* codes, int N, int B, int W,
                     hipStream_t st);
int c1s3_moments_rows(int N, int B, int H, int W, int Cout);
int c1s3_moments(const void* x, const void* gz, const unsigned short* codes, float* out, int N, int B,
                 int W, hipStream_t st);
}  // namespace avd

extern "C" {

int avd_c1r3_rows(int pass, int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad);
int avd_c1r3_launch(int pass, const void* x, const void* wk, const float* bias, const float* scale,
                    const float* shift, const float* mean, const float* invstd, const float* coef,
                    const void* gz, void* z, float* out, int N, int B, int H, int W, int Cout, int K,
                    hipStream_t st, unsigned short* codes);

// ---- the routed 3x3 first layer (1 -> 32, pad 1: the SimCLR / unimodal encoders' conv1,
// dino.py:18-73): the forward's pass 1 writes routing codes (one nibble per pooling window and
// channel, u16 per 4 channels: [N][H/2][W/2][C/4]), the backward is pass 5 (moments from x, the
// pooled gradient and the codes; no y, no BN coefficients) + the float64 combine.
int avd_cl_c1r3_codes_rows(int N, int B, int H, int W, int Cout) {
  if (Cout != 32 || B <= 0 || N % B || N / B > C1R3_GMAX) return 0;
  if (!avd_c1r3_rows(4, AVD_BF16, N, B, 1, H, W, Cout, 3, 1)) return 0;
  if (const int r = c1s3_moments_rows(N, B, H, W, Cout)) return r;     // 28^2 / 112^2: c1s3.hip
  return 4 * c1r3_grid(5, Cout, 3);
}

int avd_cl_c1r3_codes_cols(int Cout) { return Cout * 9 + 81 + 9 + Cout; }

int avd_cl_c1r3_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                            const float* shift, void* z, unsigned short* codes, int N, int B, int H,
                            int W, int Cout, void* stream) {
  if (!x || !wk || !scale || !shift || !z || !codes) return AVD_ERR_ARG;
  if (!avd_cl_c1r3_codes_rows(N, B, H, W, Cout)) return AVD_ERR_SHAPE;
  return avd_c1r3_launch(1, x, wk, bias, scale, shift, nullptr, nullptr, nullptr, nullptr, z, nullptr,
                         N, B, H, W, Cout, 3, avd_stream(stream), codes);
}

int avd_cl_c1r3_moments_codes(const void* x, const void* wk, const void* gz, const unsigned short* codes,
                              float* out, int N, int B, int H, int W, int Cout, void* stream) {
  if (!x || !wk || !gz || !codes || !out) return AVD_ERR_ARG;
  if (!avd_cl_c1r3_codes_rows(N, B, H, W, Cout)) return AVD_ERR_SHAPE;
  if (c1s3_moments_rows(N, B, H, W, Cout)) return c1s3_moments(x, gz, codes, out, N, B, W, avd_stream(stream));
  return avd_c1r3_launch(5, x, wk, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, gz, nullptr, out,
                         N, B, H, W, Cout, 3, avd_stream(stream), const_cast<unsigned short*>(codes));
}

int avd_cl_c1r3_codes_combine(const float* moments, const void* wk, const float* bias,
                              const float* gamma, const float* mean, const float* invstd,
                              long long count, float* dw, float* dgamma, float* dbeta, float* dbias,
                              float* coef, int G, int Cout, void* stream) {
  if (!moments || !wk || !gamma || !mean || !invstd || !dw) return AVD_ERR_ARG;
  if (G <= 0 || G > C1R3_GMAX || count <= 1 || Cout != 32) return AVD_ERR_SHAPE;
  c1r3_codes_combine_kernel<32, 9><<<1, 256, 0, avd_stream(stream)>>>(
      moments, (const bf16*)wk, bias, gamma, mean, invstd, count, dw, dgamma, dbeta, dbias, coef, G);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// rows / slabs of a recompute pass for a Cin-1 first layer, 3x3 pad 1 or 5x5 pad 2 (0: not served)
int avd_c1r3_rows(int pass, int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad) {
  if (dt != AVD_BF16 || Cin != 1 || !((K == 3 && pad == 1) || (K == 5 && pad == 2)) || B <= 0 || N % B) return 0;
  // the 5x5 image conv1 (1->32 at 28^2): standalone its passes measure about what the stored-y
  // chain takes (tools/c1bench.py: 98 + 112 + 332 us vs 542 us for conv + pool + reduce + apply +
  // wgrad), but in the step they win: no 360 MB y written and re-read beside the concurrent
  // streams (round 3 same-box A/B: 175.7k vs 173.5k pairs/s, profiles/r3_ab_c1r5.txt).
  if (Cout != 16 && Cout != 32 && Cout != 64) return 0;
  if (K == 5 && Cout != 32) return 0;                   // instantiated: the CentralNet image conv1
  if (H % TRW || W % 4 || W > 128 || pass < 0 || pass > 4) return 0;
  const int TR = c1r3_tr(H, W);
  if (TR != TRW && ((W > 32) || Cout > 32)) return 0;   // whole-sample tiles: gz staging bound
  if ((TR + K - 1) * (W % 8 ? W / 4 : W / 8) > 256) return 0;                // one x vector per thread
  if (c1r3_lds(3, Cout, W, K, TR) > 80 * 1024 || c1r3_lds(4, Cout, W, K, TR) > 80 * 1024) return 0;   // every pass, or none
  // 3x3 1 -> 32 at 28^2 / 112^2: statistics on the pixel-major pass (c1s3.hip)
  if (K == 3 && pass == 0 && c1s3_serves(N, B, H, W, Cout)) return c1s3_stats_rows(N, B, W);
  const int grid = c1r3_grid(pass, Cout, K);
  return pass == 1 ? 1 : pass == 3 ? grid : 4 * grid;   // pass 4: rows R of both its outputs
}

int avd_c1r3_launch(int pass, const void* x, const void* wk, const float* bias, const float* scale,
                    const float* shift, const float* mean, const float* invstd, const float* coef,
                    const void* gz, void* z, float* out, int N, int B, int H, int W, int Cout, int K,
                    hipStream_t st, unsigned short* codes) {
  if (K == 3 && (pass == 0 || pass == 1) && c1s3_serves(N, B, H, W, Cout)) {
    // the pixel-major passes (c1s3.hip): one pooling window per lane
    if (pass == 0) return c1s3_stats(x, wk, bias, out, N, B, W, st);
    return c1s3_apply_codes(x, wk, bias, scale, shift, z, codes, N, B, W, st);
  }
  const int grid = c1r3_grid(pass, Cout, K);
  const int TR = c1r3_tr(H, W);
  const size_t lds = c1r3_lds(pass, Cout, W, K, TR);
#define AVD_P(P_, C_, K_, TR_)                                                                 \
  if (pass == P_ && Cout == C_ && K == K_ && TR == TR_)                                        \
    c1r3_kernel<P_, C_, K_, TR_><<<grid, 256, lds, st>>>((const bf16*)x, (const bf16*)wk, bias,   \
                                                         scale, shift, mean, invstd, coef,      \
                                                         (const bf16*)gz, (bf16*)z, out, N, B, H, W, codes);
#define AVD_PC(C_, K_, TR_) AVD_P(0, C_, K_, TR_) else AVD_P(1, C_, K_, TR_) else AVD_P(2, C_, K_, TR_) \
  else AVD_P(3, C_, K_, TR_) else AVD_P(4, C_, K_, TR_)
  AVD_PC(16, 3, 4) else AVD_PC(32, 3, 4) else AVD_PC(64, 3, 4) else AVD_PC(32, 5, 4)
  else AVD_PC(16, 3, 28) else AVD_PC(32, 3, 28) else AVD_PC(32, 5, 28)
  else AVD_P(5, 32, 3, 4) else AVD_P(5, 32, 3, 28) else return AVD_ERR_SHAPE;
#undef AVD_PC
#undef AVD_P
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_c1r3_combine(const float* m, const float* coef, const void* wk, const float* bias,
                     float* dw, int G, int Cout, int K, hipStream_t st) {
  const int KK = K * K;
  c1r3_combine_kernel<<<avd_cdiv(Cout * KK, 64), 64, 0, st>>>(m, coef, (const bf16*)wk, bias, dw, G,
                                                              Cout, KK);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
