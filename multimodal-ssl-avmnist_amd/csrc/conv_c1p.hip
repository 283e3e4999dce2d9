// First-layer convolution of the CentralNet audio branch (CentralUnimodalAudio.conv1,
// unimodal.py:160-190: Conv2d(1, 8, 5, padding=2) on 112x112 spectrograms) as a "pixel-pair"
// implicit GEMM on v_mfma_f32_16x16x32_bf16, channels-last bf16 output + fused BatchNorm
// partial statistics -- a drop-in for conv_c1_kernel on this shape (same outputs, same
// partial-row layout).
//
// Why a dedicated kernel: with 8 output channels the generic Cin=1 kernel fills half of the
// MFMA M dimension and gathers every B element with its own 2-byte LDS read (~100 VALU
// instructions per 16 outputs).  Here the M dimension holds (pixel offset j in a horizontal
// pair, channel c) -- 16 useful rows -- and K holds the 5x6 input patch that covers BOTH
// pixels of the pair (30 of 32 taps):
//   A[(j,c)][ky*6 + kx'] = w[c][ky][kx' - j]      (0 where kx' - j is outside [0,5))
//   B[ky*6 + kx'][pair]  = x[y + ky - 2][x0 + kx' - 2]     (x0 = even column of the pair)
// A lane's 8 consecutive k of B are 4 aligned bf16 PAIRS of the input rows, so the whole
// B fragment is 4 ds_read_b32 with constant offsets (no packing), and one MFMA produces
// 32 outputs x 8 channels.  C layout (col = lane&15 = pair, row = 4*(lane>>4)+i): lane l holds
// pixel (pair l&15, j = l>>5), channels 4*((l>>4)&1) .. +3 -> one 8-byte NHWC store.
// A 16-pixel-wide, 2-row strip is one MFMA column tile: pairs 0-7 = row 0, 8-15 = row 1.
#include <algorithm>
#include <cstdlib>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(2))) unsigned u2;
typedef __attribute__((ext_vector_type(2))) unsigned short us2;

constexpr int TH = 16;         // output rows per block (one sample)
constexpr int XOFF = 8;        // LDS column of image column 0 (16-byte aligned data)
constexpr int ITW = 144;       // LDS row stride in bf16 (72 dwords = 8 mod 64 banks)
constexpr int ITWD = ITW / 2;
constexpr int COUT = 8;
constexpr int MTMAX = 7;       // 16-pixel column tiles per strip (W <= 112)

// (row, dword) of the 4 B-fragment dwords for lane half h = lane>>4 (see header)
__device__ __forceinline__ int boff(int h, int d) {
  constexpr int R[4][4] = {{0, 0, 0, 1}, {1, 1, 2, 2}, {2, 3, 3, 3}, {4, 4, 4, 4}};
  constexpr int D[4][4] = {{0, 1, 2, 0}, {1, 2, 0, 1}, {2, 0, 1, 2}, {0, 1, 2, 0}};
  return R[h][d] * ITWD + D[h][d];
}

__device__ const u4 kZeroF = {0u, 0u, 0u, 0u};

__global__ __launch_bounds__(256) void conv_c1p8_kernel(const bf16* __restrict__ x,
                                                        const bf16* __restrict__ wk,
                                                        const float* __restrict__ bias,
                                                        bf16* __restrict__ y,
                                                        float* __restrict__ stats, int N, int H,
                                                        int W, int tps) {
  __shared__ __attribute__((aligned(16))) bf16 xs[(TH + 4) * ITW];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n = blockIdx.x;                     // one block = one sample, all its row tiles
  const int h = lane >> 4, p = lane & 15, j = lane >> 5, cs = h & 1;

  // ---- A fragment (weights) for this lane: row m = (j', c'), k = 8h .. 8h+7; wk is the
  // avd_cl_weight_layout image (bf16 [16 rows][32]: wk[c*32 + tap] = w[c][0][tap])
  bf16x8 a;
  {
    const int m = lane & 15, jj = m >> 3, c = m & 7;
    __bf16 e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 8 * h + q, ky = k / 6, kx = k % 6 - jj;
      const bool ok = k < 30 && kx >= 0 && kx < 5;
      const float v = bf2f(wk[c * 32 + (ok ? ky * 5 + kx : 0)]);
      e[q] = (__bf16)(ok ? v : 0.f);
    }
    a = bf16x8{e[0], e[1], e[2], e[3], e[4], e[5], e[6], e[7]};
  }
  float bv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bv[i] = bias ? bias[4 * cs + i] : 0.f;
  const unsigned* xd = reinterpret_cast<const unsigned*>(xs);
  const int q = p & 7, rp = p >> 3;
  int off[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) off[d] = boff(h, d) + rp * ITWD + q + 3;   // + (x0 - 2 + XOFF)/2
  float ss[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
  const int mts = W >> 4, cpr = W >> 3;
  // input rows: <= 2 16-byte vectors per thread (W <= 128), register-prefetched one tile ahead
  // so their latency hides under the current tile's MFMAs and stores
  const int nxt = (TH + 4) * cpr;
  int xr[2], xoff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = tid + 256 * s;
    const int r = t / cpr, c = t - r * cpr;
    xr[s] = t < nxt ? r : -(1 << 20);
    xoff[s] = (r - 2) * W + 8 * c;
  }
  u4 xv[2];
  auto load_x = [&](int ty0) {
    const bf16* xb = x + ((size_t)n * H + ty0) * W;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool ok = (unsigned)(ty0 - 2 + xr[s]) < (unsigned)H;
      xv[s] = ldg16(ok ? (const void*)(xb + xoff[s]) : &kZeroF);
    }
  };
  load_x(0);
  for (int tile = 0; tile < tps; ++tile) {
    const int ty0 = tile * TH;
    if (tile) __syncthreads();
    // ---- stage rows ty0-2 .. ty0+TH+1 (zero outside the image); pad columns zeroed
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = tid + 256 * s;
      if (t < nxt) {
        const int r = t / cpr, c = t - r * cpr;
        *reinterpret_cast<u4*>(xs + r * ITW + XOFF + 8 * c) = xv[s];
      }
    }
    if (tid < (TH + 4) * 2) {
      const int r = tid >> 1, side = tid & 1;
      *reinterpret_cast<u4*>(xs + r * ITW + (side ? XOFF + W : 0)) = u4{0u, 0u, 0u, 0u};
    }
    if (tile + 1 < tps) load_x(ty0 + TH);
    __syncthreads();
    for (int s = wave; s < TH / 2; s += 4) {      // 2-row strips
      const int oy = ty0 + 2 * s + rp;
      bf16* yrow = y + ((size_t)n * H + oy) * W * COUT + 4 * cs;
      for (int mt = 0; mt < mts; ++mt) {
        const int base = 2 * s * ITWD + 8 * mt;
        const u4 bw = u4{xd[base + off[0]], xd[base + off[1]], xd[base + off[2]], xd[base + off[3]]};
        f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, bw),
                                                         f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const uint32_t lo = pack_bf16x2(acc[0] + bv[0], acc[1] + bv[1]);
        const uint32_t hi = pack_bf16x2(acc[2] + bv[2], acc[3] + bv[3]);
        const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                            __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ss[i] += v[i];
          sq[i] = fmaf(v[i], v[i], sq[i]);
        }
        const int ox = 16 * mt + 2 * q + j;
        *reinterpret_cast<uint2*>(yrow + (size_t)ox * COUT) = make_uint2(lo, hi);
      }
    }
  }
  if (!stats) return;
  // per-wave BN partial row (sum, sumsq of the stored values): reduce over the 32 lanes that
  // hold the same 4 channels (lane bits 0-3: pair, bit 5: j)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int m = 1; m <= 32; m <<= 1) {
      if (m == 16) continue;
      ss[i] += __shfl_xor(ss[i], m, 64);
      sq[i] += __shfl_xor(sq[i], m, 64);
    }
  }
  if ((lane & 47) == 0) {                        // lanes 0 (channels 0-3) and 16 (4-7)
    const size_t nrows = (size_t)N * 4;             // one row per (sample, wave)
    const size_t row = (size_t)blockIdx.x * 4 + wave;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 4 * cs + i;
      stats[((size_t)co * nrows + row) * 2] = ss[i];
      stats[((size_t)co * nrows + row) * 2 + 1] = sq[i];
    }
  }
}

}  // namespace

// Shape served by this kernel: Cin 1, Cout 8, 5x5, bf16, output (= input, pad 2) H % 16 == 0,
// W % 16 == 0, W <= 128 (the caller rejects other paddings for this shape).
bool avd_c1p8_eligible(int dt, int Cin, int Cout, int K, int Ho, int Wo) {
  return dt == AVD_BF16 && Cin == 1 && Cout == 8 && K == 5 && Ho % TH == 0 && Wo % 16 == 0 &&
         Wo <= 16 * MTMAX;
}

int avd_c1p8_stat_rows(int H, int B) { (void)H; return B * 4; }

int avd_c1p8_fwd(const void* x, const void* wk, const float* bias, void* y, float* stats, int N,
                 int H, int W, hipStream_t st) {
  const int tps = H / TH;
  conv_c1p8_kernel<<<N, 256, 0, st>>>((const bf16*)x, (const bf16*)wk, bias, (bf16*)y, stats, N,
                                      H, W, tps);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// ============================================================================ backward
// BatchNorm-backward apply + weight gradient of the same layer, fused (dy never reaches HBM):
//   dy[p, c] = k1 * dz + kx * y + k0,  dz = pooled grad at the window's first-max of
//   relu(y*scale + shift) when that max is > 0 (bwd_apply_cl_kernel semantics, bn_cl.hip)
//   dW[c][ky][kx] = sum_p dy[p, c] * x[p + (ky-2, kx-2)]
// as the pixel-pair GEMM D[(j,c)][ky*6 + kx'] = sum_pairs dY[(j,c)][pair] * X[pair][tap],
// dW[c][ky][kx] = D[(0,c)][ky*6+kx] + D[(1,c)][ky*6+kx+1]:
//   A = dY: the block's dy tile in LDS in natural NHWC order, i.e. one 32-byte row of 16
//       (j,c) values per pixel pair, read column-major with two ds_read_b64_tr_b16;
//   B = X: 8 consecutive pairs of one tap = 8 input pixels 2 apart -> deinterleaved (by
//       column parity) and shifted (by -1/0/+1 pair) copies of the input rows make it one
//       aligned ds_read_b128.
// Each block walks tiles of TH rows x W of one sample and writes one partial dW slab
// (deterministic: reduced by avd_sum_rows in slab order).
namespace {

constexpr int WMAX = 112;                 // widest map served (the 112x112 spectrogram)
constexpr int XCW = 64;                   // pairs per copy row (>= WMAX/2, 16-byte rows)

typedef __attribute__((ext_vector_type(4))) short s4;
typedef __attribute__((address_space(3))) s4 lds_s4;

__device__ __forceinline__ void st16(bf16* p, bf16 v) { *p = v; }
__device__ const u4 kZeroC1 = {0u, 0u, 0u, 0u};

// parity/shift input copies of the backward kernel: element offset of (b, a, r, P).  Row /
// copy strides of 80 / 1648 / 5056 elements (160 / 3296 / 10112 B) spread the 16 taps of a
// B-fragment read over distinct 16-byte bank windows: 13.1 instead of 52 LDS cycles per
// pair of ds_read_b128 (tools/lds_bank_sim.py); 20.2 KB instead of 15.4 KB
constexpr int XB_RS = 80, XB_CA = 1648, XB_CB = 5056;
__device__ __forceinline__ int xbo(int b, int a, int r, int P) {
  return b * XB_CB + a * XB_CA + r * XB_RS + P;
}
// dy tile column of pixel cx in tile row ry: in the odd k-blocks (kb = ry * segs + cx / 16)
// the two 8-pixel halves of the 16-pixel segment trade places, so the 4 k-blocks one MFMA
// step reads (kb = 4ks .. 4ks+3, 256 B apart) fall on both halves of the 64 banks:
// no 2-way conflict between the lane halves of ds_read_b64_tr_b16
__device__ __forceinline__ int dys_px(int ry, int cx, int segs) {
  return cx ^ (((ry * segs + (cx >> 4)) & 1) << 3);
}

__global__ __launch_bounds__(256) void c1p8_bwd_wgrad_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ y, const bf16* __restrict__ gz,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ coef, float* __restrict__ parts, int B, int H, int W, int ntiles,
    int tps) {
  static_assert(XB_CA >= (TH + 4) * XB_RS && XB_CB >= 3 * XB_CA && XB_RS >= WMAX / 2, "xc strides");
  __shared__ __attribute__((aligned(16))) bf16 xc[2 * XB_CB];
  __shared__ __attribute__((aligned(16))) bf16 dys[TH * WMAX * COUT];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int gq = lane >> 4, col = lane & 15;
  const int Hp = H >> 1, Wp = W >> 1, cpr = W >> 3, segs = W >> 4;
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  // B-operand copy / row offset for this lane's tap in each tap tile
  int bb[2], ba[2], bky[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    int t = 16 * tt + col;
    if (t >= 30) t = 29;                   // padded taps: any finite data (their D is unused);
                                           // tap 29 as column 13 reads: a broadcast, no bank conflict
    const int ky = t / 6, k2 = t % 6 - 2;  // kx' - 2 = 2a' + b
    bky[tt] = ky;
    bb[tt] = k2 & 1;
    ba[tt] = (k2 >= 0 ? k2 >> 1 : -1) + 1;
  }
  // every global load of a tile is issued before the block's barrier (the previous tile's
  // MFMAs may still read LDS): per thread <= 2 input-row vectors and <= 2 pooling windows
  // (W <= WMAX), past-the-end slots read a zero vector (no select on the loaded data)
  const int nxt = (TH + 4) * cpr, nwin = (TH / 2) * Wp;
  // tile-invariant per-lane offsets (elements, relative to the tile's first row): the loads
  // are then a block-uniform base + one 32-bit offset
  int xr[2], xoff[2], yoff[2], goff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = tid + 256 * s;
    const int r = t / cpr, c = t - r * cpr;
    xr[s] = t < nxt ? r : -(1 << 20);         // out-of-slot lanes: never a valid row
    xoff[s] = (r - 2) * W + 8 * c;
    const int w = min(tid + 256 * s, nwin - 1);   // out-of-slot windows re-read the last one
    const int hp = w / Wp, wp = w - hp * Wp;
    yoff[s] = (2 * hp * W + 2 * wp) * COUT;
    goff[s] = (hp * Wp + wp) * COUT;
  }
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tps, ty0 = (tile - n * tps) * TH, grp = n / B;
    const bf16* xb = x + ((size_t)n * H + ty0) * W;
    const bf16* yb = y + ((size_t)n * H + ty0) * W * COUT;
    const bf16* gb = gz + ((size_t)n * Hp + (ty0 >> 1)) * Wp * COUT;
    u4 xv[2], yv4[2][4], gv[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool ok = (unsigned)(ty0 - 2 + xr[s]) < (unsigned)H;
      xv[s] = ldg16(ok ? (const void*)(xb + xoff[s]) : &kZeroC1);
      const bf16* p = yb + yoff[s];
      yv4[s][0] = ldg16(p);
      yv4[s][1] = ldg16(p + COUT);
      yv4[s][2] = ldg16(p + W * COUT);
      yv4[s][3] = ldg16(p + (W + 1) * COUT);
      gv[s] = ldg16(gb + goff[s]);
    }
    float sc[COUT], sf[COUT], k1[COUT], kx[COUT], k0[COUT];
#pragma unroll
    for (int e = 0; e < COUT; ++e) {
      const int gc = grp * COUT + e;
      sc[e] = scale[gc];
      sf[e] = shift[gc];
      k1[e] = coef[gc * 3];
      kx[e] = coef[gc * 3 + 1];
      k0[e] = coef[gc * 3 + 2];
    }
    __syncthreads();
    // ---- input rows ty0-2 .. ty0+THB+1 -> parity/shift copies xc[b][a][r][P] = x[2(P+a-1)+b]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = tid + 256 * s;
      if (t >= nxt) continue;
      const int r = t / cpr, c = t - r * cpr;
      const unsigned wv[4] = {xv[s].x, xv[s].y, xv[s].z, xv[s].w};
      // wv[d] holds pixels 8c+2d (low) and 8c+2d+1 (high) = pair 4c+d of parity 0 / 1
      const unsigned e0 = (wv[0] & 0xffffu) | (wv[1] << 16), e1 = (wv[2] & 0xffffu) | (wv[3] << 16);
      const unsigned o0 = (wv[0] >> 16) | (wv[1] & 0xffff0000u), o1 = (wv[2] >> 16) | (wv[3] & 0xffff0000u);
      const unsigned ev[2] = {e0, e1}, od[2] = {o0, o1};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const unsigned lo = b ? od[0] : ev[0], hi = b ? od[1] : ev[1];   // pairs 4c..4c+3
        *reinterpret_cast<uint2*>(&xc[xbo(b, 1, r, 4 * c)]) = make_uint2(lo, hi);
        // a = 0: P = pair + 1;  a = 2: P = pair - 1
        bf16* d0 = &xc[xbo(b, 0, r, 4 * c + 1)];
        st16(d0, (bf16)(lo & 0xffffu));
        *reinterpret_cast<unsigned*>(d0 + 1) = (lo >> 16) | (hi << 16);
        st16(d0 + 3, (bf16)(hi >> 16));
        bf16* d2 = &xc[xbo(b, 2, r, 4 * c)];
        if (c > 0) st16(d2 - 1, (bf16)(lo & 0xffffu));
        *reinterpret_cast<unsigned*>(d2) = (lo >> 16) | (hi << 16);
        st16(d2 + 2, (bf16)(hi >> 16));
      }
    }
    // pairs whose source pixel lies outside the row: P = 0 of a = 0, P = W/2 - 1 of a = 2
    if (tid < (TH + 4) * 2) {
      const int r = tid >> 1, b = tid & 1;
      xc[xbo(b, 0, r, 0)] = bf16(0);
      xc[xbo(b, 2, r, Wp - 1)] = bf16(0);
    }
    // ---- dy of the tile's windows into dys (natural NHWC rows)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int w = tid + 256 * s;
      if (w >= nwin) continue;
      const int hp = w / Wp, wp = w - hp * Wp;
      float yv[4][COUT];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned wv[4] = {yv4[s][k].x, yv4[s][k].y, yv4[s][k].z, yv4[s][k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          yv[k][2 * i] = __uint_as_float(wv[i] << 16);
          yv[k][2 * i + 1] = __uint_as_float(wv[i] & 0xffff0000u);
        }
      }
      float gg[COUT];
      {
        const unsigned wv[4] = {gv[s].x, gv[s].y, gv[s].z, gv[s].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gg[2 * i] = __uint_as_float(wv[i] << 16);
          gg[2 * i + 1] = __uint_as_float(wv[i] & 0xffff0000u);
        }
      }
      float dv[4][COUT];
#pragma unroll
      for (int e = 0; e < COUT; ++e) {
        // first max of relu(y*scale + shift) over the window (max-pool's tie rule) as lane
        // masks: the first k whose value equals the maximum
        float rv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) rv[k] = fmaxf(fmaf(yv[k][e], sc[e], sf[e]), 0.f);
        const float m = fmaxf(fmaxf(rv[0], rv[1]), fmaxf(rv[2], rv[3]));
        const bool e0 = rv[0] == m, e1 = !e0 && rv[1] == m, e2 = !e0 && !e1 && rv[2] == m;
        const bool e3 = !e0 && !e1 && !e2;
        const float dz = m > 0.f ? gg[e] : 0.f;
        dv[0][e] = fmaf(k1[e], e0 ? dz : 0.f, fmaf(kx[e], yv[0][e], k0[e]));
        dv[1][e] = fmaf(k1[e], e1 ? dz : 0.f, fmaf(kx[e], yv[1][e], k0[e]));
        dv[2][e] = fmaf(k1[e], e2 ? dz : 0.f, fmaf(kx[e], yv[2][e], k0[e]));
        dv[3][e] = fmaf(k1[e], e3 ? dz : 0.f, fmaf(kx[e], yv[3][e], k0[e]));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ry = 2 * hp + (k >> 1), cx = 2 * wp + (k & 1);
        *reinterpret_cast<u4*>(&dys[(ry * WMAX + dys_px(ry, cx, segs)) * COUT]) =
            u4{pack_bf16x2(dv[k][0], dv[k][1]), pack_bf16x2(dv[k][2], dv[k][3]),
               pack_bf16x2(dv[k][4], dv[k][5]), pack_bf16x2(dv[k][6], dv[k][7])};
      }
    }
    __syncthreads();
    // ---- MFMA over the tile's pixel pairs: k-block kb = (row r, 8-pair segment sg); wave w
    // takes kb = 4 ks + gq for ks = w, w + 4, ... (kb advances by 16: its parity, i.e. the
    // dys half swap, is fixed per lane).  The next k-block's operands are read before the
    // current MFMAs issue.
    const int nkb = TH * segs;
    if (4 * wave < nkb) {
      typedef __attribute__((ext_vector_type(8))) short s8;
      const int q = col >> 2, pp = col & 3;
      const int kb0 = 4 * wave + gq;
      int r = kb0 / segs, sg = kb0 - r * segs;
      const int hsw = (kb0 & 1) << 3;
      // A: rows P0 + 4*half + q, columns 4p .. 4p+3 of the pair rows (32 B each)
      const int aoff0 = ((2 * q) ^ hsw) * COUT + 4 * pp, aoff1 = ((8 + 2 * q) ^ hsw) * COUT + 4 * pp;
      const int boff0 = xbo(bb[0], ba[0], bky[0], 0), boff1 = xbo(bb[1], ba[1], bky[1], 0);
      const int dr = 16 / segs, dsg = 16 - dr * segs;
      s4 h0, h1;
      u4 w0, w1;
      auto load = [&](s4& a0, s4& a1, u4& c0, u4& c1) {
        const int P0 = 8 * sg, ab = (r * WMAX + 2 * P0) * COUT, bs = r * XB_RS + P0;
        a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&dys[ab + aoff0]);
        a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&dys[ab + aoff1]);
        c0 = *reinterpret_cast<const u4*>(&xc[bs + boff0]);
        c1 = *reinterpret_cast<const u4*>(&xc[bs + boff1]);
      };
      load(h0, h1, w0, w1);
      for (int ks = wave;; ks += 4) {
        const bool more = 4 * (ks + 4) < nkb;
        s4 n0, n1;
        u4 v0, v1;
        if (more) {            // past the end: re-read the current block (stays in LDS bounds)
          sg += dsg;
          r += dr;
          if (sg >= segs) { sg -= segs; ++r; }
        }
        load(n0, n1, v0, v1);  // unconditional: straight-line code keeps the wait partial
        const bf16x8 A = __builtin_bit_cast(bf16x8, s8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]});
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, __builtin_bit_cast(bf16x8, w0), acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, __builtin_bit_cast(bf16x8, w1), acc[1], 0, 0, 0);
        if (!more) break;
        h0 = n0; h1 = n1; w0 = v0; w1 = v1;
      }
    }
  }
  // ---- per-block slab: sum the 4 waves' D, fold the pair offset j into the taps
  __syncthreads();
  float* red = reinterpret_cast<float*>(dys);     // [4 waves][16 rows][32 taps]
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * 16 + 4 * gq + i) * 32 + 16 * tt + col] = acc[tt][i];
  __syncthreads();
  for (int o = tid; o < COUT * 25; o += 256) {
    const int c = o / 25, t = o - c * 25, ky = t / 5, kx = t - ky * 5;
    float s = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv)
      s += red[(wv * 16 + c) * 32 + ky * 6 + kx] + red[(wv * 16 + 8 + c) * 32 + ky * 6 + kx + 1];
    parts[(size_t)blockIdx.x * (COUT * 25) + o] = s;
  }
}

}  // namespace

// one resident wave of blocks (CUs x blocks per CU): the blocks walk the tiles in step,
// with no tail round of partly filled CUs
int avd_c1p8_wgrad_slabs(int N, int H) {
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, c1p8_bwd_wgrad_kernel, 256, 0) !=
            hipSuccess || per <= 0)
      per = 3;
    resident = cus * per;
  }
  return grid_cap(std::min(N * (H / TH), resident));
}
static int rc_wgrad_slabs(int N, int H) { return grid_cap(std::min(N * (H / TH), 2048)); }

int avd_c1p8_bwd_apply_wgrad(const void* y, const void* gout, const float* scale,
                             const float* shift, const float* coef, const void* x, float* parts,
                             int N, int B, int H, int W, hipStream_t st) {
  const int tps = H / TH, ntiles = N * tps;
  c1p8_bwd_wgrad_kernel<<<avd_c1p8_wgrad_slabs(N, H), 256, 0, st>>>(
      (const bf16*)x, (const bf16*)y, (const bf16*)gout, scale, shift, coef, parts, B, H, W, ntiles,
      tps);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// ============================================================================ recompute path
// The same layer without ever storing its conv output y (1.44 GB per config-2 step): every
// pass re-derives y from the 180 MB input with the pixel-pair MFMA (4 ds_read_b32 + 1 MFMA per
// 32 outputs, bit-identical bf16 values in every pass) into an LDS tile, then runs its own
// epilogue:
//   RC_STATS   BN partial (sum, sumsq) rows of the rounded values  (= conv_c1p8_kernel's)
//   RC_APPLY   BN -> ReLU -> 2x2 max-pool -> z (the next layer's input; avd_cl_bn_relu_pool)
//   RC_REDUCE  BN-backward partials (sum dz, sum dz*xhat) rows      (= avd_cl_bn_bwd_reduce)
//   RC_WGRAD   BN-backward apply + weight gradient slabs            (= avd_cl_bn_bwd_apply_wgrad)
namespace {

enum { RC_STATS = 0, RC_APPLY = 1, RC_REDUCE = 2, RC_WGRAD = 3 };

__device__ __forceinline__ void unpack8(u4 v, float (&f)[8]) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

template <int PASS>
__global__ __launch_bounds__(256) void c1p8_recompute_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coef, const bf16* __restrict__ gz, bf16* __restrict__ z,
    float* __restrict__ out, int B, int H, int W, int ntiles, int tps,
    unsigned* __restrict__ codes) {
  constexpr bool NEED_Y = PASS != RC_STATS;
  constexpr bool WG = PASS == RC_WGRAD;
  __shared__ __attribute__((aligned(16))) bf16 xs[(TH + 4) * ITW];
  // RC_APPLY keeps y rows parity-split (even pixels, then odd: a window's two columns are 56
  // pixels apart), odd rows with their two 4-channel halves swapped, at a 1856-byte row stride
  // (64 mod 128): the MFMA phase's 8-byte writes (rows 2s and 2s+1 in one 16-lane group) and the
  // window threads' 16-byte reads (which wrap to the next window row) are then bank-conflict
  // free (tools/lds_conflicts.py); the other passes keep natural rows (their tr16 reads want them)
  constexpr bool PSPLIT = PASS == RC_APPLY;
  constexpr int YRS = PSPLIT ? 928 : WMAX * COUT;
  static_assert(!PSPLIT || (YRS >= WMAX * COUT && (YRS * 2) % 128 == 64), "apply y row stride");
  __shared__ __attribute__((aligned(16))) bf16 ys[NEED_Y ? TH * YRS : 8];
  auto ypos = [&](int ox) { return PSPLIT ? (ox >> 1) + (ox & 1) * (WMAX / 2) : ox; };
  __shared__ __attribute__((aligned(16))) bf16 xc[WG ? 2 : 1][WG ? 3 : 1][WG ? TH + 4 : 1][XCW];
  __shared__ float red[WG ? 4 * 16 * 32 : 4 * 16];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h = lane >> 4, p = lane & 15, j = lane >> 5, cs = h & 1;
  const int q = p & 7, rp = p >> 3;
  const int Hp = H >> 1, Wp = W >> 1, cpr = W >> 3, mts = W >> 4;

  bf16x8 a;
  {
    const int m = lane & 15, jj = m >> 3, c = m & 7;
    __bf16 e[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int k = 8 * h + t, ky = k / 6, kx = k % 6 - jj;
      const bool ok = k < 30 && kx >= 0 && kx < 5;
      const float v = bf2f(wk[c * 32 + (ok ? ky * 5 + kx : 0)]);
      e[t] = (__bf16)(ok ? v : 0.f);
    }
    a = bf16x8{e[0], e[1], e[2], e[3], e[4], e[5], e[6], e[7]};
  }
  float bv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bv[i] = bias ? bias[4 * cs + i] : 0.f;
  int off[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) off[d] = boff(h, d) + rp * ITWD + q + 3;

  float ss[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};   // STATS
  float s1[COUT], s2[COUT];                                           // REDUCE
#pragma unroll
  for (int e = 0; e < COUT; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};      // WGRAD
  int bb[2], ba[2], bky[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    int t = 16 * tt + p;
    if (t >= 30) t = 29;   // padded taps (unused, or replaced by ones): column 13's address, a broadcast
    const int ky = t / 6, k2 = t % 6 - 2;
    bky[tt] = ky;
    bb[tt] = k2 & 1;
    ba[tt] = (k2 >= 0 ? k2 >> 1 : -1) + 1;
  }

  // WGRAD: blocks stride over all tiles (one dW slab each); the other passes: one block = one
  // sample (its tps row tiles), so the per-block setup is amortised and rows are per sample
  const int t_begin = WG ? (int)blockIdx.x : (int)blockIdx.x * tps;
  const int t_end = WG ? ntiles : t_begin + tps;
  const int t_step = WG ? (int)gridDim.x : 1;
  // input rows of a tile: <= 2 16-byte vectors per thread (W <= WMAX), register-prefetched one
  // tile ahead (issued before the current tile's MFMAs and epilogue)
  // input rows: 16 lanes per row (lane c < cpr holds pixels 8c .. 8c+7), so the 8-lane groups
  // of the 16-byte LDS stores never straddle two rows (conflict-free staging)
  int xr[2], xoff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = tid + 256 * s;
    const int r = t >> 4, c = t & 15;
    xr[s] = (r < TH + 4 && c < cpr) ? r : -(1 << 20);
    xoff[s] = (r - 2) * W + 8 * c;
  }
  // register ring of PF tiles' input rows: tile i's loads are issued PF tiles ahead, so a
  // block keeps PF x 4.5 KB in flight instead of one tile's (the pass is load-latency bound)
  constexpr int PF = 1;
  u4 xv[PF][2];
  auto load_x = [&](int tl, u4 (&dst)[2]) {
    const int n = tl / tps, ty0 = (tl - n * tps) * TH;
    const bf16* xb = x + ((size_t)n * H + ty0) * W;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool ok = (unsigned)(ty0 - 2 + xr[s]) < (unsigned)H;
      dst[s] = ldg16(ok ? (const void*)(xb + xoff[s]) : &kZeroC1);
    }
  };
#pragma unroll
  for (int d = 0; d < PF; ++d)
    if (t_begin + d * t_step < t_end) load_x(t_begin + d * t_step, xv[d]);
  auto tile_body = [&](int tile, u4 (&xvd)[2]) {
    const int n = tile / tps, ty0 = (tile - n * tps) * TH, grp = n / B;
    __syncthreads();
    // ---- input tile (natural layout, zero pads)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = tid + 256 * s;
      const int r = t >> 4, c = t & 15;
      if (r < TH + 4 && c < cpr) *reinterpret_cast<u4*>(xs + r * ITW + XOFF + 8 * c) = xvd[s];
    }
    for (int t = tid; t < (TH + 4) * 2; t += 256) {
      const int r = t >> 1, side = t & 1;
      *reinterpret_cast<u4*>(xs + r * ITW + (side ? XOFF + W : 0)) = u4{0u, 0u, 0u, 0u};
    }
    if (tile + PF * t_step < t_end) load_x(tile + PF * t_step, xvd);
    __syncthreads();
    // ---- recompute y (rounded to bf16 exactly as the stored-y path)
    const unsigned* xd = reinterpret_cast<const unsigned*>(xs);
    for (int s = wave; s < TH / 2; s += 4) {
      // statistics pass: every column tile's B fragments first (their LDS reads in flight
      // together), then the MFMAs, then the epilogues (213 vs 224 us); the other passes keep
      // one tile at a time (the unrolled registers cost the apply pass an occupancy step)
      constexpr int MTU = PASS == RC_STATS ? MTMAX : 1;
      for (int mt0 = 0; mt0 < mts; mt0 += MTU) {
      u4 bws[MTU];
#pragma unroll
      for (int u = 0; u < MTU; ++u) {
        const int mt = mt0 + u;
        if (mt >= mts) break;
        const int base = 2 * s * ITWD + 8 * mt;
        bws[u] = u4{xd[base + off[0]], xd[base + off[1]], xd[base + off[2]], xd[base + off[3]]};
      }
      f4 r4s[MTU];
#pragma unroll
      for (int u = 0; u < MTU; ++u) {
        if (mt0 + u >= mts) break;
        r4s[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, bws[u]),
                                                         f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < MTU; ++u) {
        const int mt = mt0 + u;
        if (mt >= mts) break;
        const f4 r4 = r4s[u];
        const uint32_t lo = pack_bf16x2(r4[0] + bv[0], r4[1] + bv[1]);
        const uint32_t hi = pack_bf16x2(r4[2] + bv[2], r4[3] + bv[3]);
        if constexpr (PASS == RC_STATS) {
          const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                              __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            ss[i] += v[i];
            sq[i] = fmaf(v[i], v[i], sq[i]);
          }
        } else {
          const int ox = 16 * mt + 2 * q + j;
          *reinterpret_cast<uint2*>(&ys[(2 * s + rp) * YRS + ypos(ox) * COUT + 4 * (PSPLIT ? cs ^ rp : cs)]) =
              make_uint2(lo, hi);
        }
      }
      }
    }
    if constexpr (!NEED_Y) return;
    __syncthreads();
    // ---- per-window epilogues (one thread = one 2x2 window, all 8 channels)
    float sc[COUT], sf[COUT];
#pragma unroll
    for (int e = 0; e < COUT; ++e) {
      sc[e] = scale[grp * COUT + e];
      sf[e] = shift[grp * COUT + e];
    }
    if constexpr (PASS == RC_APPLY) {
      // z = relu(bn(max / min y)) and the first argmax: BN (fma, in channel pairs) per pixel,
      // then one max3 pair per channel and an equality chain for the code nibble -- the same
      // values as max_k relu(fma(y_k)) with a strict-> argmax update (fma and relu are monotone)
      typedef __attribute__((ext_vector_type(2))) float f2;
      f2 sc2[COUT / 2], sf2[COUT / 2];
#pragma unroll
      for (int i = 0; i < COUT / 2; ++i) {
        sc2[i] = f2{sc[2 * i], sc[2 * i + 1]};
        sf2[i] = f2{sf[2 * i], sf[2 * i + 1]};
      }
      for (int w = tid; w < (TH / 2) * Wp; w += 256) {
        const int hp = w / Wp, wp = w - hp * Wp;
        u4 yr[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
          const u4 v = *reinterpret_cast<const u4*>(&ys[(2 * hp + (k >> 1)) * YRS + (wp + (k & 1) * (WMAX / 2)) * COUT]);
          yr[k] = k >> 1 ? u4{v.z, v.w, v.x, v.y} : v;     // odd rows: halves swapped
        }
        unsigned o[4], code = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f2 r[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const unsigned d = i == 0 ? yr[k].x : i == 1 ? yr[k].y : i == 2 ? yr[k].z : yr[k].w;
            const f2 yy = f2{__uint_as_float(d << 16), __uint_as_float(d & 0xffff0000u)};
            r[k] = __builtin_elementwise_fma(yy, sc2[i], sf2[i]);
          }
          float best[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            best[e] = fmaxf(fmaxf(fmaxf(r[0][e], r[1][e]), fmaxf(r[2][e], r[3][e])), 0.f);
            unsigned nib = 4u;
            nib = r[2][e] == best[e] ? 3u : nib;
            nib = r[1][e] == best[e] ? 2u : nib;
            nib = r[0][e] == best[e] ? 1u : nib;
            nib = best[e] > 0.f ? nib : 0u;
            code |= nib << (4 * (2 * i + e));
          }
          o[i] = pack_bf16x2(best[0], best[1]);
        }
        const size_t pw = ((size_t)n * Hp + (ty0 >> 1) + hp) * Wp + wp;
        *reinterpret_cast<u4*>(z + pw * COUT) = u4{o[0], o[1], o[2], o[3]};
        if (codes) codes[pw] = code;
      }
      return;
    }
    for (int w = tid; w < (TH / 2) * Wp; w += 256) {
      const int hp = w / Wp, wp = w - hp * Wp;
      float yv[4][COUT];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        unpack8(*reinterpret_cast<const u4*>(
                    &ys[((2 * hp + (k >> 1)) * WMAX + 2 * wp + (k & 1)) * COUT]), yv[k]);
      float best[COUT];
      int arg[COUT];
#pragma unroll
      for (int e = 0; e < COUT; ++e) {
        best[e] = fmaxf(fmaf(yv[0][e], sc[e], sf[e]), 0.f);
        arg[e] = 0;
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          const float r = fmaxf(fmaf(yv[k][e], sc[e], sf[e]), 0.f);
          if (r > best[e]) { best[e] = r; arg[e] = k; }
        }
      }
      const size_t pw = ((size_t)n * Hp + (ty0 >> 1) + hp) * Wp + wp;
      if constexpr (PASS == RC_APPLY) {
        unsigned o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = pack_bf16x2(best[2 * i], best[2 * i + 1]);
        *reinterpret_cast<u4*>(z + pw * COUT) = u4{o[0], o[1], o[2], o[3]};
        if (codes) {   // routing code of the window: nibble e = 1 + first argmax, 0 = no route
          unsigned code = 0u;
#pragma unroll
          for (int e = 0; e < COUT; ++e) code |= (best[e] > 0.f ? (unsigned)(arg[e] + 1) : 0u) << (4 * e);
          codes[pw] = code;
        }
      } else {
        float gg[COUT];
        unpack8(*reinterpret_cast<const u4*>(gz + pw * COUT), gg);
        if constexpr (PASS == RC_REDUCE) {
#pragma unroll
          for (int e = 0; e < COUT; ++e) {
            const int ag = arg[e];
            const float ya = ag == 0 ? yv[0][e] : ag == 1 ? yv[1][e] : ag == 2 ? yv[2][e] : yv[3][e];
            const float dz = best[e] > 0.f ? gg[e] : 0.f;
            s1[e] += dz;
            s2[e] += dz * (ya - mean[grp * COUT + e]) * invstd[grp * COUT + e];
          }
        } else {   // RC_WGRAD: dy in place of the window's y
          unsigned ow[4][4];
#pragma unroll
          for (int e = 0; e < COUT; ++e) {
            const int gc = (grp * COUT + e) * 3;
            const float k1 = coef[gc], kx = coef[gc + 1], k0 = coef[gc + 2];
            const float dz = best[e] > 0.f ? gg[e] : 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float d = fmaf(k1, arg[e] == k ? dz : 0.f, fmaf(kx, yv[k][e], k0));
              const uint32_t hb = __builtin_bit_cast(uint16_t, (__bf16)d);
              if (e & 1) ow[k][e >> 1] |= hb << 16;
              else ow[k][e >> 1] = hb;
            }
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
            *reinterpret_cast<u4*>(&ys[((2 * hp + (k >> 1)) * WMAX + 2 * wp + (k & 1)) * COUT]) =
                u4{ow[k][0], ow[k][1], ow[k][2], ow[k][3]};
        }
      }
    }
    if constexpr (WG) {
      // parity/shift copies of the input rows, from the natural tile:
      // xc[b][a][r][P] = x[2(P+a-1)+b] = xs[r][XOFF + 2(P+a-1) + b]  (pads are zero)
      for (int t = tid; t < (TH + 4) * 3 * (Wp >> 1); t += 256) {
        const int r = t / (3 * (Wp >> 1)), rem = t - r * 3 * (Wp >> 1);
        const int aa = rem / (Wp >> 1), P = 2 * (rem - aa * (Wp >> 1));
        const unsigned* src = reinterpret_cast<const unsigned*>(xs + r * ITW + XOFF) + (P + aa - 1);
        const unsigned d0 = src[0], d1 = src[1];
        *reinterpret_cast<unsigned*>(&xc[0][aa][r][P]) = (d0 & 0xffffu) | (d1 << 16);
        *reinterpret_cast<unsigned*>(&xc[1][aa][r][P]) = (d0 >> 16) | (d1 & 0xffff0000u);
      }
      __syncthreads();
      const int segs = W >> 4, nkb = TH * segs;
      for (int ks = wave; 4 * ks < nkb; ks += 4) {
        const int kb = 4 * ks + h;
        const int r = kb / segs, P0 = 8 * (kb - r * segs);
        const int qq = p >> 2, pp = p & 3;
        s4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)&ys[(r * WMAX + 2 * (P0 + qq)) * COUT + 4 * pp]);
        s4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)&ys[(r * WMAX + 2 * (P0 + 4 + qq)) * COUT + 4 * pp]);
        typedef __attribute__((ext_vector_type(8))) short s8;
        const bf16x8 A = __builtin_bit_cast(bf16x8, s8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]});
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const u4 bw = *reinterpret_cast<const u4*>(&xc[bb[tt]][ba[tt]][r + bky[tt]][P0]);
          acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, __builtin_bit_cast(bf16x8, bw),
                                                           acc[tt], 0, 0, 0);
        }
      }
    }
  };
  for (int base = t_begin; base < t_end; base += PF * t_step) {
#pragma unroll
    for (int d = 0; d < PF; ++d)
      if (base + d * t_step < t_end) tile_body(base + d * t_step, xv[d]);
  }

  if constexpr (PASS == RC_STATS || PASS == RC_REDUCE) {
    // per-wave partial rows [C][G][R][2], R = B * 4 (one block = one sample)
    const int n = blockIdx.x, grp = n / B;
    const size_t R = (size_t)B * 4;
    const size_t row = (size_t)(n - grp * B) * 4 + wave;
    const int G = ntiles / (B * tps);
    if constexpr (PASS == RC_STATS) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int m = 1; m <= 32; m <<= 1) {
          if (m == 16) continue;
          ss[i] += __shfl_xor(ss[i], m, 64);
          sq[i] += __shfl_xor(sq[i], m, 64);
        }
      if ((lane & 47) == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = 4 * cs + i;
          out[(((size_t)co * G + grp) * R + row) * 2] = ss[i];
          out[(((size_t)co * G + grp) * R + row) * 2 + 1] = sq[i];
        }
    } else {
#pragma unroll
      for (int e = 0; e < COUT; ++e) {
        s1[e] = wave_sum(s1[e]);
        s2[e] = wave_sum(s2[e]);
      }
      if (lane == 0)
#pragma unroll
        for (int e = 0; e < COUT; ++e) {
          out[(((size_t)e * G + grp) * R + row) * 2] = s1[e];
          out[(((size_t)e * G + grp) * R + row) * 2 + 1] = s2[e];
        }
    }
  }
  if constexpr (WG) {
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(wave * 16 + 4 * h + i) * 32 + 16 * tt + p] = acc[tt][i];
    __syncthreads();
    for (int o = tid; o < COUT * 25; o += 256) {
      const int c = o / 25, t = o - c * 25, ky = t / 5, kx = t - ky * 5;
      float s = 0.f;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv)
        s += red[(wv * 16 + c) * 32 + ky * 6 + kx] + red[(wv * 16 + 8 + c) * 32 + ky * 6 + kx + 1];
      out[(size_t)blockIdx.x * (COUT * 25) + o] = s;
    }
  }
}


// ---------------------------------------------------------------------------- moments pass
// Backward of the layer in ONE pass that reads only the input x and the pooled gradient gz
// (no stored y, no dy): dy = k1 dz + kx y + k0 is linear in (dz, y, 1) and y = w . x25 + b, so
//   dW[c][t] = sum_g k1 M[g][c][t] + kx (sum_t' w[c][t'] G[g][t'][t] + b[c] S[g][t]) + k0 S[g][t]
// with, per BN group g, M = sum dz x25 (dz = the routed pooled gradient), G = sum x25 x25^T (the
// patch Gram matrix) and S = sum x25 -- none of which needs the BN-backward coefficients, so the
// same pass also forms the BN-backward sums (sum dz, sum dz xhat) those coefficients come from
// (avd_bn_bwd_finalize) and a tiny combine kernel finishes dW.  Per tile: x rows staged twice
// (natural rows for the y recompute, parity/shift copies for the B operand), y recomputed by
// the pixel-pair MFMA into LDS (bit-identical bf16 values), one thread per pooling window forms
// dz in place of y, then per k-block of pixel pairs: D += dZ X (2 MFMAs, the wgrad kernel's
// operands) and the Gram tiles X^T X (3 MFMAs; the B fragment doubles as the A fragment, and
// pair column 30 reads ones so its Gram column is S).  Blocks own contiguous tile ranges of
// one BN group; outputs per block row r of group g:
//   out[((c * G + g) * R + r) * 2 + {0, 1}]                 BN sums of channel c
//   out[C * G * R * 2 + (r * G + g) * MOM5 + ...]             M [8][25] | G [25][25] | S [25]
constexpr int MOM5 = COUT * 25 + 25 * 25 + 25;

typedef __attribute__((ext_vector_type(2))) float f2;

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}

__global__ __launch_bounds__(256, 2) void c1p8_moments_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const bf16* __restrict__ gz, float* __restrict__ out, int B, int G, int R, int H, int W,
    int tps) {
  __shared__ __attribute__((aligned(16))) bf16 xs[(TH + 4) * ITW];
  __shared__ __attribute__((aligned(16))) bf16 xc[2 * XB_CB];
  __shared__ __attribute__((aligned(16))) bf16 dys[TH * WMAX * COUT];
  __shared__ __attribute__((aligned(16))) bf16 gzs[(TH / 2) * (WMAX / 2) * COUT];
  __shared__ float bsum[4][2 * COUT];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int gq = lane >> 4, col = lane & 15;
  const int Hp = H >> 1, Wp = W >> 1, cpr = W >> 3, segs = W >> 4, mts = W >> 4;
  const int grp = (int)blockIdx.x / R, rr = (int)blockIdx.x - grp * R;
  const long long tpg = (long long)B * tps;                 // tiles of one BN group
  const int t_begin = (int)(grp * tpg + (tpg * rr) / R), t_end = (int)(grp * tpg + (tpg * (rr + 1)) / R);

  // y recompute: A = weights (rows (j, c)), B = 4 dwords of the natural rows (conv_c1p8_kernel);
  // D lane = pixel (pair q + 8 rp, j) of a 2-row strip, channels 4 cs .. 4 cs + 3
  bf16x8 aw;
  {
    const int m = lane & 15, jj = m >> 3, c = m & 7;
    __bf16 e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 8 * gq + q, ky = k / 6, kx = k % 6 - jj;
      const bool ok = k < 30 && kx >= 0 && kx < 5;
      const float v = bf2f(wk[c * 32 + (ok ? ky * 5 + kx : 0)]);
      e[q] = (__bf16)(ok ? v : 0.f);
    }
    aw = bf16x8{e[0], e[1], e[2], e[3], e[4], e[5], e[6], e[7]};
  }
  const int cs = gq & 1, jy = lane >> 5, qy = col & 7, rp = col >> 3;
  float bv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bv[i] = bias ? bias[4 * cs + i] : 0.f;
  int yo[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) yo[d] = boff(gq, d) + rp * ITWD + qy + 3;
  // this block's group: BN coefficients; per-thread sums over its pooling windows (all 8
  // channels): sum dz and sum dz * y (xhat applied once at the end)
  float sc[COUT], sf[COUT], s1[COUT], s2[COUT];
#pragma unroll
  for (int e = 0; e < COUT; ++e) {
    sc[e] = scale[grp * COUT + e];
    sf[e] = shift[grp * COUT + e];
    s1[e] = 0.f; s2[e] = 0.f;
  }
  // wgrad / Gram operands (c1p8_bwd_wgrad_kernel's): tap tiles tt = 0, 1
  int bb[2], ba[2], bky[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    int t = 16 * tt + col;
    if (t >= 30) t = 29;   // padded taps (unused, or replaced by ones): column 13's address, a broadcast
    const int ky = t / 6, k2 = t % 6 - 2;
    bky[tt] = ky;
    bb[tt] = k2 & 1;
    ba[tt] = (k2 >= 0 ? k2 >> 1 : -1) + 1;
  }
  const bool ones = col == 14;                               // pair column 30: constant 1
  // fp32 MFMA accumulators over the block's tiles (8 waves of blocks: ~12 tiles each at bench
  // size; moments within 1e-7 of float64 there)
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  f4 ga[3] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};

  // global loads one tile ahead: <= 2 input-row vectors and <= 2 pooled-gradient vectors
  const int nxt = (TH + 4) * cpr, nwin = (TH / 2) * Wp;
  int xr[2], xoff[2], goff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = tid + 256 * s;
    const int r = t / cpr, c = t - r * cpr;
    xr[s] = t < nxt ? r : -(1 << 20);
    xoff[s] = (r - 2) * W + 8 * c;
    goff[s] = min(t, nwin - 1) * COUT;        // window (hp, wp) of the tile = row-major index
  }
  u4 xv[2], gv[2];
  auto load = [&](int tile) {
    const int n = tile / tps, ty0 = (tile - n * tps) * TH;
    const bf16* xb = x + ((size_t)n * H + ty0) * W;
    const bf16* gb = gz + ((size_t)n * Hp + (ty0 >> 1)) * Wp * COUT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool ok = (unsigned)(ty0 - 2 + xr[s]) < (unsigned)H;
      xv[s] = ldg16(ok ? (const void*)(xb + xoff[s]) : &kZeroC1);
      gv[s] = ldg16(gb + goff[s]);
    }
  };
  if (t_begin < t_end) load(t_begin);
  for (int tile = t_begin; tile < t_end; ++tile) {
    __syncthreads();                     // the previous tile's MFMAs are done with LDS
    // ---- natural rows (y recompute), parity/shift copies (B operand), pooled gradients
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = tid + 256 * s;
      if (t < nwin) *reinterpret_cast<u4*>(&gzs[t * COUT]) = gv[s];
      if (t >= nxt) continue;
      const int r = t / cpr, c = t - r * cpr;
      *reinterpret_cast<u4*>(xs + r * ITW + XOFF + 8 * c) = xv[s];
      const unsigned wv[4] = {xv[s].x, xv[s].y, xv[s].z, xv[s].w};
      const unsigned e0 = (wv[0] & 0xffffu) | (wv[1] << 16), ee1 = (wv[2] & 0xffffu) | (wv[3] << 16);
      const unsigned o0 = (wv[0] >> 16) | (wv[1] & 0xffff0000u), o1 = (wv[2] >> 16) | (wv[3] & 0xffff0000u);
      const unsigned ev[2] = {e0, ee1}, od[2] = {o0, o1};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const unsigned lo = b ? od[0] : ev[0], hi = b ? od[1] : ev[1];
        *reinterpret_cast<uint2*>(&xc[xbo(b, 1, r, 4 * c)]) = make_uint2(lo, hi);
        bf16* d0 = &xc[xbo(b, 0, r, 4 * c + 1)];
        st16(d0, (bf16)(lo & 0xffffu));
        *reinterpret_cast<unsigned*>(d0 + 1) = (lo >> 16) | (hi << 16);
        st16(d0 + 3, (bf16)(hi >> 16));
        bf16* d2 = &xc[xbo(b, 2, r, 4 * c)];
        if (c > 0) st16(d2 - 1, (bf16)(lo & 0xffffu));
        *reinterpret_cast<unsigned*>(d2) = (lo >> 16) | (hi << 16);
        st16(d2 + 2, (bf16)(hi >> 16));
      }
    }
    if (tid < (TH + 4) * 2) {
      const int r = tid >> 1, b = tid & 1;
      xc[xbo(b, 0, r, 0)] = bf16(0);
      xc[xbo(b, 2, r, Wp - 1)] = bf16(0);
      *reinterpret_cast<u4*>(xs + r * ITW + (b ? XOFF + W : 0)) = u4{0u, 0u, 0u, 0u};
    }
    if (tile + 1 < t_end) load(tile + 1);   // in flight under this tile's work
    __syncthreads();
    // ---- y (bf16, as every other pass rounds it) into dys at the wgrad A-operand positions:
    // per 2-row strip every column tile's operands first, then the MFMAs, then the stores
    {
      const unsigned* xd = reinterpret_cast<const unsigned*>(xs);
      for (int s = wave; s < TH / 2; s += 4) {
        const int ry = 2 * s + rp;
        u4 bw[MTMAX];
#pragma unroll
        for (int mt = 0; mt < MTMAX; ++mt) {
          if (mt >= mts) break;
          const int base = 2 * s * ITWD + 8 * mt;
          bw[mt] = u4{xd[base + yo[0]], xd[base + yo[1]], xd[base + yo[2]], xd[base + yo[3]]};
        }
#pragma unroll
        for (int mt = 0; mt < MTMAX; ++mt) {
          if (mt >= mts) break;
          const f4 r4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, __builtin_bit_cast(bf16x8, bw[mt]),
                                                                f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          const int cx = 16 * mt + 2 * qy + jy;
          *reinterpret_cast<uint2*>(&dys[(ry * WMAX + dys_px(ry, cx, segs)) * COUT + 4 * cs]) =
              make_uint2(pack_bf16x2(r4[0] + bv[0], r4[1] + bv[1]), pack_bf16x2(r4[2] + bv[2], r4[3] + bv[3]));
        }
      }
    }
    __syncthreads();
    // ---- one thread per pooling window: first-max routing, BN sums, dz in place of y
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int w = tid + 256 * s;
      if (w >= nwin) continue;
      const int hp = w / Wp, wp = w - hp * Wp;
      int po[4];
      float yv[4][COUT];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ry = 2 * hp + (k >> 1), cx = 2 * wp + (k & 1);
        po[k] = (ry * WMAX + dys_px(ry, cx, segs)) * COUT;
        const u4 v = *reinterpret_cast<const u4*>(&dys[po[k]]);
        const unsigned wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          yv[k][2 * i] = __uint_as_float(wv[i] << 16);
          yv[k][2 * i + 1] = __uint_as_float(wv[i] & 0xffff0000u);
        }
      }
      const u4 gvw = *reinterpret_cast<const u4*>(&gzs[w * COUT]);
      float gg[COUT];
      {
        const unsigned wv[4] = {gvw.x, gvw.y, gvw.z, gvw.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gg[2 * i] = __uint_as_float(wv[i] << 16);
          gg[2 * i + 1] = __uint_as_float(wv[i] & 0xffff0000u);
        }
      }
      uint32_t ow[4][4];
      // BN values of the window, two channels per packed FMA; the first max of relu(v) routes
      // the gradient only when it is > 0, where it is the first max of v itself (no relu needed)
      float bnv[4][COUT];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < COUT; e += 2) {
          const f2 v = __builtin_elementwise_fma(f2{yv[k][e], yv[k][e + 1]}, f2{sc[e], sc[e + 1]},
                                                 f2{sf[e], sf[e + 1]});
          bnv[k][e] = v[0];
          bnv[k][e + 1] = v[1];
        }
#pragma unroll
      for (int e = 0; e < COUT; ++e) {
        const float rv[4] = {bnv[0][e], bnv[1][e], bnv[2][e], bnv[3][e]};
        const float m = fmaxf(fmaxf(rv[0], rv[1]), fmaxf(rv[2], rv[3]));
        const bool e0 = rv[0] == m, e1 = !e0 && rv[1] == m, e2 = !e0 && !e1 && rv[2] == m;
        const float dz = m > 0.f ? gg[e] : 0.f;
        const float ya = e0 ? yv[0][e] : e1 ? yv[1][e] : e2 ? yv[2][e] : yv[3][e];
        s1[e] += dz;
        s2[e] = fmaf(dz, ya, s2[e]);
        // dz (exact in bf16: a pooled gradient or zero) at the first max, 0 elsewhere
        const uint32_t db = __float_as_uint(dz) >> 16;
        const uint32_t d[4] = {e0 ? db : 0u, e1 ? db : 0u, e2 ? db : 0u, (!e0 && !e1 && !e2) ? db : 0u};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (e & 1) ow[k][e >> 1] |= d[k] << 16;
          else ow[k][e >> 1] = d[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        *reinterpret_cast<u4*>(&dys[po[k]]) = u4{ow[k][0], ow[k][1], ow[k][2], ow[k][3]};
    }
    __syncthreads();
    // ---- k-blocks of pixel pairs: D += dZ X (tap tiles 0, 1) and the Gram tiles (0,0) (0,1) (1,1)
    const int nkb = TH * segs;
    if (4 * wave < nkb) {
      typedef __attribute__((ext_vector_type(8))) short s8;
      const int q = col >> 2, pp = col & 3;
      const int kb0 = 4 * wave + gq;
      int r = kb0 / segs, sg = kb0 - r * segs;
      const int hsw = (kb0 & 1) << 3;
      const int aoff0 = ((2 * q) ^ hsw) * COUT + 4 * pp, aoff1 = ((8 + 2 * q) ^ hsw) * COUT + 4 * pp;
      const int boff0 = xbo(bb[0], ba[0], bky[0], 0), boff1 = xbo(bb[1], ba[1], bky[1], 0);
      const int dr = 16 / segs, dsg = 16 - dr * segs;
      const u4 one4 = u4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
      s4 h0, h1;
      u4 w0, w1;
      auto ld = [&](s4& a0, s4& a1, u4& c0, u4& c1) {
        const int P0 = 8 * sg, ab = (r * WMAX + 2 * P0) * COUT, bs = r * XB_RS + P0;
        a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&dys[ab + aoff0]);
        a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&dys[ab + aoff1]);
        c0 = *reinterpret_cast<const u4*>(&xc[bs + boff0]);
        c1 = *reinterpret_cast<const u4*>(&xc[bs + boff1]);
      };
      // two k-blocks of operand reads ahead of the MFMAs (past the end: re-read the last
      // block, in LDS bounds)
      auto adv = [&](bool go) {
        if (go) {
          sg += dsg;
          r += dr;
          if (sg >= segs) { sg -= segs; ++r; }
        }
      };
      ld(h0, h1, w0, w1);
      s4 n0, n1;
      u4 v0, v1;
      adv(4 * (wave + 4) < nkb);
      ld(n0, n1, v0, v1);
      for (int ks = wave;; ks += 4) {
        const bool more = 4 * (ks + 4) < nkb;
        s4 m0, m1;
        u4 x0v, x1v;
        adv(4 * (ks + 8) < nkb);
        ld(m0, m1, x0v, x1v);
        const bf16x8 A = __builtin_bit_cast(bf16x8, s8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]});
        const bf16x8 X0 = __builtin_bit_cast(bf16x8, w0);
        const bf16x8 X1 = __builtin_bit_cast(bf16x8, ones ? one4 : w1);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, X0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, X1, acc[1], 0, 0, 0);
        {
          ga[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X0, X0, ga[0], 0, 0, 0);
          ga[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X0, X1, ga[1], 0, 0, 0);
          ga[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X1, X1, ga[2], 0, 0, 0);
        }
        if (!more) break;
        h0 = n0; h1 = n1; w0 = v0; w1 = v1;
        n0 = m0; n1 = m1; v0 = x0v; v1 = x1v;
      }
    }
  }
  // ---- block outputs: BN sums (one row), then M / Gram / S folded from pairs to taps
#pragma unroll
  for (int e = 0; e < COUT; ++e) {
    const int gc = grp * COUT + e;
    const float a1 = wave_sum(s1[e]), a2 = wave_sum(s2[e]);
    s1[e] = a1;
    s2[e] = (a2 - mean[gc] * a1) * invstd[gc];       // sum dz * xhat
  }
  if (lane == 0)
#pragma unroll
    for (int e = 0; e < COUT; ++e) { bsum[wave][e] = s1[e]; bsum[wave][COUT + e] = s2[e]; }
  __syncthreads();                        // also: every wave is done with dys / xc
  float* red = reinterpret_cast<float*>(dys);        // [4][16][32]  D
  float* g6 = red + 4 * 16 * 32;                     // [4][32][32]  Gram tiles (upper blocks)
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * 16 + 4 * gq + i) * 32 + 16 * tt + col] = acc[tt][i];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int ti = b == 2 ? 1 : 0, tj = b == 0 ? 0 : 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      g6[(wave * 32 + 16 * ti + 4 * gq + i) * 32 + 16 * tj + col] = ga[b][i];
  }
  __syncthreads();
  if (tid < 2 * COUT) {
    const int e = tid % COUT, k = tid / COUT;
    const float v = bsum[0][tid] + bsum[1][tid] + bsum[2][tid] + bsum[3][tid];
    out[(((size_t)e * G + grp) * R + rr) * 2 + k] = v;
  }
  float* o = out + (size_t)COUT * G * R * 2 + ((size_t)rr * G + grp) * MOM5;
  auto g6v = [&](int t1, int t2) {        // the lower block (1,0) is the transpose of (0,1)
    if (t1 >= 16 && t2 < 16) { const int tmp = t1; t1 = t2; t2 = tmp; }
    float v = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) v += g6[(wv * 32 + t1) * 32 + t2];
    return v;
  };
  for (int e = tid; e < MOM5; e += 256) {
    float v;
    if (e < COUT * 25) {
      const int c = e / 25, t = e - c * 25, ky = t / 5, kx = t - ky * 5;
      v = 0.f;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv)
        v += red[(wv * 16 + c) * 32 + ky * 6 + kx] + red[(wv * 16 + 8 + c) * 32 + ky * 6 + kx + 1];
    } else if (e < COUT * 25 + 625) {
      const int a = (e - COUT * 25) / 25, b = (e - COUT * 25) % 25;
      const int pa = (a / 5) * 6 + a % 5, pb = (b / 5) * 6 + b % 5;
      v = g6v(pa, pb) + g6v(pa + 1, pb + 1);      // even pixel of the pair, then the odd one
    } else {
      const int a = e - COUT * 25 - 625, pa = (a / 5) * 6 + a % 5;
      v = g6v(pa, 30) + g6v(pa + 1, 30);
    }
    o[e] = v;
  }
}

// dW [8][25] from the row-summed moments m [G][MOM5] and the BN-backward coefficients
__global__ void c1p8_combine_kernel(const float* __restrict__ m, const float* __restrict__ coef,
                                    const bf16* __restrict__ wk, const float* __restrict__ bias,
                                    float* __restrict__ dw, int G) {
  // float64: the kx and k0 terms are large and cancel (dy is centred by the BN backward), so
  // they are formed and summed in double (fp32 here cost ~1e-3 relative in dW at bench size)
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= COUT * 25) return;
  const int c = e / 25, t = e - c * 25;
  double wr[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) wr[k] = (double)bf2f(wk[c * 32 + k]);
  const double b = bias ? (double)bias[c] : 0.0;
  double acc = 0.0;
  for (int g = 0; g < G; ++g) {
    const float* mg = m + (size_t)g * MOM5;
    const float* gram = mg + COUT * 25;
    const double sx = gram[625 + t];
    double sy = b * sx;
#pragma unroll
    for (int k = 0; k < 25; ++k) sy = fma(wr[k], (double)gram[k * 25 + t], sy);
    const float* k3 = coef + ((size_t)g * COUT + c) * 3;
    acc += (double)k3[0] * mg[e] + (double)k3[1] * sy + (double)k3[2] * sx;
  }
  dw[e] = (float)acc;
}

// ---------------------------------------------------------------------------- routed backward
// The training backward of the layer from the forward's routing codes instead of a recomputed y.
// The forward apply pass (RC_APPLY with codes) already decides, per pooling window and channel,
// where the pooled gradient goes: codes[n][hp][wp] nibble e = 1 + the first argmax of
// relu(bn(y)) when that max is > 0, else 0 (bwd_apply_cl_kernel's routing).  So this pass needs
// neither y nor the BN coefficients: per tile it places dz = gz at the coded pixel (zero
// elsewhere), then per k-block of pixel pairs D += dZ X and the Gram tiles X^T X (the moments
// kernel's 5 MFMAs; pair column 30 reads ones, so D's column 30 is sum dz and the Gram's is S).
// The BN-backward sum dz * y at the routed pixels is not accumulated at all: y = w . x25 + b, so
// sum dz y = w . M + b sum dz, formed in float64 by the combine (c1p8_codes_combine_kernel)
// with the exact (unrounded) conv output.  Per block row r of group g, MOMC floats:
//   M [8][25] | Gram [25][25] | S [25] | sum dz [8]
constexpr int MOMC = COUT * 25 + 25 * 25 + 25 + COUT;


// MM (what the pass accumulates): 0 = M, sum dz, Gram and S (the routed backward, MOMC floats
// per row); 1 = Gram and S only (no pooled gradient: the FORWARD statistics pass -- y = w . x25 +
// b, so sum y = w . S + n b and sum y^2 = w^T Gram w + 2 b w . S + n b^2 follow from it exactly,
// GRAMC floats per row); 2 = M and sum dz only (the backward when the forward's Gram is kept;
// MOMC floats, the Gram / S slots zero).
constexpr int GRAMC = 25 * 25 + 25;

template <int MM>
__global__ __launch_bounds__(256, 3) void c1p8_moments_codes_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ gz, const unsigned* __restrict__ codes,
    float* __restrict__ out, int B, int G, int R, int H, int W, int tps) {
  __shared__ __attribute__((aligned(16))) bf16 xc[2 * XB_CB];
  // the Gram pass (MM 1) has no dz map: its LDS is the input copies alone (20 KB: 7 blocks per
  // CU instead of 3), which also hold its Gram-tile reduction at the end
  __shared__ __attribute__((aligned(16))) bf16 dys[MM == 1 ? 8 : TH * WMAX * COUT];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int gq = lane >> 4, col = lane & 15;
  const int Hp = H >> 1, Wp = W >> 1, cpr = W >> 3, segs = W >> 4;
  const int grp = (int)blockIdx.x / R, rr = (int)blockIdx.x - grp * R;
  const long long tpg = (long long)B * tps;                 // tiles of one BN group
  const int t_begin = (int)(grp * tpg + (tpg * rr) / R), t_end = (int)(grp * tpg + (tpg * (rr + 1)) / R);
  int bb[2], ba[2], bky[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    int t = 16 * tt + col;
    if (t >= 30) t = 29;   // padded taps (unused, or replaced by ones): column 13's address, a broadcast
    const int ky = t / 6, k2 = t % 6 - 2;
    bky[tt] = ky;
    bb[tt] = k2 & 1;
    ba[tt] = (k2 >= 0 ? k2 >> 1 : -1) + 1;
  }
  const bool ones = col == 14;                               // pair column 30: constant 1
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  f4 ga[3] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};

  // global loads one tile ahead: <= 2 input-row vectors, and the pooled gradients + codes of
  // this thread's <= 2 windows
  // input rows: one row per 16-lane DPP row (lane c < cpr holds pixels 8c .. 8c+7), so the
  // parity/shift copies take a neighbour's edge pair by DPP instead of sub-dword LDS stores
  const int nwin = (TH / 2) * Wp;
  int xr[2], xoff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = tid + 256 * s;
    const int r = t >> 4, c = t & 15;
    xr[s] = (r < TH + 4 && c < cpr) ? r : -(1 << 20);
    xoff[s] = (r - 2) * W + 8 * c;
  }
  u4 xv[2], gv[2];
  unsigned cv[2];
  auto load = [&](int tile) {
    const int n = tile / tps, ty0 = (tile - n * tps) * TH;
    const bf16* xb = x + ((size_t)n * H + ty0) * W;
    const size_t w0 = ((size_t)n * Hp + (ty0 >> 1)) * Wp;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool ok = (unsigned)(ty0 - 2 + xr[s]) < (unsigned)H;
      xv[s] = ldg16(ok ? (const void*)(xb + xoff[s]) : &kZeroC1);
      if constexpr (MM != 1) {
        const int w = min(tid + 256 * s, nwin - 1);
        gv[s] = ldg16(gz + (w0 + w) * COUT);
        cv[s] = codes[w0 + w];
      }
    }
  };
  if (t_begin < t_end) load(t_begin);
  for (int tile = t_begin; tile < t_end; ++tile) {
    __syncthreads();                     // the previous tile's MFMAs are done with LDS
    // ---- parity/shift copies of the input rows (B operand): xc[b][a][r][P] = x[2(P+a-1)+b],
    // three aligned 8-byte stores per parity; the pairs across a thread's edges come from its
    // row neighbours by DPP (row_shr / row_shl 1; lanes past the row end hold zeros = the pads)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = tid + 256 * s;
      const int r = t >> 4, c = t & 15;
      const unsigned wv[4] = {xv[s].x, xv[s].y, xv[s].z, xv[s].w};
      const unsigned ev[2] = {(wv[0] & 0xffffu) | (wv[1] << 16), (wv[2] & 0xffffu) | (wv[3] << 16)};
      const unsigned od[2] = {(wv[0] >> 16) | (wv[1] & 0xffff0000u), (wv[2] >> 16) | (wv[3] & 0xffff0000u)};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const unsigned lo = b ? od[0] : ev[0], hi = b ? od[1] : ev[1];
        const unsigned prev_hi = (unsigned)dpp_i<0x111>((int)hi);   // lane c-1 (0 at c = 0)
        const unsigned next_lo = (unsigned)dpp_i<0x101>((int)lo);   // lane c+1
        if (r < TH + 4 && c < cpr) {
          *reinterpret_cast<uint2*>(&xc[xbo(b, 0, r, 4 * c)]) =
              make_uint2((prev_hi >> 16) | (lo << 16), (lo >> 16) | (hi << 16));
          *reinterpret_cast<uint2*>(&xc[xbo(b, 1, r, 4 * c)]) = make_uint2(lo, hi);
          *reinterpret_cast<uint2*>(&xc[xbo(b, 2, r, 4 * c)]) =
              make_uint2((lo >> 16) | (hi << 16), (hi >> 16) | (next_lo << 16));
        }
      }
    }
    // ---- dz at the coded pixel of every window (4 pixels x 8 channels per window thread)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int w = tid + 256 * s;
      if (MM == 1 || w >= nwin) continue;
      const int hp = w / Wp, wp = w - hp * Wp;
      const unsigned gw[4] = {gv[s].x, gv[s].y, gv[s].z, gv[s].w}, code = cv[s];
      unsigned ow[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned nl = (code >> (8 * i)) & 0xFu, nh = (code >> (8 * i + 4)) & 0xFu;
        const unsigned glo = gw[i] & 0xffffu, ghi = gw[i] & 0xffff0000u;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          ow[k][i] = (nl == (unsigned)(k + 1) ? glo : 0u) | (nh == (unsigned)(k + 1) ? ghi : 0u);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ry = 2 * hp + (k >> 1), cx = 2 * wp + (k & 1);
        *reinterpret_cast<u4*>(&dys[(ry * WMAX + dys_px(ry, cx, segs)) * COUT]) =
            u4{ow[k][0], ow[k][1], ow[k][2], ow[k][3]};
      }
    }
    if (tile + 1 < t_end) load(tile + 1);   // in flight under this tile's MFMAs
    __syncthreads();
    // ---- k-blocks of pixel pairs: D += dZ X (tap tiles 0, 1) and the Gram tiles (0,0) (0,1) (1,1)
    const int nkb = TH * segs;
    if (4 * wave < nkb) {
      typedef __attribute__((ext_vector_type(8))) short s8;
      const int q = col >> 2, pp = col & 3;
      const int kb0 = 4 * wave + gq;
      int r = kb0 / segs, sg = kb0 - r * segs;
      const int hsw = (kb0 & 1) << 3;
      const int aoff0 = ((2 * q) ^ hsw) * COUT + 4 * pp, aoff1 = ((8 + 2 * q) ^ hsw) * COUT + 4 * pp;
      const int boff0 = xbo(bb[0], ba[0], bky[0], 0), boff1 = xbo(bb[1], ba[1], bky[1], 0);
      const int dr = 16 / segs, dsg = 16 - dr * segs;
      const u4 one4 = u4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
      s4 h0, h1;
      u4 w0, w1;
      auto ld = [&](s4& a0, s4& a1, u4& c0, u4& c1) {
        const int P0 = 8 * sg, ab = (r * WMAX + 2 * P0) * COUT, bs = r * XB_RS + P0;
        if constexpr (MM != 1) {
          a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&dys[ab + aoff0]);
          a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&dys[ab + aoff1]);
        } else {
          a0 = s4{0, 0, 0, 0};
          a1 = s4{0, 0, 0, 0};
        }
        c0 = *reinterpret_cast<const u4*>(&xc[bs + boff0]);
        c1 = *reinterpret_cast<const u4*>(&xc[bs + boff1]);
      };
      auto adv = [&](bool go) {
        if (go) {
          sg += dsg;
          r += dr;
          if (sg >= segs) { sg -= segs; ++r; }
        }
      };
      ld(h0, h1, w0, w1);
      s4 n0, n1;
      u4 v0, v1;
      adv(4 * (wave + 4) < nkb);
      ld(n0, n1, v0, v1);
      for (int ks = wave;; ks += 4) {
        const bool more = 4 * (ks + 4) < nkb;
        s4 m0, m1;
        u4 x0v, x1v;
        adv(4 * (ks + 8) < nkb);
        ld(m0, m1, x0v, x1v);
        const bf16x8 A = __builtin_bit_cast(bf16x8, s8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]});
        const bf16x8 X0 = __builtin_bit_cast(bf16x8, w0);
        const bf16x8 X1 = __builtin_bit_cast(bf16x8, ones ? one4 : w1);
        if constexpr (MM != 1) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, X0, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, X1, acc[1], 0, 0, 0);
        }
        if constexpr (MM != 2) {
          ga[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X0, X0, ga[0], 0, 0, 0);
          ga[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X0, X1, ga[1], 0, 0, 0);
          ga[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X1, X1, ga[2], 0, 0, 0);
        }
        if (!more) break;
        h0 = n0; h1 = n1; w0 = v0; w1 = v1;
        n0 = m0; n1 = m1; v0 = x0v; v1 = x1v;
      }
    }
  }
  // ---- block outputs: M / Gram / S folded from pairs to taps, sum dz from D's column 30
  __syncthreads();                        // every wave is done with dys / xc
  static_assert(4 * 32 * 32 * 4 <= 2 * XB_CB * 2, "the Gram tiles fit the input copies");
  float* red = reinterpret_cast<float*>(dys);        // [4][16][32]  D
  // [4][32][32]  Gram tiles (upper blocks)
  float* g6 = MM == 1 ? reinterpret_cast<float*>(xc) : red + 4 * 16 * 32;
  if constexpr (MM != 1) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(wave * 16 + 4 * gq + i) * 32 + 16 * tt + col] = acc[tt][i];
  }
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int ti = b == 2 ? 1 : 0, tj = b == 0 ? 0 : 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      g6[(wave * 32 + 16 * ti + 4 * gq + i) * 32 + 16 * tj + col] = ga[b][i];
  }
  __syncthreads();
  constexpr int OC = MM == 1 ? GRAMC : MOMC;
  float* o = out + ((size_t)rr * G + grp) * OC;
  auto g6v = [&](int t1, int t2) {        // the lower block (1,0) is the transpose of (0,1)
    if (t1 >= 16 && t2 < 16) { const int tmp = t1; t1 = t2; t2 = tmp; }
    float v = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) v += g6[(wv * 32 + t1) * 32 + t2];
    return v;
  };
  if constexpr (MM == 1) {
    for (int e = tid; e < GRAMC; e += 256) {
      float v;
      if (e < 625) {
        const int a = e / 25, b = e % 25;
        const int pa = (a / 5) * 6 + a % 5, pb = (b / 5) * 6 + b % 5;
        v = g6v(pa, pb) + g6v(pa + 1, pb + 1);
      } else {
        const int a = e - 625, pa = (a / 5) * 6 + a % 5;
        v = g6v(pa, 30) + g6v(pa + 1, 30);
      }
      o[e] = v;
    }
    return;
  }
  for (int e = tid; e < MOMC; e += 256) {
    float v = 0.f;
    if (MM == 2 && e >= COUT * 25 && e < COUT * 25 + 650) {
      o[e] = 0.f;                         // Gram / S: the forward's (MM 1) are used instead
      continue;
    }
    if (e < COUT * 25) {
      const int c = e / 25, t = e - c * 25, ky = t / 5, kx = t - ky * 5;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv)
        v += red[(wv * 16 + c) * 32 + ky * 6 + kx] + red[(wv * 16 + 8 + c) * 32 + ky * 6 + kx + 1];
    } else if (e < COUT * 25 + 625) {
      const int a = (e - COUT * 25) / 25, b = (e - COUT * 25) % 25;
      const int pa = (a / 5) * 6 + a % 5, pb = (b / 5) * 6 + b % 5;
      v = g6v(pa, pb) + g6v(pa + 1, pb + 1);      // even pixel of the pair, then the odd one
    } else if (e < COUT * 25 + 650) {
      const int a = e - COUT * 25 - 625, pa = (a / 5) * 6 + a % 5;
      v = g6v(pa, 30) + g6v(pa + 1, 30);
    } else {
      const int c = e - (COUT * 25 + 650);
#pragma unroll
      for (int wv = 0; wv < 4; ++wv) v += red[(wv * 16 + c) * 32 + 30] + red[(wv * 16 + 8 + c) * 32 + 30];
    }
    o[e] = v;
  }
}

// ---------------------------------------------------------------------------- window moments
// The routed backward's M and sum dz (MM 2's output) in window space: dz is nonzero only at the
// coded pixel (ky, kx) of each 2x2 pooling window, so with the window's 6x6 input footprint
// x6[w][oy][ox] = x[2hp + oy - 2][2wp + ox - 2]
//   M[c][dy][dx] = sum_{ky,kx} N[2ky+kx][c][(ky+dy)*6 + kx+dx],  N[k][c][o] = sum_w dz_k[c][w] x6[w][o]
// with dz_k[c][w] = gz[w][c] where the window's code nibble for c is k + 1.  N is one GEMM per
// tile: rows (k, c) = 32 (two 16-row tiles, ky), columns o = 36 footprint offsets + a ones column
// (sum dz) in three 16-column tiles, K = windows.  The A operand is the pooled gradient tile read
// transposed (ds_read_b64_tr_b16 of [window][8 channels], channels duplicated onto rows 8-15) and
// masked in registers by the codes; the B operand is 8 consecutive windows of one parity / shift
// copy of an input row (the xc copies of the pixel-pair kernel).  So the pass stores the pooled
// gradient as it arrives (one 16-byte LDS write per window) instead of scattering a full-
// resolution dz map, and its LDS (29 KB) leaves room for 5 blocks per CU.
constexpr int NWINMAX = (TH / 2) * (WMAX / 2);


__global__ __launch_bounds__(256, 4) void c1p8_moments_win_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ gz, const unsigned* __restrict__ codes,
    float* __restrict__ out, int B, int G, int R, int H, int W, int tps) {
  static_assert(4 * 32 * 48 * 4 <= (2 * XB_CB + NWINMAX * COUT) * 2, "reduction fits the block");
  // xc: the parity/shift input copies, then 16 bytes of bf16 ones and 16 of zeros (the B
  // operand of the sum-dz column and of the padding columns: read like any other column)
  constexpr int KONE = 2 * XB_CB, KZERO = KONE + 8, GZOFF = 2 * XB_CB + 16;
  // one LDS block (the final reduction spans all of it): xc | ones, zeros | gzs | cds
  __shared__ __attribute__((aligned(16))) bf16 smem[GZOFF + NWINMAX * COUT + 2 * NWINMAX];
  bf16* xc = smem;
  bf16* gzs = smem + GZOFF;
  // routing of window pairs per row tile t (ky): word [t][w / 2], bit 2c + kx of the low half =
  // window w routes channel c to pixel (ky, kx), the high half the same for window w + 1
  unsigned (*cds)[NWINMAX / 2] = reinterpret_cast<unsigned (*)[NWINMAX / 2]>(smem + GZOFF + NWINMAX * COUT);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int gq = lane >> 4, col = lane & 15;
  const int Hp = H >> 1, Wp = W >> 1, gpr = Wp >> 3;        // 8-window groups per window row
  const int nwin = (TH / 2) * Wp, ngrp = (TH / 2) * gpr, nstep = (ngrp + 3) >> 2;
  const int grp = (int)blockIdx.x / R, rr = (int)blockIdx.x - grp * R;
  const long long tpg = (long long)B * tps;
  const int t_begin = (int)(grp * tpg + (tpg * rr) / R), t_end = (int)(grp * tpg + (tpg * (rr + 1)) / R);
  if (tid < 16) xc[KONE + tid] = tid < 8 ? (bf16)0x3F80u : (bf16)0u;     // bf16 1.0, 0.0
  // B columns: o = 16u + col < 36 reads copy (b, a) of tile row 2 hp + oy; o = 36 the ones,
  // o > 36 the zeros (their address ignores the k-step: bmask 0)
  int boff[3], bmask[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int o = 16 * u + col, oy = o / 6, ox = o - 6 * oy;
    bmask[u] = o < 36 ? -1 : 0;
    boff[u] = o < 36 ? xbo(ox & 1, ox >> 1, oy, 0) : o == 36 ? KONE : KZERO;
  }
  const unsigned rsh = 2 * (col & 7) + (col >> 3);          // routing bit of this A row
  const int q = col >> 2, p = col & 3;
  // this lane group's first 8-window group and the per-step advance (16 groups)
  const int m0 = 4 * wave + gq, dh = 16 / gpr, dg = 16 - dh * gpr;
  f4 acc[2][3];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 3; ++u) acc[t][u] = f4{0.f, 0.f, 0.f, 0.f};

  int xr[2], xoff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = tid + 256 * s;
    const int r = t >> 4, c = t & 15;
    xr[s] = (r < TH + 4 && c < (W >> 3)) ? r : -(1 << 20);
    xoff[s] = (r - 2) * W + 8 * c;
  }
  u4 xv[2], gv[2];
  unsigned cv[2];
  auto load = [&](int tile) {
    const int n = tile / tps, ty0 = (tile - n * tps) * TH;
    const bf16* xb = x + ((size_t)n * H + ty0) * W;
    const size_t w0 = ((size_t)n * Hp + (ty0 >> 1)) * Wp;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool ok = (unsigned)(ty0 - 2 + xr[s]) < (unsigned)H;
      xv[s] = ldg16(ok ? (const void*)(xb + xoff[s]) : &kZeroC1);
      const int w = min(tid + 256 * s, nwin - 1);
      gv[s] = ldg16(gz + (w0 + w) * COUT);
      cv[s] = codes[w0 + w];
    }
  };
  if (t_begin < t_end) load(t_begin);
  for (int tile = t_begin; tile < t_end; ++tile) {
    __syncthreads();                     // the previous tile's reads of xc / gzs / cds are done
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = tid + 256 * s;
      const int r = t >> 4, c = t & 15;
      const unsigned wv[4] = {xv[s].x, xv[s].y, xv[s].z, xv[s].w};
      const unsigned ev[2] = {(wv[0] & 0xffffu) | (wv[1] << 16), (wv[2] & 0xffffu) | (wv[3] << 16)};
      const unsigned od[2] = {(wv[0] >> 16) | (wv[1] & 0xffff0000u), (wv[2] >> 16) | (wv[3] & 0xffff0000u)};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const unsigned lo = b ? od[0] : ev[0], hi = b ? od[1] : ev[1];
        const unsigned prev_hi = (unsigned)dpp_i<0x111>((int)hi);   // lane c-1 (0 at c = 0)
        const unsigned next_lo = (unsigned)dpp_i<0x101>((int)lo);   // lane c+1
        if (r < TH + 4 && c < (W >> 3)) {
          *reinterpret_cast<uint2*>(&xc[xbo(b, 0, r, 4 * c)]) =
              make_uint2((prev_hi >> 16) | (lo << 16), (lo >> 16) | (hi << 16));
          *reinterpret_cast<uint2*>(&xc[xbo(b, 1, r, 4 * c)]) = make_uint2(lo, hi);
          *reinterpret_cast<uint2*>(&xc[xbo(b, 2, r, 4 * c)]) =
              make_uint2((lo >> 16) | (hi << 16), (hi >> 16) | (next_lo << 16));
        }
      }
      // routing bits: nibble n (0 none, 1 + 2 ky + kx) of channel c -> bit 2c + kx of row tile
      // ky, for all 8 channels at once (nibble-parallel), then paired with the next window
      const unsigned v = cv[s];
      const unsigned n0 = v & 0x11111111u, n1 = (v >> 1) & 0x11111111u, n2 = (v >> 2) & 0x11111111u;
      unsigned rt[2] = {(n0 & ~n1) | ((n1 & ~n0) << 1),      // n == 1, 2: ky 0
                        (n0 & n1) | (n2 << 1)};               // n == 3, 4: ky 1
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {                       // 2-bit fields at 4c -> at 2c
        unsigned f = rt[t2];
        f = (f | (f >> 2)) & 0x0F0F0F0Fu;
        f = (f | (f >> 4)) & 0x00FF00FFu;
        f = (f | (f >> 8)) & 0x0000FFFFu;
        rt[t2] = f | ((unsigned)dpp_i<0x101>((int)f) << 16);  // the next lane's (= window's)
      }
      const int w = tid + 256 * s;
      if (w < nwin) {
        *reinterpret_cast<u4*>(&gzs[w * COUT]) = gv[s];
        if (!(w & 1)) {
          cds[0][w >> 1] = rt[0];
          cds[1][w >> 1] = rt[1];
        }
      }
    }
    if (tile + 1 < t_end) load(tile + 1);   // in flight under this tile's MFMAs
    __syncthreads();
    int hpl = m0 / gpr, gi = m0 - hpl * gpr;
    // a step's LDS operands: pooled-gradient fragment, routing words, three input fragments
    auto fetch = [&](int hp, int gq2, u4& a4, u4& r0, u4& r1, u4 (&bv)[3]) {
      const bool valid = hp < TH / 2;
      const int w0 = hp * Wp + 8 * gq2;
      a4 = u4{0u, 0u, 0u, 0u};
      r0 = u4{0u, 0u, 0u, 0u};
      r1 = u4{0u, 0u, 0u, 0u};
      if (valid) {
        const s4 g0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&gzs[(w0 + q) * COUT + 4 * (p & 1)]);
        const s4 g1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)&gzs[(w0 + 4 + q) * COUT + 4 * (p & 1)]);
        const u2 lo2 = __builtin_bit_cast(u2, g0), hi2 = __builtin_bit_cast(u2, g1);
        a4 = u4{lo2.x, lo2.y, hi2.x, hi2.y};
        r0 = *reinterpret_cast<const u4*>(&cds[0][w0 >> 1]);
        r1 = *reinterpret_cast<const u4*>(&cds[1][w0 >> 1]);
      }
      const int bs = 2 * hp * XB_RS + 8 * gq2;
#pragma unroll
      for (int u = 0; u < 3; ++u) bv[u] = *reinterpret_cast<const u4*>(&xc[(bs & bmask[u]) + boff[u]]);
    };
    for (int j = wave; j < nstep; j += 4) {
      u4 a4, r0, r1, bv[3];
      fetch(hpl, gi, a4, r0, r1, bv);
      const unsigned av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const u4 rw = t ? r1 : r0;
        const unsigned rv[4] = {rw.x, rw.y, rw.z, rw.w};
        unsigned am[4];
        // a routed window keeps its pooled gradient: (bit) x bf16 pattern, both halves at once
#pragma unroll
        for (int d = 0; d < 4; ++d)
          am[d] = __builtin_bit_cast(unsigned, __builtin_bit_cast(us2, av[d]) *
                                                   __builtin_bit_cast(us2, (rv[d] >> rsh) & 0x00010001u));
        const bf16x8 A = __builtin_bit_cast(bf16x8, u4{am[0], am[1], am[2], am[3]});
#pragma unroll
        for (int u = 0; u < 3; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, __builtin_bit_cast(bf16x8, bv[u]), acc[t][u], 0, 0, 0);
      }
      gi += dg;
      hpl += dh;
      if (gi >= gpr) { gi -= gpr; ++hpl; }
    }
  }
  // ---- block output: fold N's rows (k, c) and footprint columns into M, sum dz from column 36
  __syncthreads();
  float* red = reinterpret_cast<float*>(xc);          // [4 waves][32 rows][48 cols]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(wave * 32 + 16 * t + 4 * gq + i) * 48 + 16 * u + col] = acc[t][u][i];
  __syncthreads();
  float* o = out + ((size_t)rr * G + grp) * MOMC;
  for (int e = tid; e < MOMC; e += 256) {
    float v = 0.f;
    if (e < COUT * 25) {
      const int c = e / 25, t = e - c * 25, dy = t / 5, dx = t - dy * 5;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v += red[(wv * 32 + 8 * k + c) * 48 + ((k >> 1) + dy) * 6 + (k & 1) + dx];
    } else if (e >= COUT * 25 + 650) {
      const int c = e - (COUT * 25 + 650);
#pragma unroll
      for (int wv = 0; wv < 4; ++wv)
#pragma unroll
        for (int k = 0; k < 4; ++k) v += red[(wv * 32 + 8 * k + c) * 48 + 36];
    }
    o[e] = v;                             // Gram / S slots zero: the forward's Gram is used
  }
}

// BN backward + dW of the layer from the row-summed routed moments m [G][MOMC] (float64):
//   sum dz y = w . M + b sum dz  (the exact conv output at the routed pixels)
//   sum dz xhat = (sum dz y - mean sum dz) invstd;  coef (k1, kx, k0) as avd_bn_bwd_finalize;
//   dW[c][t] = sum_g k1 M + kx (sum_t' w[c][t'] Gram[t'][t] + b S[t]) + k0 S[t]
// and dgamma / dbeta / dbias (= sum dy, analytically 0) summed over the groups.
__global__ __launch_bounds__(256) void c1p8_codes_combine_kernel(
    const float* __restrict__ m, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    long long count, float* __restrict__ dw, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dbias, float* __restrict__ coef, int G, const float* __restrict__ gram_ext) {
  __shared__ double sk[32 * COUT][3];
  __shared__ double s12[32 * COUT][2];
  const int tid = threadIdx.x;
  const double n = (double)count;
  if (tid < G * COUT) {
    const int g = tid / COUT, c = tid - g * COUT;
    const float* mg = m + (size_t)g * MOMC;
    const double b = bias ? (double)bias[c] : 0.0;
    const double s1 = mg[COUT * 25 + 650 + c];
    double sy = b * s1;
    for (int t = 0; t < 25; ++t) sy = fma((double)bf2f(wk[c * 32 + t]), (double)mg[c * 25 + t], sy);
    const double mu = mean[g * COUT + c], is = invstd[g * COUT + c], ga = gamma[c];
    const double s2 = (sy - mu * s1) * is;                   // sum dz * xhat
    const double k1 = ga * is, kx = -ga * is * is * s2 / n, k0 = -ga * is * s1 / n + ga * is * is * mu * s2 / n;
    sk[tid][0] = k1; sk[tid][1] = kx; sk[tid][2] = k0;
    s12[tid][0] = s1; s12[tid][1] = s2;
    if (coef) {
      coef[tid * 3 + 0] = (float)k1;
      coef[tid * 3 + 1] = (float)kx;
      coef[tid * 3 + 2] = (float)k0;
    }
  }
  __syncthreads();
  if (tid < COUT) {
    double dg = 0.0, db = 0.0, dbi = 0.0;
    for (int g = 0; g < G; ++g) {
      const int i = g * COUT + tid;
      const double mu = mean[i];
      dg += s12[i][1];
      db += s12[i][0];
      dbi += sk[i][0] * s12[i][0] + sk[i][1] * mu * n + sk[i][2] * n;
    }
    if (dgamma) dgamma[tid] = (float)dg;
    if (dbeta) dbeta[tid] = (float)db;
    if (dbias) dbias[tid] = (float)dbi;
  }
  for (int e = tid; e < COUT * 25; e += 256) {
    const int c = e / 25, t = e - c * 25;
    double wr[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) wr[k] = (double)bf2f(wk[c * 32 + k]);
    const double b = bias ? (double)bias[c] : 0.0;
    double acc = 0.0;
    for (int g = 0; g < G; ++g) {
      const float* mg = m + (size_t)g * MOMC;
      // Gram / S: the forward statistics pass's (gram_ext [G][GRAMC]) or this pass's own
      const float* gram = gram_ext ? gram_ext + (size_t)g * GRAMC : mg + COUT * 25;
      const double sx = gram[625 + t];
      double sy = b * sx;
#pragma unroll
      for (int k = 0; k < 25; ++k) sy = fma(wr[k], (double)gram[k * 25 + t], sy);
      const int i = g * COUT + c;
      acc += sk[i][0] * mg[e] + sk[i][1] * sy + sk[i][2] * sx;
    }
    dw[e] = (float)acc;
  }
}

// BatchNorm statistics of the conv output from the Gram pass (MM 1), float64: per group and
// channel sum y = w . S + n b and sum y^2 = w^T Gram w + 2 b w . S + n b^2 (the exact conv
// output y = w . x25 + b with the bf16 weights), then avd_bn_finalize's outputs: mean, invstd,
// BN scale / shift, and the running statistics in group (view) order.
__global__ __launch_bounds__(256) void c1p8_gram_finalize_kernel(
    const float* __restrict__ gram, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    long long count, float* __restrict__ mean_o, float* __restrict__ invstd_o,
    float* __restrict__ scale_o, float* __restrict__ shift_o, float* __restrict__ rm,
    float* __restrict__ rv, int G) {
  // thread (c, a) < 200 forms w[c][a] (Gram w[c])[a] and w[c][a] S[a] of one group; the 25
  // partials per channel are summed by thread c (fixed order), which also carries the running
  // statistics through the groups in order
  __shared__ double wsh[COUT * 25];
  __shared__ double pq[COUT * 25], ps[COUT * 25];
  const int tid = threadIdx.x;
  if (tid < COUT * 25) wsh[tid] = (double)bf2f(wk[(tid / 25) * 32 + tid % 25]);
  const int c = tid / 25, a = tid - c * 25;
  const double n = (double)count;
  double rmean = 0.0, rvar = 0.0, b = 0.0;
  if (tid < COUT) {
    rmean = rm ? (double)rm[tid] : 0.0;
    rvar = rv ? (double)rv[tid] : 0.0;
    b = bias ? (double)bias[tid] : 0.0;
  }
  __syncthreads();
  for (int g = 0; g < G; ++g) {
    const float* gm = gram + (size_t)g * GRAMC;
    if (tid < COUT * 25) {
      double r = 0.0;
#pragma unroll
      for (int t = 0; t < 25; ++t) r = fma((double)gm[a * 25 + t], wsh[c * 25 + t], r);
      const double wa = wsh[tid];
      pq[tid] = wa * r;
      ps[tid] = wa * (double)gm[625 + a];
    }
    __syncthreads();
    if (tid < COUT) {
      double q = 0.0, ws = 0.0;
      for (int k = 0; k < 25; ++k) {
        q += pq[tid * 25 + k];
        ws += ps[tid * 25 + k];
      }
      const double mean = (ws + n * b) / n;
      const double ey2 = (q + 2.0 * b * ws + n * b * b) / n;
      double var = ey2 - mean * mean;
      if (var < 0) var = 0;
      const double invstd = 1.0 / sqrt(var + (double)eps);
      const double sc = (double)gamma[tid] * invstd;
      mean_o[g * COUT + tid] = (float)mean;
      invstd_o[g * COUT + tid] = (float)invstd;
      scale_o[g * COUT + tid] = (float)sc;
      shift_o[g * COUT + tid] = (float)((double)beta[tid] - mean * sc);
      rmean = (1.0 - momentum) * rmean + momentum * mean;
      rvar = (1.0 - momentum) * rvar + momentum * var * n / (n - 1.0);
    }
    __syncthreads();
  }
  if (rm && tid < COUT) {
    rm[tid] = (float)rmean;
    rv[tid] = (float)rvar;
  }
}

int c1p8_codes_rows(int N, int B) {
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, c1p8_moments_codes_kernel<0>, 256, 0) !=
            hipSuccess || per <= 0)
      per = 2;
    resident = cus * per;
  }
  constexpr int waves = 8;
  const int G = N / B;
  return std::max(1, std::min(grid_cap(resident * waves) / G, B));
}

int c1p8_moment_rows(int N, int B) {
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, c1p8_moments_kernel, 256, 0) !=
            hipSuccess || per <= 0)
      per = 2;
    resident = cus * per;
  }
  // several waves of blocks: beside the concurrent streams' persistent kernels a block may start
  // late, and shorter blocks bound that tail
  constexpr int waves = 8;
  const int G = N / B;
  return std::max(1, std::min(grid_cap(resident * waves) / G, B));
}

}  // namespace

// rows per BN group (stats / reduce passes; moments pass 4: rows of both its outputs) or slabs
// (wgrad pass)
int avd_c1r_rows(int pass, int N, int B, int H) {
  if (pass == 4) return c1p8_moment_rows(N, B);
  return pass == RC_WGRAD ? rc_wgrad_slabs(N, H) : B * 4;
}

int avd_c1p8_moment_cols() { return MOM5; }

int avd_c1p8_combine(const float* m, const float* coef, const void* wk, const float* bias,
                     float* dw, int G, hipStream_t st) {
  c1p8_combine_kernel<<<avd_cdiv(COUT * 25, 64), 64, 0, st>>>(m, coef, (const bf16*)wk, bias, dw, G);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_c1r_launch(int pass, const void* x, const void* wk, const float* bias, const float* scale,
                   const float* shift, const float* mean, const float* invstd, const float* coef,
                   const void* gz, void* z, float* out, int N, int B, int H, int W,
                   hipStream_t st) {
  const int tps = H / TH, ntiles = N * tps;
  if (pass == 4) {
    const int G = N / B, R = c1p8_moment_rows(N, B);
    c1p8_moments_kernel<<<G * R, 256, 0, st>>>((const bf16*)x, (const bf16*)wk, bias, scale, shift,
                                               mean, invstd, (const bf16*)gz, out, B, G, R, H, W, tps);
    AVD_CHECK_LAUNCH();
    return AVD_OK;
  }
  const int grid = pass == RC_WGRAD ? rc_wgrad_slabs(N, H) : N;
#define AVD_RC(PS)                                                                             \
  c1p8_recompute_kernel<PS><<<grid, 256, 0, st>>>(                                             \
      (const bf16*)x, (const bf16*)wk, bias, scale, shift, mean, invstd, coef, (const bf16*)gz, \
      (bf16*)z, out, B, H, W, ntiles, tps, nullptr)
  switch (pass) {
    case RC_STATS: AVD_RC(RC_STATS); break;
    case RC_APPLY: AVD_RC(RC_APPLY); break;
    case RC_REDUCE: AVD_RC(RC_REDUCE); break;
    case RC_WGRAD: AVD_RC(RC_WGRAD); break;
    default: return AVD_ERR_ARG;
  }
#undef AVD_RC
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// ---------------------------------------------------------------------------- routed backward API
int avd_c1_codes_rows(int N, int B) { return c1p8_codes_rows(N, B); }
int avd_c1_codes_cols() { return MOMC; }

int avd_c1_apply_codes_launch(const void* x, const void* wk, const float* bias, const float* scale,
                              const float* shift, void* z, unsigned* codes, int N, int B, int H,
                              int W, hipStream_t st) {
  const int tps = H / TH;
  c1p8_recompute_kernel<RC_APPLY><<<N, 256, 0, st>>>(
      (const bf16*)x, (const bf16*)wk, bias, scale, shift, nullptr, nullptr, nullptr, nullptr,
      (bf16*)z, nullptr, B, H, W, N * tps, tps, codes);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_c1_moments_codes_launch(const void* x, const void* gz, const unsigned* codes, float* out,
                                int N, int B, int H, int W, hipStream_t st) {
  const int tps = H / TH, G = N / B, R = c1p8_codes_rows(N, B);
  c1p8_moments_codes_kernel<0><<<G * R, 256, 0, st>>>((const bf16*)x, (const bf16*)gz, codes, out, B,
                                                      G, R, H, W, tps);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// the Gram pass (forward statistics) and the backward's moments without the Gram (MM 1 / 2)
int avd_c1_gram_launch(const void* x, float* out, int N, int B, int H, int W, hipStream_t st) {
  const int tps = H / TH, G = N / B, R = c1p8_codes_rows(N, B);
  c1p8_moments_codes_kernel<1><<<G * R, 256, 0, st>>>((const bf16*)x, nullptr, nullptr, out, B, G, R,
                                                      H, W, tps);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_c1_moments_nogram_launch(const void* x, const void* gz, const unsigned* codes, float* out,
                                 int N, int B, int H, int W, hipStream_t st) {
  const int tps = H / TH, G = N / B, R = c1p8_codes_rows(N, B);
  // the window-space pass (round 4; the pixel-pair pass it replaced: 226 vs 159 us at N = 7168)
  c1p8_moments_win_kernel<<<G * R, 256, 0, st>>>((const bf16*)x, (const bf16*)gz, codes, out, B, G, R,
                                                 H, W, tps);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_c1_gram_cols() { return GRAMC; }

int avd_c1_gram_finalize_launch(const float* gram, const void* wk, const float* bias,
                                const float* gamma, const float* beta, float eps, float momentum,
                                long long count, float* mean, float* invstd, float* scale,
                                float* shift, float* rm, float* rv, int G, hipStream_t st) {
  c1p8_gram_finalize_kernel<<<1, 256, 0, st>>>(gram, (const bf16*)wk, bias, gamma, beta, eps, momentum,
                                              count, mean, invstd, scale, shift, rm, rv, G);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_c1_codes_combine_launch(const float* m, const void* wk, const float* bias,
                                const float* gamma, const float* mean, const float* invstd,
                                long long count, float* dw, float* dgamma, float* dbeta,
                                float* dbias, float* coef, int G, hipStream_t st,
                                const float* gram) {
  if (G <= 0 || G > 32) return AVD_ERR_SHAPE;
  c1p8_codes_combine_kernel<<<1, 256, 0, st>>>(m, (const bf16*)wk, bias, gamma, mean, invstd, count,
                                               dw, dgamma, dbeta, dbias, coef, G, gram);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}
