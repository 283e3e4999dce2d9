// The CentralNet IMAGE conv1 backward routed by forward codes (CentralUnimodalImage conv1 -> bn1
// -> relu -> maxpool, unimodal.py:127-141: Conv2d(1, 32, 5, padding=2) on 28x28 images, bf16).
//
// The forward's BN -> ReLU -> pool pass (c1r5_apply_kernel below) writes, per
// pooling window and channel, where nn.MaxPool2d's gradient goes (nibble = 1 + the window
// position of the first argmax of relu(bn(y)) when that max is > 0, else 0).  The backward of
// conv1 + bn1 is then linear in three moments of the input patches x25 (as the audio conv1's,
// conv_c1p.hip): dy = k1 dz + kx y + k0 and y = w . x25 + b give
//   dW[c][t] = sum_g k1 M[g][c][t] + kx (sum_t' w[c][t'] Gram[g][t'][t] + b[c] S[g][t]) + k0 S[g][t]
//   sum dz y = w . M + b sum dz     (the BN backward's second sum, at the exact conv output)
// with M = sum dz x25, Gram = sum x25 x25^T, S = sum x25 per BN group.  This pass forms them with
// no y, no argmax and no im2col gather (the recomputing pass 4 of c1r3_kernel spends its time
// there: 25 scalar LDS reads per pixel):
//   * GEMM view M = dZ^T X over K = pixels: a 32-pixel k-block is one image row on a 32-column
//     virtual width (columns 28..31 zero), so a lane's 8 consecutive k of X for tap (ty, tx) are
//     8 consecutive pixels of ONE row of a shifted copy of the image -- one aligned ds_read_b128
//     from copy[tx][row + ty], no gather.  Five copies (tx = -2..2, columns >= 28 zeroed) plus a
//     constant "ones" copy (tap 25: sum dz and S come out of the same MFMAs) are built per sample.
//   * dZ is channel-major in LDS ([32][28][32]): dz = gz at the coded pixel of each window, 0 at
//     the other three -- an A fragment is one ds_read_b128 of 8 pixels of one channel.
//   * per image row: 2 channel tiles x 2 tap tiles of D += dZ X and the Gram tiles (0,0) (0,1)
//     (1,1) (the X fragment is its own transpose's A operand): 7 MFMAs, 4 LDS reads.
// Blocks own contiguous sample ranges of one BN group (G x R blocks); each writes one row of
// MOMC5 = M [32][25] | Gram [25][25] | S [25] | sum dz [32] floats, reduced with avd_sum_rows.
#include <algorithm>
#include <cstdlib>

#include "common.h"

using namespace avd;

namespace {

constexpr int C = 32, KK = 25, IH = 28, IW = 28;            // channels, taps, image
constexpr int HP = IH / 2, WP = IW / 2, NWIN = HP * WP;     // pooling windows per sample
constexpr int MOMC5 = C * KK + KK * KK + KK + C;
constexpr int C1R5_GMAX = 32;                              // BN groups served by the combine
constexpr int XS_R = IH + 4, XS_C = 40;                     // staged image, 2-pixel halo, 16-B rows
constexpr int LDS_X = XS_R * XS_C;                           // bf16 elements

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;   // raw bf16 bits
typedef __attribute__((ext_vector_type(2))) unsigned short us2;
typedef __attribute__((ext_vector_type(2))) unsigned us2x;
typedef __attribute__((ext_vector_type(4))) short s4;

template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}

// per-thread global vectors of one sample: x 98, gz 784, codes 196 (16-byte vectors)
constexpr int NXV = IH * IW / 8, NGV = NWIN * C / 8, NCV = NWIN * 8 / 8;
constexpr int NVEC = NXV + NGV + NCV, VPT = (NVEC + 255) / 256;

// ---------------------------------------------------------------------------- window moments
// The same moments in window space (as the audio conv1's c1p8_moments_win_kernel): dz is
// nonzero only at the coded pixel (ky, kx) of each 2x2 pooling window, so with the window's 6x6
// input footprint x6[w][oy][ox] = x[2hp + oy - 2][2wp + ox - 2]
//   M[c][dy][dx] = sum_{ky,kx} N[2ky+kx][c][(ky+dy)*6 + kx+dx],  N[k][c][o] = sum_w dz_k[c][w] x6[w][o]
// and the pixel Gram is the fold of the window-footprint Gram G6 = sum_w x6 x6^T over the four
// window positions (S from G6's ones column).  Wave o owns channel octet o: its A operand is the
// pooled gradient of 8 channels read transposed from the [window slot][32 ch] tile and masked by
// routing bits in registers -- no dz map, no scatter (the round-3 kernel's 16-way / 4-way LDS
// bank conflicts).  Windows sit in slots hp * 16 + wp (wp 14, 15: zero padding, and their input
// copies are zeroed so G6 sees no phantom windows); a k-step is 4 groups of 8 slots.
constexpr int C1R5W_OCC = 3;                                  // blocks per CU
constexpr int WSLOT = 16, NSLOT = HP * WSLOT;                 // 224 window slots per sample
// input copies [parity][shift][P half][row][8 P]: B reads 0.67 extra cycles, copy writes 0
// (tools/lds_conflicts.py)
constexpr int WX_R = 8, WX_H = 256, WX_A = 536, WX_B = 1728;
constexpr int W_XS = 0, W_XC = W_XS + LDS_X, W_K1 = W_XC + 2 * WX_B, W_GZ = W_K1 + 16;
constexpr int GZS = C + 8;                                     // window slot stride: 80 B (tr16 reads of the
                                                               // four slot groups on distinct banks)
constexpr int W_CDS = W_GZ + NSLOT * GZS;                      // u32 routing words follow (bf16 units)
constexpr int W_END = W_CDS + 2 * (4 * 2 * (NSLOT / 2));
constexpr int W_RED = 4 * 2 * 16 * 48 + 48 * 48;               // epilogue floats
constexpr int W_LDS = (W_END * 2 > W_RED * 4 ? W_END * 2 : W_RED * 4);

__global__ __launch_bounds__(256, C1R5W_OCC) void c1r5_moments_win_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ gz, const unsigned short* __restrict__ codes,
    float* __restrict__ out, int B, int G, int R) {
  static_assert(W_XC % 8 == 0 && W_GZ % 8 == 0 && W_CDS % 8 == 0, "16-byte aligned regions");
  __shared__ __attribute__((aligned(16))) char lds[W_LDS];
  bf16* sm = reinterpret_cast<bf16*>(lds);
  bf16* xs = sm + W_XS;
  bf16* xc = sm + W_XC;
  bf16* gzs = sm + W_GZ;
  unsigned* cds = reinterpret_cast<unsigned*>(sm + W_CDS);     // [octet][ky][pair]
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int gq = lane >> 4, col = lane & 15, q = col >> 2, p = col & 3;
  const int grp = (int)blockIdx.x / R, rr = (int)blockIdx.x - grp * R;
  const int s_begin = grp * B + (int)(((long long)B * rr) / R);
  const int s_end = grp * B + (int)(((long long)B * (rr + 1)) / R);

  // constant parts: zero image halo, zero padding slots / routing, the ones / zeros B columns
  for (int i = tid; i < (W_END - W_XS) / 8; i += 256) reinterpret_cast<u4*>(sm)[i] = u4{0u, 0u, 0u, 0u};
  __syncthreads();
  if (tid < 8) sm[W_K1 + tid] = (bf16)0x3F80u;                 // bf16 1.0 (W_K1 + 8.. stay 0)

  // B columns: o = 16u + col < 36 reads copy (b, a) at row 2 hp + oy; 36 the ones, > 36 zeros
  int boff[3], bmask[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int o = 16 * u + col, oy = o / 6, ox = o - 6 * oy;
    bmask[u] = o < 36 ? -1 : 0;
    boff[u] = o < 36 ? W_XC + (ox & 1) * WX_B + (ox >> 1) * WX_A + oy * WX_R
                     : W_K1 + (o == 36 ? 0 : 8);
  }
  const unsigned rsh = 2 * (col & 7) + (col >> 3);            // routing bit of this A row
  // G6 tiles (tu <= tv) of this wave: tiles wave and wave + 4 of (00 01 02 11 12 22)
  const int gt0 = wave, gt1 = wave + 4;
  auto tu_of = [](int t) { return t < 3 ? 0 : t < 5 ? 1 : 2; };
  auto tv_of = [](int t) { return t < 3 ? t : t < 5 ? t - 2 : 2; };
  f4 acc[2][3], ga[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    ga[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 3; ++u) acc[t][u] = f4{0.f, 0.f, 0.f, 0.f};
  }

  u4 vv[VPT];
  auto load = [&](int n) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int e = tid + 256 * j;
      if (e < NXV) vv[j] = ldg16(x + (size_t)n * IH * IW + 8 * e);
      else if (e < NXV + NGV) vv[j] = ldg16(gz + (size_t)n * NWIN * C + 8 * (e - NXV));
      else if (e < NVEC) vv[j] = ldg16(codes + (size_t)n * NWIN * 8 + 8 * (e - NXV - NGV));
    }
  };
  if (s_begin < s_end) load(s_begin);
  for (int n = s_begin; n < s_end; ++n) {
    __syncthreads();                      // the previous sample's k-loop is done with the tiles
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int e = tid + 256 * j;
      if (e < NXV) {
        const unsigned w4[4] = {vv[j].x, vv[j].y, vv[j].z, vv[j].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int pix = 8 * e + 2 * k, r = pix / IW, c = pix - r * IW;
          *reinterpret_cast<unsigned*>(xs + (r + 2) * XS_C + c + 2) = w4[k];
        }
      } else if (e < NXV + NGV) {
        const int qv = e - NXV, w = qv >> 2, hp = w / WP, wp = w - hp * WP;
        *reinterpret_cast<u4*>(gzs + (hp * WSLOT + wp) * GZS + 8 * (qv & 3)) = vv[j];
      }
      // routing bits of one window (codes vectors: one per window, lanes = consecutive windows):
      // per channel octet o and row tile ky a 16-bit word (bit 2c + kx), paired with the next
      // window's in the high half (computed by every lane: the DPP reads the neighbour)
      if (256 * j + 255 < NXV + NGV || 256 * j >= NVEC) continue;   // no codes vector in slot j
      const int w = e - NXV - NGV;
      const unsigned cw[4] = {vv[j].x, vv[j].y, vv[j].z, vv[j].w};
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const unsigned v = cw[o];
        const unsigned n0 = v & 0x11111111u, n1 = (v >> 1) & 0x11111111u, n2 = (v >> 2) & 0x11111111u;
        unsigned rt[2] = {(n0 & ~n1) | ((n1 & ~n0) << 1), (n0 & n1) | (n2 << 1)};
#pragma unroll
        for (int ky = 0; ky < 2; ++ky) {
          unsigned f = rt[ky];
          f = (f | (f >> 2)) & 0x0F0F0F0Fu;
          f = (f | (f >> 4)) & 0x00FF00FFu;
          f = (f | (f >> 8)) & 0x0000FFFFu;
          f |= (unsigned)dppi<0x101>((int)f) << 16;
          if (e >= NXV + NGV && e < NVEC) {
            const int hp = w / WP, wp = w - hp * WP;
            if (!(wp & 1)) cds[(o * 2 + ky) * (NSLOT / 2) + ((hp * WSLOT + wp) >> 1)] = f;
          }
        }
      }
    }
    __syncthreads();
    if (n + 1 < s_end) load(n + 1);       // in flight under this sample's copies and MFMAs
    // parity / shift copies: xc[b][a][r][P] = x[r - 2][2(P + a - 1) + b] = xs[r][2P + 2a + b]
    // (P 14, 15: zero); chunk (b, a, r, P0): one wave per (b, a), two aligned row reads
    for (int i = tid; i < 6 * 32 * 2; i += 256) {
      const int ba = __builtin_amdgcn_readfirstlane(i >> 6), b = ba / 3, a = ba - 3 * b;
      const int r = i & 31, P0 = 8 * ((i >> 5) & 1);          // 16 lanes = 16 rows: distinct slots
      const bf16* srow = xs + r * XS_C + 2 * P0;
      const u4 l0 = *reinterpret_cast<const u4*>(srow), l1 = *reinterpret_cast<const u4*>(srow + 8);
      const u4 l2 = *reinterpret_cast<const u4*>(srow + 16);
      const unsigned d[12] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w, l2.x, l2.y, l2.z, l2.w};
      unsigned o4[4];
      // element 2(P + a) + b of the row: low (b = 0) / high (b = 1) half of dword P + a
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {
        unsigned lo, hi;
        switch (a) {
          case 0: lo = d[2 * dd]; hi = d[2 * dd + 1]; break;
          case 1: lo = d[2 * dd + 1]; hi = d[2 * dd + 2]; break;
          default: lo = d[2 * dd + 2]; hi = d[2 * dd + 3]; break;
        }
        o4[dd] = b ? __builtin_amdgcn_perm(hi, lo, 0x07060302u) : __builtin_amdgcn_perm(hi, lo, 0x05040100u);
      }
      if (P0) o4[3] = 0u;                                      // P = 14, 15: padding windows
      *reinterpret_cast<u4*>(xc + b * WX_B + a * WX_A + (P0 ? WX_H : 0) + r * WX_R) = u4{o4[0], o4[1], o4[2], o4[3]};
    }
    __syncthreads();
    // k-loop: 7 steps of 4 slot groups; wave = channel octet
    for (int j = 0; j < 7; ++j) {
      const int m = 4 * j + gq, hp = m >> 1, wp0 = 8 * (m & 1), s0 = hp * WSLOT + wp0;
      const s4 g0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s4*)(gzs + (s0 + q) * GZS + 8 * wave + 4 * (p & 1)));
      const s4 g1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s4*)(gzs + (s0 + 4 + q) * GZS + 8 * wave + 4 * (p & 1)));
      const u4 rw0 = *reinterpret_cast<const u4*>(cds + (wave * 2 + 0) * (NSLOT / 2) + (s0 >> 1));
      const u4 rw1 = *reinterpret_cast<const u4*>(cds + (wave * 2 + 1) * (NSLOT / 2) + (s0 >> 1));
      const int bs = 2 * hp * WX_R + (wp0 ? WX_H : 0);
      u4 bv[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) bv[u] = *reinterpret_cast<const u4*>(sm + (bs & bmask[u]) + boff[u]);
      const us2x lo2 = __builtin_bit_cast(us2x, g0), hi2 = __builtin_bit_cast(us2x, g1);
      const unsigned av[4] = {lo2.x, lo2.y, hi2.x, hi2.y};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const u4 rw = t ? rw1 : rw0;
        const unsigned rv[4] = {rw.x, rw.y, rw.z, rw.w};
        unsigned am[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
          am[d] = __builtin_bit_cast(unsigned, __builtin_bit_cast(us2, av[d]) *
                                                   __builtin_bit_cast(us2, (rv[d] >> rsh) & 0x00010001u));
        const bf16x8 A = __builtin_bit_cast(bf16x8, u4{am[0], am[1], am[2], am[3]});
#pragma unroll
        for (int u = 0; u < 3; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, __builtin_bit_cast(bf16x8, bv[u]), acc[t][u], 0, 0, 0);
      }
      // this wave's window-footprint Gram tiles (the B fragments are their own transposes)
#pragma unroll
      for (int gi = 0; gi < 2; ++gi) {
        const int gt = gi ? gt1 : gt0;
        if (gt < 6) {
          const int tu = tu_of(gt), tv = tv_of(gt);
          const u4 bu = tu == 0 ? bv[0] : tu == 1 ? bv[1] : bv[2];
          const u4 bw = tv == 0 ? bv[0] : tv == 1 ? bv[1] : bv[2];
          ga[gi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bu),
                                                           __builtin_bit_cast(bf16x8, bw), ga[gi], 0, 0, 0);
        }
      }
    }
  }
  // ---- block row: N per wave (its octet), G6 tiles, folded to M / Gram / S / sum dz
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);          // [4 waves][2 ky][16 rows][48 cols]
  float* g6 = red + 4 * 2 * 16 * 48;                   // [48][48] (tiles tu <= tv)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[((wave * 2 + t) * 16 + 4 * gq + i) * 48 + 16 * u + col] = acc[t][u][i];
#pragma unroll
  for (int gi = 0; gi < 2; ++gi) {
    const int gt = gi ? gt1 : gt0;
    if (gt < 6) {
      const int tu = tu_of(gt), tv = tv_of(gt);
#pragma unroll
      for (int i = 0; i < 4; ++i) g6[(16 * tu + 4 * gq + i) * 48 + 16 * tv + col] = ga[gi][i];
    }
  }
  __syncthreads();
  auto G6 = [&](int i, int jj) {           // symmetric: the lower tiles from the upper
    return (i >> 4) <= (jj >> 4) ? g6[i * 48 + jj] : g6[jj * 48 + i];
  };
  float* o = out + ((size_t)rr * G + grp) * MOMC5;
  for (int e = tid; e < MOMC5; e += 256) {
    float v = 0.f;
    if (e < C * KK) {
      const int c = e / KK, t = e - c * KK, dy = t / 5, dx = t - 5 * dy;
      const int ow = c >> 3, c8 = c & 7;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v += red[((ow * 2 + (k >> 1)) * 16 + 8 * (k & 1) + c8) * 48 + ((k >> 1) + dy) * 6 + (k & 1) + dx];
    } else if (e < C * KK + KK * KK) {
      const int qq = e - C * KK, t1 = qq / KK, t2 = qq - KK * t1;
      const int y1 = t1 / 5, x1 = t1 - 5 * y1, y2 = t2 / 5, x2 = t2 - 5 * y2;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v += G6(((k >> 1) + y1) * 6 + (k & 1) + x1, ((k >> 1) + y2) * 6 + (k & 1) + x2);
    } else if (e < C * KK + KK * KK + KK) {
      const int t = e - C * KK - KK * KK, dy = t / 5, dx = t - 5 * dy;
#pragma unroll
      for (int k = 0; k < 4; ++k) v += G6(((k >> 1) + dy) * 6 + (k & 1) + dx, 36);
    } else {
      const int c = e - (C * KK + KK * KK + KK), ow = c >> 3, c8 = c & 7;
#pragma unroll
      for (int k = 0; k < 4; ++k) v += red[((ow * 2 + (k >> 1)) * 16 + 8 * (k & 1) + c8) * 48 + 36];
    }
    o[e] = v;
  }
}

// ---------------------------------------------------------------------------- forward apply
// BN -> ReLU -> 2x2 max-pool of the recomputed conv output plus the routing codes, in one pass
// over the 180 MB input (the layer's y is never stored).  The MFMA runs PIXEL-major: A = the
// im2col fragment of 16 pixels (all 25 taps in one K = 32 step), B = the weights of 16 channels
// (the same registers the channel-major passes use as A), so D lane l holds y for pixels
// 4 (l / 16) .. +3 of one channel.  With the 16 pixels of a group ordered window by window
// (pixel p = 4 w + k: window w of 4 side by side, k = (0,0) (0,1) (1,0) (1,1)), every lane holds
// ONE whole pooling window of one channel: the max, the first argmax and the > 0 test are
// in-lane integer compares of the f32 bn(y) bits -- no cross-lane exchange -- and y is the same
// bf16(acc + b) as the stored-y conv's (bit-identical pooled map, tests/test_gpu_benchsize.py).
constexpr int AP_XS = IW + 8, AP_XR = IH + 4;                // staged rows: 2-pixel halo + pad
constexpr int AP_GROUPS = (IH / 2) * 4;                      // 16-pixel groups per sample

__global__ __launch_bounds__(256) void c1r5_apply_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, bf16* __restrict__ z,
    unsigned short* __restrict__ codes, int N, int B) {
  __shared__ __attribute__((aligned(16))) bf16 xs[2][AP_XR * AP_XS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int per = N / (int)gridDim.x, extra = N % (int)gridDim.x;
  const int s0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int s1 = s0 + per + ((int)blockIdx.x < extra ? 1 : 0);

  bf16x8 aw[2];
  float bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    aw[t] = *reinterpret_cast<const bf16x8*>(wk + (16 * t + r16) * 32 + 8 * g);
    bv[t] = bias ? bias[16 * t + r16] : 0.f;
  }
  // this lane's A row: pixel r16 of a group = window r16 / 4, position r16 % 4; its taps
  // 8 g .. 8 g + 7 (>= 25: zero)
  const int pk = r16 & 3, pcol = 2 * (r16 >> 2) + (pk & 1), prow = pk >> 1;
  int toff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = 8 * g + j;
    toff[j] = t < KK ? (prow + t / 5) * AP_XS + pcol + t % 5 : -1;
  }
  for (int i = tid; i < 2 * AP_XR * AP_XS / 2; i += 256) reinterpret_cast<unsigned*>(xs)[i] = 0u;

  u4 xv = u4{0u, 0u, 0u, 0u};
  auto load = [&](int n) {
    if (tid < NXV) xv = ldg16(x + (size_t)n * IH * IW + 8 * tid);
  };
  if (s0 < s1) load(s0);
  __syncthreads();
  int cg = -1;
  float sc[2], sf[2];
  for (int n = s0; n < s1; ++n) {
    bf16* xb = xs[(n - s0) & 1];
    if (tid < NXV) {
      // a pixel pair never straddles a row (28 even): dword stores, 4-byte aligned
      const unsigned w4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int pix = 8 * tid + 2 * k, r = pix / IW, c = pix - r * IW;
        *reinterpret_cast<unsigned*>(xb + (r + 2) * AP_XS + c + 2) = w4[k];
      }
    }
    __syncthreads();                      // this buffer complete; every wave is past sample n-2
    if (n + 1 < s1) load(n + 1);
    if (n / B != cg) {
      cg = n / B;
#pragma unroll
      for (int t = 0; t < 2; ++t) { sc[t] = scale[cg * C + 16 * t + r16]; sf[t] = shift[cg * C + 16 * t + r16]; }
    }
    for (int q = wave; q < AP_GROUPS; q += 4) {
      const int rp = q >> 2, cq = q & 3;                       // row pair, 8-column group
      const bf16* xp = xb + 2 * rp * AP_XS + 8 * cq;
      us8 bs;
#pragma unroll
      for (int j = 0; j < 8; ++j) bs[j] = toff[j] >= 0 ? xp[toff[j]] : (unsigned short)0;
      const bf16x8 px = __builtin_bit_cast(bf16x8, bs);
      const int wcol = 4 * cq + g;                             // the lane's window column
      unsigned zw = 0u, cw = 0u;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(px, aw[t], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const uint32_t y01 = pack_bf16x2(acc[0] + bv[t], acc[1] + bv[t]);
        const uint32_t y23 = pack_bf16x2(acc[2] + bv[t], acc[3] + bv[t]);
        const float y[4] = {__uint_as_float(y01 << 16), __uint_as_float(y01 & 0xffff0000u),
                            __uint_as_float(y23 << 16), __uint_as_float(y23 & 0xffff0000u)};
        int v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __float_as_int(fmaf(y[i], sc[t], sf[t]));
        // signed-int order = float order where either side is > 0; max with 0 = the ReLU
        const int mx = max(max(v[0], v[1]), max(v[2], max(v[3], 0)));
        const int a = v[0] == mx ? 1 : v[1] == mx ? 2 : v[2] == mx ? 3 : 4;   // first argmax + 1
        const unsigned nib = mx > 0 ? (unsigned)a : 0u;
        zw |= (pack_bf16x2(__int_as_float(mx), 0.f) & 0xffffu) << (16 * t);
        cw |= nib << (4 * pk + 16 * t);
      }
      // pooled map: lane pairs trade halves so each stores 2 adjacent channels (4 bytes):
      // even r16 -> channels (r16, r16 + 1), odd r16 -> (15 + r16, 16 + r16)
      const unsigned zo = (unsigned)dppi<0xB1>((int)zw);
      const bool ev = (r16 & 1) == 0;
      const unsigned word = ev ? (zw & 0xffffu) | (zo << 16) : (zo >> 16) | (zw & 0xffff0000u);
      // codes: the 4 channels of a word sit in one lane quad
      cw |= (unsigned)dppi<0xB1>((int)cw);
      cw |= (unsigned)dppi<0x4E>((int)cw);
      if (wcol < WP) {
        const size_t win = (size_t)n * NWIN + rp * WP + wcol;
        *reinterpret_cast<unsigned*>(z + win * C + (ev ? r16 : 15 + r16)) = word;
        if (codes && pk < 2) codes[win * 8 + 4 * pk + (r16 >> 2)] = (unsigned short)(cw >> (16 * pk));
      }
    }
  }
}

// BatchNorm partial sums (sum y, sum y^2 of the bf16 y) of the same recomputed conv output, on
// the same pixel-major MFMA: each lane accumulates its channel over its window's 4 pixels in
// registers; the block's 16 lane partials per channel are summed through LDS in fixed order
// into one row of parts [C][G][R][2] (avd_bn_finalize's layout).  Block (group, r) owns a
// contiguous slice of one BN group, so every (group, row) is written exactly once.
__global__ __launch_bounds__(256) void c1r5_stats_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    float* __restrict__ out, int B, int G, int R) {
  __shared__ __attribute__((aligned(16))) bf16 xs[2][AP_XR * AP_XS];
  __shared__ float red[4][4][2][16][2];   // [wave][lane group][t][channel r16][sum, sumsq]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int grp = (int)blockIdx.x / R, rr = (int)blockIdx.x - grp * R;
  const int s0 = grp * B + (int)(((long long)B * rr) / R);
  const int s1 = grp * B + (int)(((long long)B * (rr + 1)) / R);

  bf16x8 aw[2];
  float bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    aw[t] = *reinterpret_cast<const bf16x8*>(wk + (16 * t + r16) * 32 + 8 * g);
    bv[t] = bias ? bias[16 * t + r16] : 0.f;
  }
  const int pk = r16 & 3, pcol = 2 * (r16 >> 2) + (pk & 1), prow = pk >> 1;
  int toff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = 8 * g + j;
    toff[j] = t < KK ? (prow + t / 5) * AP_XS + pcol + t % 5 : -1;
  }
  for (int i = tid; i < 2 * AP_XR * AP_XS / 2; i += 256) reinterpret_cast<unsigned*>(xs)[i] = 0u;
  u4 xv = u4{0u, 0u, 0u, 0u};
  auto load = [&](int n) {
    if (tid < NXV) xv = ldg16(x + (size_t)n * IH * IW + 8 * tid);
  };
  if (s0 < s1) load(s0);
  __syncthreads();
  float sm[2] = {0.f, 0.f}, sq[2] = {0.f, 0.f};
  for (int n = s0; n < s1; ++n) {
    bf16* xb = xs[(n - s0) & 1];
    if (tid < NXV) {
      const unsigned w4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int pix = 8 * tid + 2 * k, r = pix / IW, c = pix - r * IW;
        *reinterpret_cast<unsigned*>(xb + (r + 2) * AP_XS + c + 2) = w4[k];
      }
    }
    __syncthreads();
    if (n + 1 < s1) load(n + 1);
    for (int q = wave; q < AP_GROUPS; q += 4) {
      const int rp = q >> 2, cq = q & 3;
      const bool wv = 4 * cq + g < WP;                         // not virtual columns 28..31
      const bf16* xp = xb + 2 * rp * AP_XS + 8 * cq;
      us8 bs;
#pragma unroll
      for (int j = 0; j < 8; ++j) bs[j] = toff[j] >= 0 ? xp[toff[j]] : (unsigned short)0;
      const bf16x8 px = __builtin_bit_cast(bf16x8, bs);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(px, aw[t], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const uint32_t y01 = pack_bf16x2(acc[0] + bv[t], acc[1] + bv[t]);
        const uint32_t y23 = pack_bf16x2(acc[2] + bv[t], acc[3] + bv[t]);
        const float y0 = __uint_as_float(y01 << 16), y1 = __uint_as_float(y01 & 0xffff0000u);
        const float y2 = __uint_as_float(y23 << 16), y3 = __uint_as_float(y23 & 0xffff0000u);
        if (wv) {   // after the MFMA: the whole wave issues it
          sm[t] += (y0 + y1) + (y2 + y3);
          sq[t] += fmaf(y0, y0, y1 * y1) + fmaf(y2, y2, y3 * y3);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    red[wave][g][t][r16][0] = sm[t];
    red[wave][g][t][r16][1] = sq[t];
  }
  __syncthreads();
  if (tid < 2 * C) {
    const int c = tid >> 1, k = tid & 1, t = c >> 4, ch = c & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) v += red[w][gg][t][ch][k];
    out[(((size_t)c * G + grp) * R + rr) * 2 + k] = v;
  }
}

// BN backward + dW of the layer from the row-summed routed moments m [G][MOMC5], float64:
//   sum dz y = w . M + b sum dz;  sum dz xhat = (sum dz y - mean sum dz) invstd;
//   coef (k1, kx, k0) as avd_bn_bwd_finalize;  dW[c][t] = sum_g k1 M + kx (w Gram + b S) + k0 S;
//   dgamma / dbeta / dbias (= sum dy) summed over the groups.
__global__ __launch_bounds__(256) void c1r5_codes_combine_kernel(
    const float* __restrict__ m, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    long long count, float* __restrict__ dw, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dbias, float* __restrict__ coef, int G) {
  __shared__ double sk[C1R5_GMAX * C][3];
  __shared__ double s12[C1R5_GMAX * C][2];
  const int tid = threadIdx.x;
  const double n = (double)count;
  for (int i = tid; i < G * C; i += 256) {
    const int gq = i / C, c = i - gq * C;
    const float* mg = m + (size_t)gq * MOMC5;
    const double b = bias ? (double)bias[c] : 0.0;
    const double s1 = mg[C * KK + KK * KK + KK + c];
    double sy = b * s1;
    for (int t = 0; t < KK; ++t) sy = fma((double)bf2f(wk[c * 32 + t]), (double)mg[c * KK + t], sy);
    const double mu = mean[gq * C + c], is = invstd[gq * C + c], ga = gamma[c];
    const double s2 = (sy - mu * s1) * is;                   // sum dz * xhat
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
      const float* mg = m + (size_t)gq * MOMC5;
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

int c1r5_rows(int N, int B) {
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, c1r5_moments_win_kernel, 256, 0) !=
            hipSuccess || per <= 0)
      per = 2;
    resident = cus * per;
  }
  const int G = N / B;
  // one resident wave of blocks over the G groups, at least 4 samples per block
  return std::max(1, std::min(grid_cap(resident) / G, B / 4));
}

}  // namespace

extern "C" {

// shape served: Cin 1, Cout 32, 5x5 pad 2 on 28x28, bf16 (the CentralNet image conv1)
int avd_cl_c1r5_codes_rows(int N, int B, int H, int W) {
  if (N <= 0 || B <= 0 || N % B || H != IH || W != IW || N / B > C1R5_GMAX) return 0;
  return c1r5_rows(N, B);
}

int avd_cl_c1r5_codes_cols(void) { return MOMC5; }

// rows per BN group of avd_cl_c1r5_stats (0 = shape not served)
int avd_cl_c1r5_stats_rows(int N, int B, int H, int W) {
  if (N <= 0 || B <= 0 || N % B || H != IH || W != IW) return 0;
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, c1r5_stats_kernel, 256, 0) != hipSuccess ||
        per <= 0)
      per = 2;
    resident = cus * per;
  }
  const int G = N / B;
  return std::max(1, std::min(grid_cap(resident) / G, std::max(1, B / 4)));
}

int avd_cl_c1r5_stats(const void* x, const void* wk, const float* bias, float* out, int N, int B,
                      int H, int W, void* stream) {
  if (!x || !wk || !out) return AVD_ERR_ARG;
  const int R = avd_cl_c1r5_stats_rows(N, B, H, W);
  if (!R) return AVD_ERR_SHAPE;
  const int G = N / B;
  c1r5_stats_kernel<<<G * R, 256, 0, avd_stream(stream)>>>((const bf16*)x, (const bf16*)wk, bias, out,
                                                          B, G, R);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_cl_c1r5_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                            const float* shift, void* z, unsigned short* codes, int N, int B, int H,
                            int W, void* stream) {
  if (!x || !wk || !scale || !shift || !z) return AVD_ERR_ARG;   // codes may be null (no backward)
  if (N <= 0 || B <= 0 || N % B || H != IH || W != IW) return AVD_ERR_SHAPE;
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, c1r5_apply_kernel, 256, 0) != hipSuccess ||
        per <= 0)
      per = 2;
    resident = cus * per;
  }
  const int grid = grid_cap(std::min(N, resident));
  c1r5_apply_kernel<<<grid, 256, 0, avd_stream(stream)>>>((const bf16*)x, (const bf16*)wk, bias, scale,
                                                          shift, (bf16*)z, codes, N, B);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_cl_c1r5_moments_codes(const void* x, const void* gz, const unsigned short* codes, float* out,
                              int N, int B, int H, int W, void* stream) {
  if (!x || !gz || !codes || !out) return AVD_ERR_ARG;
  const int R = avd_cl_c1r5_codes_rows(N, B, H, W);
  if (!R) return AVD_ERR_SHAPE;
  const int G = N / B;
  // the window-space pass (round 4; the dz-map pass it replaced: 90 vs 55 us at N = 7168)
  c1r5_moments_win_kernel<<<G * R, 256, 0, avd_stream(stream)>>>(
      (const bf16*)x, (const bf16*)gz, codes, out, B, G, R);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_cl_c1r5_codes_combine(const float* moments, const void* wk, const float* bias,
                              const float* gamma, const float* mean, const float* invstd,
                              long long count, float* dw, float* dgamma, float* dbeta, float* dbias,
                              float* coef, int G, void* stream) {
  if (!moments || !wk || !gamma || !mean || !invstd || !dw) return AVD_ERR_ARG;
  if (G <= 0 || G > C1R5_GMAX || count <= 1) return AVD_ERR_SHAPE;
  c1r5_codes_combine_kernel<<<1, 256, 0, avd_stream(stream)>>>(moments, (const bf16*)wk, bias, gamma,
                                                               mean, invstd, count, dw, dgamma, dbeta,
                                                               dbias, coef, G);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
