// The 3x3 first layer of the SimCLR / unimodal encoders without a stored conv output:
// Conv2d(1, 32, 3, padding=1) -> BN2d -> ReLU -> MaxPool2d(2) of image_encoder (28x28) and
// audio_encoder (112x112) (dino.py:18-73), bf16, in three passes over the input:
//   * statistics: the per-block patch Gram (9 taps + ones) on MFMAs, turned into the BN partial
//     sums of the EXACT conv output in float64 (c1r3 pass 0's row contract; as the audio
//     conv1's avd_cl_c1_gram) -- c1s3_moments_kernel<W, true>;
//   * BN -> ReLU -> 2x2 max-pool plus the routing codes the backward reads
//     (avd_cl_c1r3_apply_codes) -- c1s3_apply_kernel<W>, PIXEL-major like c1r5.hip's;
//   * the routed backward moments M = sum dz x9, Gram, S, sum dz (avd_cl_c1r3_moments_codes) --
//     c1s3_moments_kernel<W, false>, a GEMM over window-ordered pixels with dz built in registers.
// The recomputing channel-major passes they replace (c1w3.hip c1r3_kernel) took 168 / 549 /
// 540 us at config 4's N = 2048 x 112^2 (profiles/r5w_*).
#include <algorithm>

#include "common.h"

using namespace avd;

namespace {

constexpr int C = 32;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;
typedef __attribute__((ext_vector_type(8))) unsigned short us8;
typedef __attribute__((ext_vector_type(2))) float f2;

template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}

// A register copy the compiler cannot look through: the weights and biases read from global
// memory before the tile loop pass through it, so their vmcnt wait sits before the loop instead of
// at the first MFMA inside it (where a vmcnt(0) would also wait for the next tile's prefetch)
__device__ __forceinline__ unsigned vkeep(unsigned v) {
  unsigned r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v) : "memory");
  return r;
}
__device__ __forceinline__ float vkeepf(float v) { return __uint_as_float(vkeep(__float_as_uint(v))); }

template <int W>
struct Geo {
  static constexpr int H = W;                       // square maps (28^2 image, 112^2 audio)
  static constexpr int WP = W / 2;                  // pooling windows per row
  static constexpr int NGC = (WP + 3) / 4;          // 4-window (16-pixel) groups per row pair
  static constexpr int TR = W <= 32 ? W : 16;       // staged rows per sample of a tile
  static constexpr int SPT = 1;                     // samples per tile
  static constexpr int TPS = H / TR;                // tiles per sample (SPT == 1)
  static constexpr int XO = 8;                      // staged column of pixel 0 (left halo at 7)
  // row stride: the widest read is column 8 NGC (+ XO); 112: 272-B rows (4 banks of skew)
  // (a lane reads columns up to 8 NGC + 2 of a copy)
  static constexpr int XS = W % 8 == 0 ? ((XO + 8 * NGC + 3 + 7) & ~7) + 8 : ((XO + 8 * NGC + 3 + 3) & ~3);
  static constexpr int CP = (TR + 2) * XS;          // one copy of a sample's staged rows
  static constexpr int SR = 2 * CP;                 // the copy and the shifted copy
  static constexpr int BUF = SPT * SR;              // one buffer
  static constexpr int GPT = SPT * (TR / 2) * NGC;  // groups per tile
  // 16-byte vectors of one tile: W % 8 == 0: (TR + 2) rows x W / 8 (halo rows included);
  // else SPT whole samples (the halo rows stay zero)
  static constexpr int NV = W % 8 == 0 ? (TR + 2) * (W / 8) : SPT * (H * W / 8);
  static_assert(NV <= 256, "one staging vector per thread");
  static_assert(NGC >= 4, "one carry per group step");
  static_assert(W % 8 == 0 ? TR * TPS == H : TR == H, "tiles cover the sample");
};

// BN -> ReLU -> 2x2 max-pool of the recomputed conv output plus the routing codes:
//   * A = the im2col fragment of 16 pixels ordered window by window (pixel p = 4 w + k, k = (0,0)
//     (0,1) (1,0) (1,1)), B = the weights of 16 channels, so D lane l holds ONE whole pooling
//     window of one channel: max, first argmax and the > 0 test are in-lane integer compares of
//     the f32 bn(y) bits, and y is the same bf16(acc + b) as the stored-y conv's (bit-identical
//     pooled map, tests/test_gpu_c1r3_codes.py);
//   * k = tap (0..8, the stored-y conv's order: lane group 0 holds taps 0..7, group 1 tap 8, and
//     the k slots >= 9 meet zero weights).  A layout with filter row ty in lane group ty gave a
//     pooled map that differs from the stored-y chain's at N = 2048: the MFMA's sum of the nine
//     products depends on their k slots;
//   * the staged rows are kept twice, the second copy shifted right by one pixel, so a lane's 3x3
//     patch row (columns c - 1 .. c + 1) starts on a dword in one of them: 3 dword-pair reads per
//     lane and group instead of 8 two-byte gathers;
//   * tiles: TR staged rows (+ 2 halo rows) of SPT samples, register-prefetched one tile ahead,
//     one barrier per tile; pooled map stores are 4 bytes per lane (lane pairs trade channel
//     halves), codes 2 bytes per lane (one quad of channels).
template <int W>
__global__ __launch_bounds__(256) void c1s3_apply_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, bf16* __restrict__ z,
    unsigned short* __restrict__ codes, int N, int B) {
  using Gm = Geo<W>;
  constexpr int XS = Gm::XS, TR = Gm::TR, SPT = Gm::SPT, WP = Gm::WP, NGC = Gm::NGC;
  __shared__ __attribute__((aligned(16))) bf16 xs[2 * Gm::BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  // tiles: SPT samples x TR rows; a block takes a contiguous share of them
  const int tps = SPT == 1 ? Gm::TPS : 1;
  const int nt = (N + SPT - 1) / SPT * tps;
  const int per = nt / (int)gridDim.x, extra = nt % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);

  // B operand: lane (channel 16 t + r16, k = 8 g + j) = w[c][8 g + j] (taps >= 9 are zero in wk)
  bf16x8 aw[2];
  float bv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const u4 wv = *reinterpret_cast<const u4*>(wk + (16 * t + r16) * 32 + 8 * g);
    aw[t] = __builtin_bit_cast(bf16x8, u4{vkeep(wv.x), vkeep(wv.y), vkeep(wv.z), vkeep(wv.w)});
    bv[t] = vkeepf(bias ? bias[16 * t + r16] : 0.f);
  }
  // A operand: lane (pixel r16 of a group = window r16 / 4, position r16 % 4; taps 8 g + j):
  // patch rows read from the copy where column pcol - 1 sits on a dword (odd pcol: the copy,
  // even: the shifted copy, whose column j + 1 holds pixel j)
  const int pk = r16 & 3, pcol = 2 * (r16 >> 2) + (pk & 1), prow = pk >> 1;
  const int aoff = prow * XS + ((pk & 1) ? Gm::XO + pcol - 1 : Gm::CP + Gm::XO + pcol);

  for (int i = tid; i < Gm::BUF; i += 256) reinterpret_cast<unsigned*>(xs)[i] = 0u;   // both buffers
  static_assert(Gm::XO % 2 == 0 && XS % 2 == 0 && Gm::CP % 2 == 0, "dword-aligned patch rows");

  // every thread loads (threads past the tile's vectors re-read the last one) and the halo rows /
  // samples past N become zeros only at put(): no branch around the load, so the compiler's
  // vmcnt accounting is the same on every path
  u4 xv = u4{0u, 0u, 0u, 0u};
  bool xok = false;
  auto load = [&](int tl) {
    const int e = min(tid, Gm::NV - 1);
    if constexpr (W % 8 == 0) {
      const int n = tl / tps, y0 = (tl - n * tps) * TR;
      const int r = e / (W / 8), cc = e - r * (W / 8), iy = y0 - 1 + r;
      xok = (unsigned)iy < (unsigned)W;
      xv = ldg16(x + ((size_t)n * W + min(max(iy, 0), W - 1)) * W + 8 * cc);
    } else {
      const int n = tl * SPT + e / (W * W / 8);
      xok = n < N;
      xv = ldg16(x + ((size_t)min(n, N - 1) * W * W + 8 * (e % (W * W / 8))));
    }
  };
  auto put = [&](bf16* xb) {
    if (tid < Gm::NV) {
      if (!xok) xv = u4{0u, 0u, 0u, 0u};
      if constexpr (W % 8 == 0) {
        const int r = tid / (W / 8), cc = tid - r * (W / 8);
        bf16* d = xb + r * XS + Gm::XO + 8 * cc;
        *reinterpret_cast<u4*>(d) = xv;
        // the shifted copy: pixels 8 cc .. 8 cc + 7 at columns + 1 (two halves + three dwords)
        bf16* e = d + Gm::CP + 1;
        e[0] = (bf16)(xv.x & 0xffffu);
        *reinterpret_cast<unsigned*>(e + 1) = __builtin_amdgcn_alignbit(xv.y, xv.x, 16);
        *reinterpret_cast<unsigned*>(e + 3) = __builtin_amdgcn_alignbit(xv.z, xv.y, 16);
        *reinterpret_cast<unsigned*>(e + 5) = __builtin_amdgcn_alignbit(xv.w, xv.z, 16);
        e[7] = (bf16)(xv.w >> 16);
      } else {
        const int s = tid / (W * W / 8), e = tid - s * (W * W / 8);
        const unsigned w4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {           // a pixel pair never straddles a row (W even)
          const int pix = 8 * e + 2 * k, r = pix / W, c = pix - r * W;
          bf16* d = xb + s * Gm::SR + (r + 1) * XS + Gm::XO + c;
          *reinterpret_cast<unsigned*>(d) = w4[k];
          d[Gm::CP + 1] = (bf16)(w4[k] & 0xffffu);
          d[Gm::CP + 2] = (bf16)(w4[k] >> 16);
        }
      }
    }
  };
  if (t0 < t1) load(t0);
  __syncthreads();                                  // zeroed
  if (t0 < t1) put(xs);

  float sc[SPT][2] = {}, sf[SPT][2] = {};
  int cgs[SPT];
#pragma unroll
  for (int s = 0; s < SPT; ++s) cgs[s] = -1;
  for (int ti = t0; ti < t1; ++ti) {
    const bf16* xb = xs + ((ti - t0) & 1) * Gm::BUF;
    __syncthreads();                                // this buffer complete; the other one free
    const int n0 = ti / tps * SPT, y0 = (ti - ti / tps * tps) * TR;
    // BN coefficients of the tile's samples, re-read only when the BN group changes and waited
    // for right there (vkeepf): no load but the prefetch is outstanding in the group loop
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int cg = min(n0 + s, N - 1) / B;
      if (cg != cgs[s]) {
        cgs[s] = cg;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          sc[s][t] = vkeepf(scale[cg * C + 16 * t + r16]);
          sf[s][t] = vkeepf(shift[cg * C + 16 * t + r16]);
        }
      }
    }
    // in flight under this tile's MFMAs; issued on the last tile too (its own tile again), so
    // every path has the same loads outstanding and the coefficients' wait leaves it in flight
    load(min(ti + 1, t1 - 1));
    // the tile's first window; group (s, rp, cq) advanced by 4 with one carry per step
    bf16* zt = z + ((size_t)n0 * (W / 2) + y0 / 2) * WP * C;
    unsigned short* ct = codes ? codes + ((size_t)n0 * (W / 2) + y0 / 2) * WP * 8 : nullptr;
    int cq = wave, rp = 0, s = 0;                   // NGC >= 4: at most one carry per step
    for (int q = wave; q < Gm::GPT; q += 4) {
      // patch rows 0..2: (c - 1, c), (c + 1, c + 2) of each
      const int sm = SPT == 1 ? 0 : s;                        // the tile's sample (SPT 1: always 0)
      const unsigned* pr = reinterpret_cast<const unsigned*>(xb + sm * Gm::SR + 2 * rp * XS + 8 * cq + aoff);
      const unsigned d00 = pr[0], d01 = pr[1], d10 = pr[XS / 2], d11 = pr[XS / 2 + 1];
      const unsigned d20 = pr[XS], d21 = pr[XS + 1];
      // k 0..7 = taps (0,0) (0,1) | (0,2) (1,0) | (1,1) (1,2) | (2,0) (2,1); lane groups >= 1:
      // k 8 = tap (2,2) (and k 9..15 meet zero weights)
      const u4 av = u4{g == 0 ? d00 : d21, __builtin_amdgcn_perm(d10, d01, 0x05040100u),
                       __builtin_amdgcn_alignbit(d11, d10, 16), d20};
      const bf16x8 px = __builtin_bit_cast(bf16x8, av);
      const int wcol = 4 * cq + g;                            // the lane's window column
      // every window is real at 112^2 (4 NGC == WP) and every tile sample is < N with SPT 1
      const bool live = (4 * NGC == WP || wcol < WP) && (SPT == 1 || n0 + sm < N);
      const unsigned win = (unsigned)((sm * (W / 2) + rp) * WP + wcol);   // from the tile's first window
      unsigned zw = 0u, cw = 0u;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(px, aw[t], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        // y = bf16(acc + b) and bn(y) on packed pairs (the same IEEE operations per element)
        const f2 b2 = f2{bv[t], bv[t]}, sc2 = f2{sc[sm][t], sc[sm][t]}, sf2 = f2{sf[sm][t], sf[sm][t]};
        const f2 a01 = f2{acc[0], acc[1]} + b2, a23 = f2{acc[2], acc[3]} + b2;
        const uint32_t y01 = pack_bf16x2(a01.x, a01.y), y23 = pack_bf16x2(a23.x, a23.y);
        const f2 v01 = __builtin_elementwise_fma(f2{__uint_as_float(y01 << 16), __uint_as_float(y01 & 0xffff0000u)}, sc2, sf2);
        const f2 v23 = __builtin_elementwise_fma(f2{__uint_as_float(y23 << 16), __uint_as_float(y23 & 0xffff0000u)}, sc2, sf2);
        const int v[4] = {__float_as_int(v01.x), __float_as_int(v01.y), __float_as_int(v23.x), __float_as_int(v23.y)};
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
      // codes: the 4 channels of a u16 sit in one lane quad
      cw |= (unsigned)dppi<0xB1>((int)cw);
      cw |= (unsigned)dppi<0x4E>((int)cw);
      if (live) {
        // 32-bit element offsets from the tile's (uniform) base pointers
        *reinterpret_cast<unsigned*>(zt + (win * C + (unsigned)(ev ? r16 : 15 + r16))) = word;
        if (ct && pk < 2) ct[win * 8u + (unsigned)(4 * pk + (r16 >> 2))] = (unsigned short)(cw >> (16 * pk));
      }
      cq += 4;
      if (cq >= NGC) {
        cq -= NGC;
        if (++rp == TR / 2) { rp = 0; ++s; }
      }
    }
    if (ti + 1 < t1) put(xs + ((ti + 1 - t0) & 1) * Gm::BUF);
  }
}

// ---------------------------------------------------------------------------- routed moments
// The backward of conv1 + bn1 from the forward's routing codes (c1r3 pass 5's contract: one row of
// MOMR = M [32][9] | Gram [9][9] | S [9] | sum dz [32] per (block row, group), reduced with
// avd_sum_rows, then avd_cl_c1r3_codes_combine) as a GEMM over pixels in window order, a k-step
// = 8 window slots x 4 positions of one window row:
//   A (channels x pixels) = dz: the pooled gradient at the coded position of each window, 0 at
//     the other three, built in registers from gz and the codes (no dz map);
//   B (pixels x taps) = the im2col column of tap r16 (r16 = 9: ones -> sum dz and S), one dword
//     per window and row from the staged copy where the pixel pair starts on a dword;
//   M += A B (two channel tiles), Gram += B^T B (the B fragment is its own transpose's A).
// Tiles of 224 window slots (28 k-steps, 7 per wave) staged from registers prefetched one tile
// ahead: 112^2: 8 rows (4 window rows x 56 windows); 28^2: one sample (14 window rows x 16
// slots, slots 14 and 15 padding: zero gz / codes, B masked).
template <int W>
struct MGeo {
  static constexpr int WP = W / 2;
  static constexpr int TRM = W <= 32 ? W : 8;                   // rows per tile
  static constexpr int TPS = W / TRM;                           // tiles per sample
  static constexpr int WSL = W <= 32 ? 16 : WP;                 // window slots per window row
  static constexpr int KPR = WSL / 8;                           // k-steps per window row
  static constexpr int NSL = (TRM / 2) * WSL;                   // slots per tile
  static constexpr int NWIN = (TRM / 2) * WP;                   // windows per tile
  static constexpr int XO = 8;
  static constexpr int XS = W % 8 == 0 ? ((XO + W + 3 + 7) & ~7) + 8 : ((XO + 2 * WSL + 3 + 3) & ~3);
  static constexpr int CP = (TRM + 2) * XS;                     // the shifted copy
  // x vectors: W % 8 == 0: (TRM + 2) rows x W / 8 (halo rows included); else the sample
  static constexpr int NX = W % 8 == 0 ? (TRM + 2) * (W / 8) : W * W / 8;
  static constexpr int NG = NWIN * C / 8;                       // gz vectors
  static constexpr int L_GZ = 2 * CP, L_CD = L_GZ + NSL * 40, L_END = L_CD + NSL * 8;   // bf16 units
  static_assert(NSL == 224 && NX <= 256 && NG <= 1024 && NWIN <= 256, "staging shape");
  static_assert(L_GZ % 8 == 0 && L_CD % 8 == 0 && XS % 2 == 0 && CP % 2 == 0, "aligned regions");
};
constexpr int GZS = 40;                                         // window slot stride of the gz tile (80 B)
constexpr int MOMR = C * 9 + 81 + 9 + C;
constexpr int M_RED = 4 * 3 * 64 * 4 + 100;                     // epilogue floats [wave][tile][lane][4] + [10][10]

template <int W, bool GRAM>
__global__ __launch_bounds__(256) void c1s3_moments_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ gz, const unsigned short* __restrict__ codes,
    const bf16* __restrict__ wk, const float* __restrict__ bias, float* __restrict__ out, int B, int G, int R) {
  using Mg = MGeo<W>;
  constexpr int XS = Mg::XS, WP = Mg::WP;
  constexpr int LEND = GRAM ? Mg::L_GZ : Mg::L_END;            // the statistics pass stages x only
  constexpr int LDSB = LEND * 2 > M_RED * 4 ? LEND * 2 : M_RED * 4;
  __shared__ __attribute__((aligned(16))) char lds[LDSB];
  bf16* sm = reinterpret_cast<bf16*>(lds);
  const unsigned short* gzs = reinterpret_cast<const unsigned short*>(sm + Mg::L_GZ);
  const unsigned short* cds = reinterpret_cast<const unsigned short*>(sm + Mg::L_CD);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int grp = (int)blockIdx.x / R, rr = (int)blockIdx.x - grp * R;
  const int tg = B * Mg::TPS;                                   // tiles per group
  const int t0 = grp * tg + (int)(((long long)tg * rr) / R);
  const int t1 = grp * tg + (int)(((long long)tg * (rr + 1)) / R);

  // B operand: lane (tap r16 = (ty, tx)): the pixel pair (2 wc + tx - 1, 2 wc + tx) of staged
  // row 2 hr + py + ty, from the copy (tx = 1) or the shifted copy (tx = 0, 2); lanes 9..15
  // read tap 4's and take ones (9) / zeros
  const int tb = r16 < 9 ? r16 : 4, ty = tb / 3, tx = tb - 3 * ty;
  const int boff = ty * XS + (tx == 1 ? Mg::XO : Mg::CP + Mg::XO + tx);
  const unsigned bconst = r16 == 9 ? 0x3F803F80u : 0u;          // bf16 (1, 1)
  f4 macc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}}, gacc = f4{0.f, 0.f, 0.f, 0.f};

  // halos, and (28^2) the padding window slots of the gz / codes tiles: zero once
  for (int i = tid; i < LEND / 2; i += 256) reinterpret_cast<unsigned*>(sm)[i] = 0u;

  u4 xv = u4{0u, 0u, 0u, 0u}, cv = u4{0u, 0u, 0u, 0u}, gv[4];
  bool xok = false;
  // every thread loads (clamped indices: the compiler's vmcnt accounting is the same on every
  // path); halo rows become zeros at put()
  auto load = [&](int tl) {
    const int n = tl / Mg::TPS, y0 = (tl - n * Mg::TPS) * Mg::TRM;
    const int e = min(tid, Mg::NX - 1);
    if constexpr (W % 8 == 0) {
      const int r = e / (W / 8), cc = e - r * (W / 8), iy = y0 - 1 + r;
      xok = (unsigned)iy < (unsigned)W;
      xv = ldg16(x + ((size_t)n * W + min(max(iy, 0), W - 1)) * W + 8 * cc);
    } else {
      xok = true;
      xv = ldg16(x + (size_t)n * W * W + 8 * e);
    }
    if constexpr (!GRAM) {
      const size_t w0 = (size_t)n * WP * WP + (size_t)(y0 / 2) * WP;    // the tile's first window
#pragma unroll
      for (int j = 0; j < 4; ++j) gv[j] = ldg16(gz + w0 * C + 8 * min(tid + 256 * j, Mg::NG - 1));
      cv = ldg16(codes + (w0 + min(tid, Mg::NWIN - 1)) * 8);
    }
  };
  auto slot = [&](int w) { return W % 8 == 0 ? w : (w / WP) * Mg::WSL + (w - (w / WP) * WP); };
  auto put = [&]() {
    if (tid < Mg::NX) {
      if (!xok) xv = u4{0u, 0u, 0u, 0u};
      if constexpr (W % 8 == 0) {
        const int r = tid / (W / 8), cc = tid - r * (W / 8);
        bf16* d = sm + r * XS + Mg::XO + 8 * cc;
        *reinterpret_cast<u4*>(d) = xv;
        bf16* e = d + Mg::CP + 1;                               // the shifted copy
        e[0] = (bf16)(xv.x & 0xffffu);
        *reinterpret_cast<unsigned*>(e + 1) = __builtin_amdgcn_alignbit(xv.y, xv.x, 16);
        *reinterpret_cast<unsigned*>(e + 3) = __builtin_amdgcn_alignbit(xv.z, xv.y, 16);
        *reinterpret_cast<unsigned*>(e + 5) = __builtin_amdgcn_alignbit(xv.w, xv.z, 16);
        e[7] = (bf16)(xv.w >> 16);
      } else {
        const unsigned w4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {           // a pixel pair never straddles a row (W even)
          const int pix = 8 * tid + 2 * k, r = pix / W, c = pix - r * W;
          bf16* d = sm + (r + 1) * XS + Mg::XO + c;
          *reinterpret_cast<unsigned*>(d) = w4[k];
          d[Mg::CP + 1] = (bf16)(w4[k] & 0xffffu);
          d[Mg::CP + 2] = (bf16)(w4[k] >> 16);
        }
      }
    }
    if constexpr (!GRAM) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + 256 * j;
        if (e < Mg::NG) *reinterpret_cast<u4*>(sm + Mg::L_GZ + slot(e >> 2) * GZS + 8 * (e & 3)) = gv[j];
      }
      if (tid < Mg::NWIN) *reinterpret_cast<u4*>(sm + Mg::L_CD + 8 * slot(tid)) = cv;
    }
  };

  if (t0 < t1) load(t0);
  for (int ti = t0; ti < t1; ++ti) {
    __syncthreads();                    // the previous tile's k-steps are done with the LDS tile
    put();
    __syncthreads();
    load(min(ti + 1, t1 - 1));          // in flight under this tile's k-steps
    for (int j = wave; j < Mg::NSL / 8; j += 4) {
      const int hr = j / Mg::KPR, wc0 = 8 * (j - hr * Mg::KPR);
      // B: windows 2 g, 2 g + 1 of the k-step, rows py = 0, 1 (window 2 g + 1: one dword on)
      const unsigned* bp = reinterpret_cast<const unsigned*>(sm + 2 * hr * XS + 2 * (wc0 + 2 * g) + boff);
      u4 bv = u4{bp[0], bp[XS / 2], bp[1], bp[1 + XS / 2]};
      if (r16 >= 9) bv = u4{bconst, bconst, bconst, bconst};
      if constexpr (W % 8 != 0) {                               // padding slots: no pixels
        if (wc0 + 2 * g >= WP) bv.x = bv.y = 0u;
        if (wc0 + 2 * g + 1 >= WP) bv.z = bv.w = 0u;
      }
      const bf16x8 bx = __builtin_bit_cast(bf16x8, bv);
      const int w = hr * Mg::WSL + wc0 + 2 * g;                 // the lane's first window slot
#pragma unroll
      for (int ct = 0; ct < (GRAM ? 0 : 2); ++ct) {
        const int c = 16 * ct + r16;
        unsigned av[4];
#pragma unroll
        for (int wi = 0; wi < 2; ++wi) {
          const unsigned a = gzs[(w + wi) * GZS + c];
          const unsigned nib = (cds[(w + wi) * 8 + (c >> 2)] >> (4 * (c & 3))) & 0xFu;
          const unsigned v = (nib & 1u) ? a : a << 16;          // position 1, 3: low half; 2, 4: high
          av[2 * wi] = (nib - 1u) < 2u ? v : 0u;
          av[2 * wi + 1] = (nib - 3u) < 2u ? v : 0u;
        }
        const bf16x8 ax = __builtin_bit_cast(bf16x8, u4{av[0], av[1], av[2], av[3]});
        macc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax, bx, macc[ct], 0, 0, 0);
      }
      gacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx, bx, gacc, 0, 0, 0);
    }
  }
  // block row: the four waves' tiles summed in fixed order
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[((wave * 3 + 0) * 64 + lane) * 4 + i] = macc[0][i];
    red[((wave * 3 + 1) * 64 + lane) * 4 + i] = macc[1][i];
    red[((wave * 3 + 2) * 64 + lane) * 4 + i] = gacc[i];
  }
  __syncthreads();
  // D lane (g, r16) register i: row 4 g + i (channel within the tile / tap), column r16 (tap)
  auto at = [&](int tile, int row, int col) {
    const int l = (row >> 2) * 16 + col, i = row & 3;
    float v = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) v += red[((wv * 3 + tile) * 64 + l) * 4 + i];
    return v;
  };
  if constexpr (GRAM) {
    // BN partial sums of the exact conv output y = w . x9 + b from the block's patch Gram, in
    // float64: sum y = w . S + n b, sum y^2 = w' Gram w + 2 b w . S + n b^2 (n = the ones' count);
    // rows [C][G][R][2] (avd_bn_finalize's layout, c1r3 pass 0's contract)
    float* g10 = red + 4 * 3 * 64 * 4;                          // [10][10] after the wave tiles
    if (tid < 100) g10[tid] = at(2, tid / 10, tid % 10);
    __syncthreads();
    if (tid < C) {
      double ws = 0.0, wgw = 0.0;
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
        const double wt = (double)bf2f(wk[tid * 32 + t]);
        ws += wt * (double)g10[t * 10 + 9];
        double r = 0.0;
#pragma unroll 1
        for (int u = 0; u < 9; ++u) r += (double)bf2f(wk[tid * 32 + u]) * (double)g10[t * 10 + u];
        wgw += wt * r;
      }
      const double n = (double)g10[99], b = bias ? (double)bias[tid] : 0.0;
      float* o = out + (((size_t)tid * G + grp) * R + rr) * 2;
      o[0] = (float)(ws + n * b);
      o[1] = (float)(wgw + 2.0 * b * ws + n * b * b);
    }
    return;
  }
  float* o = out + ((size_t)rr * G + grp) * MOMR;
  for (int e = tid; e < MOMR; e += 256) {
    float v;
    if (e < C * 9) {
      const int c = e / 9, t = e - 9 * c;
      v = at(c >> 4, c & 15, t);
    } else if (e < C * 9 + 81) {
      const int q = e - C * 9, t1 = q / 9, t2 = q - 9 * t1;
      v = at(2, t1, t2);
    } else if (e < C * 9 + 90) {
      v = at(2, e - C * 9 - 81, 9);                             // S: the ones column
    } else {
      const int c = e - (C * 9 + 90);
      v = at(c >> 4, c & 15, 9);                                // sum dz
    }
    o[e] = v;
  }
}

template <typename Kern>
int resident_blocks(Kern k) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, 0) != hipSuccess || per <= 0) per = 2;
  return cus * per;
}

}  // namespace

namespace avd {

// shapes served: Cin 1, Cout 32, 3x3 pad 1, square 28^2 or 112^2 maps, bf16
bool c1s3_serves(int N, int B, int H, int W, int Cout) {
  if (Cout != C || H != W || N <= 0 || B <= 0 || N % B) return false;
  return W == 28 || W == 112;
}

// rows per BN group of the statistics pass (c1r3 pass 0's contract): the patch-Gram pass
int c1s3_stats_rows(int N, int B, int W) {
  static int res28 = 0, res112 = 0;
  int& res = W == 28 ? res28 : res112;
  if (!res) res = W == 28 ? resident_blocks(c1s3_moments_kernel<28, true>) : resident_blocks(c1s3_moments_kernel<112, true>);
  const int G = N / B, tg = B * (W == 28 ? MGeo<28>::TPS : MGeo<112>::TPS);
  return std::max(1, std::min(grid_cap(res) / G, std::max(1, tg / 4)));
}

int c1s3_stats(const void* x, const void* wk, const float* bias, float* out, int N, int B, int W,
               hipStream_t st) {
  const int R = c1s3_stats_rows(N, B, W), G = N / B;
  if (W == 28)
    c1s3_moments_kernel<28, true><<<G * R, 256, 0, st>>>((const bf16*)x, nullptr, nullptr, (const bf16*)wk, bias,
                                                         out, B, G, R);
  else
    c1s3_moments_kernel<112, true><<<G * R, 256, 0, st>>>((const bf16*)x, nullptr, nullptr, (const bf16*)wk,
                                                          bias, out, B, G, R);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// the routed moments pass at 28^2 / 112^2 (rows per BN group; 0: not served)
int c1s3_moments_rows(int N, int B, int H, int W, int Cout) {
  if (Cout != C || H != W || (W != 28 && W != 112) || N <= 0 || B <= 0 || N % B) return 0;
  static int res28 = 0, res112 = 0;
  int& res = W == 28 ? res28 : res112;
  if (!res)
    res = W == 28 ? resident_blocks(c1s3_moments_kernel<28, false>) : resident_blocks(c1s3_moments_kernel<112, false>);
  const int G = N / B, tg = B * (W == 28 ? MGeo<28>::TPS : MGeo<112>::TPS);
  return std::max(1, std::min(grid_cap(res) / G, std::max(1, tg / 4)));
}

int c1s3_moments(const void* x, const void* gz, const unsigned short* codes, float* out, int N, int B,
                 int W, hipStream_t st) {
  const int R = c1s3_moments_rows(N, B, W, W, C), G = N / B;
  if (W == 28)
    c1s3_moments_kernel<28, false><<<G * R, 256, 0, st>>>((const bf16*)x, (const bf16*)gz, codes, nullptr, nullptr,
                                                          out, B, G, R);
  else
    c1s3_moments_kernel<112, false><<<G * R, 256, 0, st>>>((const bf16*)x, (const bf16*)gz, codes, nullptr,
                                                           nullptr, out, B, G, R);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int c1s3_apply_codes(const void* x, const void* wk, const float* bias, const float* scale,
                     const float* shift, void* z, unsigned short* codes, int N, int B, int W,
                     hipStream_t st) {
  static int res28 = 0, res112 = 0;
  int& res = W == 28 ? res28 : res112;
  if (!res) res = W == 28 ? resident_blocks(c1s3_apply_kernel<28>) : resident_blocks(c1s3_apply_kernel<112>);
  const int tiles = N * (W == 28 ? Geo<28>::TPS : Geo<112>::TPS);
  const int grid = grid_cap(std::min(tiles, res));
  if (W == 28)
    c1s3_apply_kernel<28><<<grid, 256, 0, st>>>((const bf16*)x, (const bf16*)wk, bias, scale, shift,
                                                (bf16*)z, codes, N, B);
  else
    c1s3_apply_kernel<112><<<grid, 256, 0, st>>>((const bf16*)x, (const bf16*)wk, bias, scale, shift,
                                                 (bf16*)z, codes, N, B);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // namespace avd
