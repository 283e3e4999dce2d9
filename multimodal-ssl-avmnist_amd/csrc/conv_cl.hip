// Channels-last (NHWC) convolution on MFMA, bf16 (v_mfma_f32_16x16x32_bf16) and f32
// (v_mfma_f32_16x16x4f32, exact f32 products: the parity mode) from one template.
// Layers: CentralUnimodalImage / CentralUnimodalAudio convs (unimodal.py:105-221), the 3x3
// CNN encoders (dino.py:18-73).  Activations are [N][H][W][C].
//
// Forward / input-gradient (conv_cl_kernel), an implicit GEMM with
//   M = output channels (A = weights, pre-laid [O][tap*C + c]),
//   N = 16 output pixels per MFMA column block, taken from a flattened pixel list of the
//       block's tile (TH x TW of one sample, or NS whole small maps), GPW 16-pixel groups per
//       wave,
//   K = (tap, input channel), channel fastest; the input tile + halo sits channels-last in LDS
//       so a B fragment (KL consecutive channels of one pixel and tap) is one LDS read.
// The C fragment gives each lane 4 consecutive channels of one pixel: 8-byte (bf16) / 16-byte
// (f32) NHWC stores.  The forward epilogue adds the bias, rounds to the storage type and emits
// the BatchNorm partial (sum, sumsq) of the stored values per (channel, block).
// First layers (Cin = 1) use conv_c1_kernel: K = the K*K taps (padded), the B fragment
// gathered tap by tap from the single-channel LDS tile.
#include <algorithm>
#include <cmath>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

template <typename T> struct CL;
template <> struct CL<bf16> {
  static constexpr int KL = 8;   // k elements per lane per MFMA
  typedef bf16x8 F;
  static __device__ __forceinline__ F ld(const bf16* p) { return *reinterpret_cast<const F*>(p); }
  static __device__ __forceinline__ F zero() { return __builtin_bit_cast(F, u4{0u, 0u, 0u, 0u}); }
};
template <> struct CL<float> {
  static constexpr int KL = 1;
  typedef float F;
  static __device__ __forceinline__ F ld(const float* p) { return *p; }
  static __device__ __forceinline__ F zero() { return 0.f; }
};

// input channels per LDS chunk and the LDS pixel stride (elements): bf16 strides are odd
// multiples of 16 B (conflict-free ds_read_b128 across 16 pixels), f32 strides odd in dwords.
template <typename T, int CIN>
struct Chunk {
  static constexpr int CC = CIN < 32 ? CIN : 32;
  static constexpr int PS = sizeof(T) == 2 ? (CC == 8 ? 8 : CC + 8) : CC + 1;
};
constexpr int LDS_CAP = 64 * 1024;

__device__ __forceinline__ f4 mma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 4 consecutive channels of one pixel (the bf16 store is inlined in conv_store)
__device__ __forceinline__ void store4(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

// Output-pixel geometry of a block: tile (ty0, tx0) of TH x TW in NS samples starting at n0.
struct Tile {
  int n0, ty0, tx0, TH, TW, NS, ITH, ITW;
};

// tile index ti = sample-group * tilesPS + tile-in-sample (also the BN partial row)
__device__ __forceinline__ Tile tile_of(int ti, int tilesPS, int TH, int TW, int NS, int tilesX,
                                        int K) {
  Tile t;
  const int sg = ti / tilesPS, tile = ti - sg * tilesPS;
  t.n0 = sg * NS;
  t.ty0 = (tile / tilesX) * TH;
  t.tx0 = (tile % tilesX) * TW;
  t.TH = TH; t.TW = TW; t.NS = NS;
  t.ITH = TH + K - 1; t.ITW = TW + K - 1;
  return t;
}

// Epilogue of one batch of GPW 16-pixel groups (first group index grp0 of this wave):
// bias, rounding to T, NHWC store, and the BN partial sums of the stored values.
//   acc[j][t]: lane holds C[co = co0 + 16t + 4g + i][pixel r16 of group grp0 + j].
template <typename T, int NT, int GPW>
__device__ __forceinline__ void conv_store(const f4 (&acc)[GPW][NT], const Tile& tl, int grp0,
                                           const FastDiv& fHW, const FastDiv& fTW, int N, int Ho,
                                           int Wo, int Cout, int co0,
                                           const float* __restrict__ bias, T* __restrict__ y,
                                           float (&ss)[NT][4], float (&sq)[NT][4]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
  // bias loaded once, unconditionally (a load inside the per-pixel branch below would cost a
  // full memory round trip per group)
  float bv[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int cob = min(co0 + 16 * t + 4 * g, Cout - 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[t][i] = bias ? bias[cob + i] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int p = (grp0 + j) * 16 + r16;
    const int s = fHW.div(p), rem = p - s * fHW.d;
    const int ry = fTW.div(rem);
    const int oy = tl.ty0 + ry, ox = tl.tx0 + rem - ry * fTW.d;
    const int n = tl.n0 + s;
    const bool pv = s < tl.NS && n < N && oy < Ho && ox < Wo;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int cob = co0 + 16 * t + 4 * g;
      if (!pv || cob >= Cout) continue;
      if constexpr (sizeof(T) == 2) {
        // one v_cvt_pk_bf16_f32 per pair; the statistics are taken on the stored (rounded)
        // values, recovered from the packed bits
        const uint32_t lo = pack_bf16x2(acc[j][t][0] + bv[t][0], acc[j][t][1] + bv[t][1]);
        const uint32_t hi = pack_bf16x2(acc[j][t][2] + bv[t][2], acc[j][t][3] + bv[t][3]);
        const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                            __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ss[t][i] += v[i];
          sq[t][i] = fmaf(v[i], v[i], sq[t][i]);
        }
        *reinterpret_cast<uint2*>(y + (((size_t)n * Ho + oy) * Wo + ox) * Cout + cob) =
            make_uint2(lo, hi);
      } else {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[j][t][i] + bv[t][i];
          ss[t][i] += v[i];
          sq[t][i] += v[i] * v[i];
        }
        store4(y + (((size_t)n * Ho + oy) * Wo + ox) * Cout + cob, v);
      }
    }
  }
}

// Per-wave BN partial row: stats[co][row][2], row = tile * 4 + wave (no block barrier).
template <int NT>
__device__ __forceinline__ void conv_stats(float (&ss)[NT][4], float (&sq)[NT][4], int Cout,
                                           int co0, float* __restrict__ stats, int nrows, int row) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = ss[t][i], q = sq[t][i];
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        a += __shfl_xor(a, m, 64);
        q += __shfl_xor(q, m, 64);
      }
      const int co = co0 + 16 * t + 4 * g + i;
      if (r16 == 0 && co < Cout) {
        stats[((size_t)co * nrows + row) * 2] = a;
        stats[((size_t)co * nrows + row) * 2 + 1] = q;
      }
    }
}

// One block = one tile (TH x TW of one sample, or NS whole small maps) x NT*16 output
// channels.  Each wave walks NB batches of GPW 16-pixel groups (batch b of wave w = groups
// (b*4 + w)*GPW ...), storing each batch before the next: registers stay at one batch while the
// tile -- and so the work per staging round trip -- grows with NB.  Input channel chunks of CC
// are staged in turn when CIN > CC (then NB = 1).  Staging loads are unconditional from clamped
// addresses followed by a select (a branch around each load makes hipcc wait vmcnt(0) per
// element).
// --------------------------------------------------------------------------- Cin >= 8
template <typename T, int K, int CIN, int NT, int GPW>
__global__ __launch_bounds__(256) void conv_cl_kernel(
    const T* __restrict__ x, const T* __restrict__ wk, const float* __restrict__ bias,
    T* __restrict__ y, float* __restrict__ stats, int N, int H, int W, int Cout, int Ho, int Wo,
    int pad, int TH, int TW, int NS, int tilesX, int tilesPS, int total, int Kpad, int NB) {
  constexpr int KL = CL<T>::KL;
  constexpr int CC = Chunk<T, CIN>::CC;       // input channels per LDS chunk
  constexpr int PS = Chunk<T, CIN>::PS;       // LDS pixel stride
  constexpr int NCH = CIN / CC;
  constexpr int VE = 16 / sizeof(T);          // elements per 16-byte staging task
  constexpr int TPP = CC / VE;                // tasks per pixel (power of two)
  constexpr int GPT = CC / KL;                // k-groups per tap in a chunk
  constexpr int KG = K * K * GPT;
  constexpr int KS = (KG + 3) / 4;            // k-steps (4 k-groups each) per chunk
  typedef typename CL<T>::F F;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* xs = reinterpret_cast<T*>(smem);         // [NS][ITH][ITW][PS]
  const int ti = blockIdx.x;
  const Tile tl = tile_of(ti, tilesPS, TH, TW, NS, tilesX, K);
  const int co0 = blockIdx.z * NT * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int ITH = tl.ITH, ITW = tl.ITW;
  const FastDiv fHW(TH * TW), fTW(TW), fITW(ITW), fITH(ITH);
  const int ntask = NS * ITH * ITW * TPP;
  float ss[NT][4], sq[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) { ss[t][i] = 0.f; sq[t][i] = 0.f; }

  (void)NB;   // always 1 here: a batch loop would let the compiler hoist every k-step's
              // weight fragments out of it and blow the register budget
  const int grp0 = wave * GPW;
  int base[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int p = (grp0 + j) * 16 + r16;
    const int s = fHW.div(p), rem = p - s * fHW.d;
    const int ry = fTW.div(rem);
    base[j] = s < NS ? ((s * ITH + ry) * ITW + rem - ry * TW) * PS : 0;
  }
  f4 acc[GPW][NT];
#pragma unroll
  for (int j = 0; j < GPW; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < NCH; ++ch) {
    const int c0 = ch * CC;
    if (ch) __syncthreads();
    // ---- stage the chunk's input tile (zero outside the image)
    for (int task = tid; task < ntask; task += 256) {
      const int q = task % TPP, pix = task / TPP;
      const int rs = fITW.div(pix), c = pix - rs * ITW;
      const int s = fITH.div(rs), r = rs - s * ITH;
      const int iy = tl.ty0 - pad + r, ix = tl.tx0 - pad + c, n = tl.n0 + s;
      const bool ok = n < N && iy >= 0 && iy < H && ix >= 0 && ix < W;
      const u4 v = *reinterpret_cast<const u4*>(
          x + (ok ? (((size_t)n * H + iy) * W + ix) * CIN + c0 + VE * q : 0));
      const u4 vv = ok ? v : u4{0u, 0u, 0u, 0u};
      T* d = xs + pix * PS + VE * q;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<u4*>(d) = vv;
      } else {   // odd f32 pixel stride: scalar writes
        d[0] = __uint_as_float(vv.x); d[1] = __uint_as_float(vv.y);
        d[2] = __uint_as_float(vv.z); d[3] = __uint_as_float(vv.w);
      }
    }
    __syncthreads();
    // ---- MFMA over the chunk's (tap, channel) k-groups; the weight fragments of U k-steps
    // are loaded together ahead of their MFMAs
    constexpr int U = NT >= 4 ? 2 : 4;
    for (int ks0 = 0; ks0 < KS; ks0 += U) {
      F a[U][NT];
      int off[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kg = 4 * (ks0 + u) + g;
        const bool kok = ks0 + u < KS && kg < KG;
        const int tap = kok ? kg / GPT : 0, cg = kok ? kg % GPT : 0;
        const int kh = tap / K, kw = tap - (tap / K) * K;
        off[u] = kok ? (kh * ITW + kw) * PS + cg * KL : 0;
        const int col = tap * CIN + c0 + cg * KL;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const F v = CL<T>::ld(wk + (size_t)(co0 + 16 * t + r16) * Kpad + col);
          a[u][t] = kok ? v : CL<T>::zero();
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ks0 + u >= KS) break;
#pragma unroll
        for (int j = 0; j < GPW; ++j) {
          const F b = CL<T>::ld(xs + base[j] + off[u]);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[j][t] = mma(a[u][t], b, acc[j][t]);
        }
      }
    }
  }
  conv_store<T, NT, GPW>(acc, tl, grp0, fHW, fTW, N, Ho, Wo, Cout, co0, bias, y, ss, sq);
  if (stats) conv_stats<NT>(ss, sq, Cout, co0, stats, total * 4, ti * 4 + wave);
}

// --------------------------------------------------------------------------- Cin == 1
template <typename T, int K, int NT, int GPW>
__global__ __launch_bounds__(256) void conv_c1_kernel(
    const T* __restrict__ x, const T* __restrict__ wk, const float* __restrict__ bias,
    T* __restrict__ y, float* __restrict__ stats, int N, int H, int W, int Cout, int Ho, int Wo,
    int pad, int TH, int TW, int NS, int tilesX, int tilesPS, int total, int Kpad, int NB) {
  constexpr int KL = CL<T>::KL;
  constexpr int KK = K * K;
  constexpr int KS = (KK + 4 * KL - 1) / (4 * KL);   // bf16: 1 k-step (<= 32 taps); f32: 4 taps
  typedef typename CL<T>::F F;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* xs = reinterpret_cast<T*>(smem);                // [NS][ITH][ITW]
  const int ti = blockIdx.x;
  const Tile tl = tile_of(ti, tilesPS, TH, TW, NS, tilesX, K);
  const int co0 = blockIdx.z * NT * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r16 = lane & 15;
  const int ITH = tl.ITH, ITW = tl.ITW;
  const FastDiv fHW(TH * TW), fTW(TW), fITW(ITW), fITH(ITH);
  const int npix = NS * ITH * ITW;

  for (int pix = tid; pix < npix; pix += 256) {
    const int rs = fITW.div(pix), c = pix - rs * ITW;
    const int s = fITH.div(rs), r = rs - s * ITH;
    const int iy = tl.ty0 - pad + r, ix = tl.tx0 - pad + c, n = tl.n0 + s;
    const bool ok = n < N && iy >= 0 && iy < H && ix >= 0 && ix < W;
    const T v = x[ok ? ((size_t)n * H + iy) * W + ix : 0];
    xs[pix] = ok ? v : T(0);
  }
  // weights (A) and tap offsets are the same for every pixel group
  F a[KS][NT];
  int toff[KS][KL];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k0 = (4 * ks + g) * KL;                // this lane's first tap
#pragma unroll
    for (int t = 0; t < NT; ++t) a[ks][t] = CL<T>::ld(wk + (size_t)(co0 + 16 * t + r16) * Kpad + k0);
#pragma unroll
    for (int e = 0; e < KL; ++e) {
      const int tap = k0 + e < KK ? k0 + e : 0;      // padded taps: weight 0, any finite data
      toff[ks][e] = (tap / K) * ITW + tap % K;
    }
  }
  __syncthreads();
  float ss[NT][4], sq[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) { ss[t][i] = 0.f; sq[t][i] = 0.f; }
  for (int nb = 0; nb < NB; ++nb) {
    const int grp0 = (nb * 4 + wave) * GPW;
    f4 acc[GPW][NT];
#pragma unroll
    for (int j = 0; j < GPW; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      const int p = (grp0 + j) * 16 + r16;
      const int s = fHW.div(p), rem = p - s * fHW.d;
      const int ry = fTW.div(rem);
      const int bj = s < NS ? (s * ITH + ry) * ITW + rem - ry * TW : 0;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        F b;
        if constexpr (sizeof(T) == 2) {
          unsigned w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            w[e] = (unsigned)xs[bj + toff[ks][2 * e]] | ((unsigned)xs[bj + toff[ks][2 * e + 1]] << 16);
          b = __builtin_bit_cast(bf16x8, u4{w[0], w[1], w[2], w[3]});
        } else {
          b = xs[bj + toff[ks][0]];
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[j][t] = mma(a[ks][t], b, acc[j][t]);
      }
    }
    conv_store<T, NT, GPW>(acc, tl, grp0, fHW, fTW, N, Ho, Wo, Cout, co0, bias, y, ss, sq);
  }
  if (stats) conv_stats<NT>(ss, sq, Cout, co0, stats, total * 4, ti * 4 + wave);
}

// wk[o][tap*C + c] in T (rows padded to the NT*16 blocks, columns to Kpad, zeros elsewhere)
//   fwd:  o = co, c = ci, value w[co][ci][tap];   dgrad: o = ci, c = co, value w[co][ci][KK-1-tap]
template <typename T>
__global__ void weight_layout_cl_kernel(const float* __restrict__ w, T* __restrict__ wk, int Cout,
                                        int Cin, int KK, int dgrad, int O, int C, int Kpad,
                                        int rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * Kpad) return;
  const int o = i / Kpad, k = i % Kpad;
  float v = 0.f;
  if (o < O && k < KK * C) {
    const int tap = k / C, c = k % C;
    v = dgrad ? w[((size_t)c * Cin + o) * KK + (KK - 1 - tap)] : w[((size_t)o * Cin + c) * KK + tap];
  }
  io<T>::st(wk, i, v);
}

// Several layouts in one launch (blockIdx.y = entry): the per-step weight layouts of a conv stack
constexpr int WLB_MAX = 16;
struct WLBatch {
  const float* w[WLB_MAX];
  void* wk[WLB_MAX];
  int cout[WLB_MAX], cin[WLB_MAX], kk[WLB_MAX], dgrad[WLB_MAX], rows[WLB_MAX], kpad[WLB_MAX];
};

template <typename T>
__global__ void weight_layout_batch_kernel(WLBatch b) {
  const int e = blockIdx.y;
  const int dg = b.dgrad[e], Cout = b.cout[e], Cin = b.cin[e], KK = b.kk[e], Kpad = b.kpad[e];
  const int O = dg ? Cin : Cout, C = dg ? Cout : Cin, n = b.rows[e] * Kpad;
  const float* w = b.w[e];
  T* wk = reinterpret_cast<T*>(b.wk[e]);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int o = i / Kpad, k = i % Kpad;
    float v = 0.f;
    if (o < O && k < KK * C) {
      const int tap = k / C, c = k % C;
      v = dg ? w[((size_t)c * Cin + o) * KK + (KK - 1 - tap)] : w[((size_t)o * Cin + c) * KK + tap];
    }
    io<T>::st(wk, i, v);
  }
}

// ----------------------------------------------------------------------------- host plan
struct Plan { int TH, TW, NS, GPW, NB, tilesX, tiles; };
// widest output-channel block that may use 7 pixel groups per wave (AGPR budget / occupancy)
constexpr int GPW7_MAX_COUT = 32;

// Tiling of an Ho x Wo output map into blocks of 64*GPW*NB pixels (GPW in {4, 7}; NB batches,
// only when all input channels fit one LDS chunk).  Whole small maps are packed NS per block
// with NS | B so a block never straddles two BatchNorm groups (views).  Score = utilisation x
// (block size / ~1024 px)^1/4: larger blocks amortise the staging round trip; ties prefer the
// smaller halo.
Plan plan_cl(int Ho, int Wo, int B, int K, int pix_bytes, bool batches, int Cout) {
  Plan best{0, 0, 0, 0, 0, 0, 0};
  double bsc = -1, bh = 1e9;
  for (int gpw : {4, 7}) {
    if (gpw == 7 && Cout > GPW7_MAX_COUT) continue;   // 7 groups x NT>1 tiles cost occupancy
    for (int nb = 1; nb <= (batches ? 8 : 1); ++nb) {
      const int cap = gpw * 64 * nb;
      if (cap > 2048) continue;
      auto consider = [&](int TH, int TW, int NS) {
        if (TH <= 0 || TW <= 0 || NS <= 0 || TH * TW * NS > cap) return;
        if ((size_t)NS * (TH + K - 1) * (TW + K - 1) * pix_bytes > (size_t)LDS_CAP) return;
        const int tx = avd_cdiv(Wo, TW), ty = avd_cdiv(Ho, TH);
        // batches wholly past the tile's pixels are skipped by the launch (NB trimmed below)
        const int used = TH * TW * NS;
        const int nbu = avd_cdiv(used, gpw * 64);
        const double util = (double)Ho * Wo * NS / ((double)tx * ty * nbu * gpw * 64);
        const double sc =
            batches ? util * std::pow(std::min(1.0, nbu * gpw * 64 / 1024.0), 0.25) : util;
        const double halo = (double)(TH + K - 1) * (TW + K - 1) / (TH * TW);
        if (sc > bsc + 1e-9 || (sc > bsc - 1e-9 && halo < bh)) {
          bsc = sc; bh = halo;
          best = Plan{TH, TW, NS, gpw, nbu, tx, tx * ty};
        }
      };
      if (Ho * Wo <= cap)
        for (int ns = cap / (Ho * Wo); ns >= 1; --ns)
          if (B % ns == 0) consider(Ho, Wo, ns);
      if (Wo <= cap) consider(std::min(Ho, cap / Wo), Wo, 1);
      consider(std::min(Ho, cap / 16), 16, 1);
      for (int tw = 4; tw <= Wo && tw <= cap; tw += 2)
        if (Wo % tw == 0) consider(std::min(Ho, cap / tw), tw, 1);
    }
  }
  return best;
}

}  // namespace

// ============================================================================= entry points
int avd_cl_layout_rows_impl(int O) { return O > 32 ? (O + 63) / 64 * 64 : (O + 15) / 16 * 16; }

namespace {
int pix_bytes(int dt, int Cin) {
  if (Cin == 1) return dt == AVD_BF16 ? 2 : 4;
  if (dt == AVD_BF16) { const int cc = std::min(Cin, 32); return 2 * (cc == 8 ? 8 : cc + 8); }
  return 4 * (std::min(Cin, 32) + 1);
}
}  // namespace

bool avd_c1p8_eligible(int dt, int Cin, int Cout, int K, int Ho, int Wo);
int avd_c1p8_stat_rows(int H, int B);
int avd_c1p8_fwd(const void* x, const void* wk, const float* bias, void* y, float* stats, int N,
                 int H, int W, hipStream_t st);

// BN partial rows per group written by avd_conv_cl_fwd (0 if no tiling fits)
int avd_ws_stat_rows(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt);
int avd_ws_conv_fwd(const void* x, const void* wk, const float* bias, void* y, float* stats,
                    int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                    hipStream_t st, const float* pivot);
int avd_ws_conv_dgrad(const void* dy, const void* wk_d, void* dx, int dt, int N, int Cin, int H,
                      int W, int Cout, int K, int pad, hipStream_t st);

bool avd_c3_serves(int dt, int C, int O, int K, int pad);
int avd_c3_stat_rows(int H, int W, int B);
int avd_c3_conv(const void* x, const void* wk, const float* bias, void* y, float* stats, int N,
                int B, int H, int W, int C, int O, hipStream_t st);

int avd_cl_stat_rows_impl(int Ho, int Wo, int B, int K, int Cin, int Cout, int dt) {
  // 3x3 layers are pad 1 throughout (the conv entry point rejects other paddings there)
  if (avd_c3_serves(dt, Cin, Cout, K, 1)) return avd_c3_stat_rows(Ho, Wo, B);
  if (const int r = avd_ws_stat_rows(Ho, Wo, B, K, Cin, Cout, dt)) return r;
  if (avd_c1p8_eligible(dt, Cin, Cout, K, Ho, Wo)) return avd_c1p8_stat_rows(Ho, B);
  const Plan p = plan_cl(Ho, Wo, B, K, pix_bytes(dt, Cin), Cin == 1, Cout);
  return p.NS ? (B / p.NS) * p.tiles * 4 : 0;   // one partial row per wave
}

int avd_cl_weight_layout_batch_impl(int n, const float* const* w, void* const* wk,
                                    const int* cout, const int* cin, const int* k,
                                    const int* dgrad, int dt, hipStream_t st) {
  if (n <= 0 || n > WLB_MAX) return AVD_ERR_SHAPE;
  WLBatch b{};
  int most = 0;
  for (int e = 0; e < n; ++e) {
    if (!w[e] || !wk[e]) return AVD_ERR_ARG;
    const int O = dgrad[e] ? cin[e] : cout[e], C = dgrad[e] ? cout[e] : cin[e];
    b.w[e] = w[e];
    b.wk[e] = wk[e];
    b.cout[e] = cout[e];
    b.cin[e] = cin[e];
    b.kk[e] = k[e] * k[e];
    b.dgrad[e] = dgrad[e];
    b.kpad[e] = avd_cdiv(k[e] * k[e] * C, 32) * 32;
    b.rows[e] = avd_cl_layout_rows_impl(O);
    most = std::max(most, b.rows[e] * b.kpad[e]);
  }
  dim3 grid(std::min(avd_cdiv(most, 256), 256), n);
  if (dt == AVD_BF16) weight_layout_batch_kernel<bf16><<<grid, 256, 0, st>>>(b);
  else weight_layout_batch_kernel<float><<<grid, 256, 0, st>>>(b);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_cl_weight_layout_impl(const float* w, void* wk, int dt, int Cout, int Cin, int K,
                              int dgrad, hipStream_t st) {
  const int O = dgrad ? Cin : Cout, C = dgrad ? Cout : Cin;
  const int Kpad = avd_cdiv(K * K * C, 32) * 32;
  const int rows = avd_cl_layout_rows_impl(O);
  const int n = rows * Kpad;
  if (dt == AVD_BF16)
    weight_layout_cl_kernel<bf16><<<avd_cdiv(n, 256), 256, 0, st>>>(w, (bf16*)wk, Cout, Cin, K * K,
                                                                   dgrad, O, C, Kpad, rows);
  else
    weight_layout_cl_kernel<float><<<avd_cdiv(n, 256), 256, 0, st>>>(w, (float*)wk, Cout, Cin, K * K,
                                                                    dgrad, O, C, Kpad, rows);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

namespace {

template <typename T, int K, int CIN, int NT, int GPW>
int launch_cl(const Plan& p, const void* x, const void* wk, const float* bias, void* y,
              float* stats, int N, int H, int W, int Cout, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  constexpr int PS = Chunk<T, CIN>::PS;
  const size_t lds = (size_t)p.NS * (p.TH + K - 1) * (p.TW + K - 1) * PS * sizeof(T);
  if (lds > (size_t)LDS_CAP) return AVD_ERR_SHAPE;
  const int Kpad = avd_cdiv(K * K * CIN, 32) * 32;
  const int total = p.tiles * avd_cdiv(N, p.NS);
  dim3 grid(total, 1, avd_cdiv(Cout, NT * 16));
  conv_cl_kernel<T, K, CIN, NT, GPW><<<grid, 256, lds, st>>>(
      (const T*)x, (const T*)wk, bias, (T*)y, stats, N, H, W, Cout, Ho, Wo, pad, p.TH, p.TW, p.NS,
      p.tilesX, p.tiles, total, Kpad, p.NB);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

template <typename T, int K, int NT, int GPW>
int launch_c1(const Plan& p, const void* x, const void* wk, const float* bias, void* y,
              float* stats, int N, int H, int W, int Cout, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  const size_t lds = (size_t)p.NS * (p.TH + K - 1) * (p.TW + K - 1) * sizeof(T);
  const int Kpad = 32;
  const int total = p.tiles * avd_cdiv(N, p.NS);
  dim3 grid(total, 1, avd_cdiv(Cout, NT * 16));
  conv_c1_kernel<T, K, NT, GPW><<<grid, 256, lds, st>>>(
      (const T*)x, (const T*)wk, bias, (T*)y, stats, N, H, W, Cout, Ho, Wo, pad, p.TH, p.TW, p.NS,
      p.tilesX, p.tiles, total, Kpad, p.NB);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

template <typename T>
int dispatch_cl(const Plan& p, const void* x, const void* wk, const float* bias, void* y,
                float* stats, int N, int Cin, int H, int W, int Cout, int K, int pad,
                hipStream_t st) {
  const int NT = Cout <= 16 ? 1 : Cout <= 32 ? 2 : 4;
#define AVD_C(KK, CI, NTT, G)                                                                \
  if (K == KK && Cin == CI && NT == NTT && p.GPW == G)                                      \
    return launch_cl<T, KK, CI, NTT, G>(p, x, wk, bias, y, stats, N, H, W, Cout, pad, st);
#define AVD_CN(KK, CI) AVD_C(KK, CI, 1, 4) AVD_C(KK, CI, 2, 4) AVD_C(KK, CI, 4, 4) \
                       AVD_C(KK, CI, 1, 7) AVD_C(KK, CI, 2, 7) AVD_C(KK, CI, 4, 7)
#define AVD_1(KK, NTT, G)                                                                    \
  if (K == KK && Cin == 1 && NT == NTT && p.GPW == G)                                       \
    return launch_c1<T, KK, NTT, G>(p, x, wk, bias, y, stats, N, H, W, Cout, pad, st);
  AVD_1(5, 1, 4) AVD_1(5, 2, 4) AVD_1(5, 4, 4) AVD_1(5, 1, 7) AVD_1(5, 2, 7) AVD_1(5, 4, 7)
  AVD_1(3, 1, 4) AVD_1(3, 2, 4) AVD_1(3, 4, 4) AVD_1(3, 1, 7) AVD_1(3, 2, 7) AVD_1(3, 4, 7)
  AVD_CN(5, 8) AVD_CN(5, 16) AVD_CN(5, 32) AVD_CN(5, 64)
  AVD_CN(3, 8) AVD_CN(3, 16) AVD_CN(3, 32) AVD_CN(3, 64) AVD_CN(3, 128) AVD_CN(3, 256)
#undef AVD_1
#undef AVD_CN
#undef AVD_C
  return AVD_ERR_SHAPE;
}

}  // namespace

// y = conv(x) + bias over NHWC maps (+ BN partials stats [Cout][N/NS * tiles][2] when
// stats != NULL).  x/y/wk in dt; wk = avd_cl_weight_layout(fwd).  B = samples per BN group.
int avd_cl_conv_fwd_impl(const void* x, const void* wk, const float* bias, void* y, float* stats,
                         int dt, int N, int B, int Cin, int H, int W, int Cout, int K, int pad,
                         hipStream_t st, const float* pivot) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  if (Ho <= 0 || Wo <= 0 || B <= 0 || N % B) return AVD_ERR_SHAPE;
  // a statistics pivot is taken only by the producers whose lane-local running sums are long
  // (avd_cl_stat_pivot): anywhere else the caller must not pass one
  if (pivot && !avd_ws_stat_rows(Ho, Wo, B, K, Cin, Cout, dt)) return AVD_ERR_ARG;
  if (Cin != 1 && Cin % 8) return AVD_ERR_SHAPE;
  if (Cout % 4) return AVD_ERR_SHAPE;
  if (avd_c1p8_eligible(dt, Cin, Cout, K, Ho, Wo)) {   // the audio first layer: pixel-pair MFMA
    if (pad != 2) return AVD_ERR_SHAPE;
    return avd_c1p8_fwd(x, wk, bias, y, stats, N, H, W, st);
  }
  // the 32..256-channel 3x3 layers: LDS-staged implicit GEMM (conv3.hip)
  if (avd_c3_serves(dt, Cin, Cout, K, 1)) {
    if (pad != 1) return AVD_ERR_SHAPE;
    return avd_c3_conv(x, wk, bias, y, stats, N, B, H, W, Cin, Cout, st);
  }
  // the mid-layer shapes: weights-stationary persistent kernel (conv_ws.hip)
  if (const int r = avd_ws_conv_fwd(x, wk, bias, y, stats, dt, N, B, Cin, H, W, Cout, K, pad, st,
                                   pivot))
    return r > 0 ? AVD_OK : r;
  // batches only for Cin = 1 (its weights live in registers; the Cin >= 8 kernel would re-read
  // its weight fragments per batch)
  const Plan p = plan_cl(Ho, Wo, B, K, pix_bytes(dt, Cin), Cin == 1, Cout);
  if (!p.NS) return AVD_ERR_SHAPE;
  if (dt == AVD_BF16)
    return dispatch_cl<bf16>(p, x, wk, bias, y, stats, N, Cin, H, W, Cout, K, pad, st);
  return dispatch_cl<float>(p, x, wk, bias, y, stats, N, Cin, H, W, Cout, K, pad, st);
}

// dx = conv2d input-gradient over NHWC maps: the forward kernel on dY with the flipped,
// channel-swapped weights (avd_cl_weight_layout dgrad) and padding K-1-pad.
int avd_cl_conv_dgrad_impl(const void* dy, const void* wk_d, void* dx, int dt, int N, int Cin,
                           int H, int W, int Cout, int K, int pad, hipStream_t st) {
  const int Ho = H + 2 * pad - K + 1, Wo = W + 2 * pad - K + 1;
  if (Ho <= 0 || Wo <= 0 || Cout % 8 || Cin % 4 || K - 1 - pad < 0) return AVD_ERR_SHAPE;
  if (avd_c3_serves(dt, Cout, Cin, K, K - 1 - pad) && Ho == H && Wo == W)
    return avd_c3_conv(dy, wk_d, nullptr, dx, nullptr, N, N, H, W, Cout, Cin, st);
  if (const int r = avd_ws_conv_dgrad(dy, wk_d, dx, dt, N, Cin, H, W, Cout, K, pad, st))
    return r > 0 ? AVD_OK : r;
  const Plan p = plan_cl(H, W, N, K, pix_bytes(dt, Cout), false, Cin);
  if (!p.NS) return AVD_ERR_SHAPE;
  if (dt == AVD_BF16)
    return dispatch_cl<bf16>(p, dy, wk_d, nullptr, dx, nullptr, N, Cout, Ho, Wo, Cin, K,
                             K - 1 - pad, st);
  return dispatch_cl<float>(p, dy, wk_d, nullptr, dx, nullptr, N, Cout, Ho, Wo, Cin, K,
                            K - 1 - pad, st);
}
