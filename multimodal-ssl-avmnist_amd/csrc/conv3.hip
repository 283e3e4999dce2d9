// 3x3 convolutions (pad 1) of the SimCLR / unimodal image and spectrogram encoders
// (models/dino.py:18-73 image_encoder / audio_encoder: 32..256 channels on 56x56 .. 7x7 maps)
// as an implicit GEMM on v_mfma_f32_16x16x32_bf16, NHWC bf16, forward (+ bias and the fused
// BatchNorm partial statistics) and input gradient (the same kernel on dY with the flipped,
// channel-swapped weights).
//
// Why not conv_cl_kernel for these: it reads its weight fragments from global memory inside
// the k-loop and keeps small pixel tiles, which for 32..256-channel 3x3 layers leaves the
// MFMAs at 8-13 % of peak (config 4 profile, r2).  Here a block owns a tile of up to 448 output
// pixels (TR rows of one sample, or NS whole small maps) x 64 output channels, and for each
// 32-channel input chunk stages
//   * the input tile + 1-pixel halo, 32 channels = one 64-byte row per pixel,
//   * the 64 x 9 x 32 weight slice, one 64-byte row per (tap, output channel),
// into LDS once (LDS-DMA); every tap of the chunk then reads both operands from LDS.  64-byte
// rows carry their four 16-byte chunks XOR-swizzled (swz() below), so the rows one MFMA
// fragment read touches land on distinct 4-bank slots (conflict-free ds_read_b128).
//   A = weights  [16 output channels][32 input channels of one tap]
//   B = input    [32 input channels][16 output pixels], shifted by the tap
//   C: lane holds 4 consecutive output channels of one pixel -> one 8-byte NHWC store.
// Each wave owns GPW 16-pixel groups (interleaved over the waves) x NT 16-channel tiles.
#include <algorithm>

#include "common.h"

using namespace avd;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

constexpr int CH = 32;            // input channels per LDS chunk (one MFMA k-step per tap)
constexpr int ROWB = CH * 2;      // bytes per LDS row

__device__ const u4 kZero3 = {0u, 0u, 0u, 0u};

// a / b for 0 <= a < 2^22 through the f32 reciprocal rb = 1 / b (exact after one correction):
// a handful of VALU instructions instead of the ~30 of a runtime integer division
__device__ __forceinline__ int fdivi(int a, int b, float rb) {
  int q = (int)((float)a * rb);
  const int r = a - q * b;
  q += (r >= b) - (r < 0);
  return q;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>(p);
}
__device__ __forceinline__ bf16x8 lds16(uint32_t a) {
  return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(a);
}

// one 16-byte LDS-DMA per lane: lane l's global 16 bytes land at lds_wave + 16 * l
__device__ __forceinline__ void glds16(const void* g, const bf16* lds_wave) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(
      reinterpret_cast<uintptr_t>(lds_wave)), 16, 0, 0);
}

// LDS swizzle of the 64-byte rows (16-byte chunk q of row r sits at chunk q ^ ((r >> 1) & 2)).  ds_read_b128 is serviced in four
// 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32); a fragment read puts rows
// b..b+15 of chunks (2k, 2k+1) into a group pair, and flipping bit 1 of the chunk on every
// other 4-row block spreads each group over the 16 slots of a bank row for ANY b (a tap shift
// moves b by 1..2*IW+2): conflict-free, where (r >> 2) & 3 was 2-way for b % 16 != 4.

// Persistent, double-buffered: one block of 8 waves per CU walks a contiguous range of work
// items (tile, 64- or 32-channel output group); each item runs one unit per 32-channel input
// chunk, and the LDS-DMA of unit u+1 (input tile + halo, weight slice) is in flight while unit
// u's MFMAs run.  Waves 0-3 / 4-7 own the two halves of the output group's channel tiles, wave
// & 3 the pixel groups (wave & 3) + 4j.  Input rows are padded to IW8 (multiple of 16) pixels, so
// a tap's row shift ky * IW8 keeps the swizzle phase and becomes an immediate offset: after a
// per-unit base add, every fragment read is an immediate-offset ds_read_b128.
constexpr int XPAD = 16;

template <int BO, int GPW, int IW8>
__global__ __launch_bounds__(512, 1) void conv3p_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, const float* __restrict__ bias,
    bf16* __restrict__ y, float* __restrict__ stats, int N, int H, int W, int C, int O, int TR,
    int NS, int tilesPS, int xrows, int nitems, int G) {
  constexpr int NTW = BO / 32;                 // 16-channel tiles per wave
  constexpr int WROWS = 9 * BO;                // weight rows per unit
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  float* bs = reinterpret_cast<float*>(smem);  // [O <= 256] bias
  bf16* buf = smem + 512;                      // 2 x {input [xrows][32], weights [9*BO][32]}
  const int bufE = (xrows + WROWS) * CH;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int g = lane >> 4, r16 = lane & 15;
  const int wp = wave & 3, wt = wave >> 2;
  const int IR = TR + 2, TRW = TR * W, TP = NS * TRW;
  const int ngo = O / BO, nch = C / CH;
  const int tiles = nitems / ngo, tilesPG = tiles / G;   // items are (og, tile), og-major
  const int it0 = (int)((long long)blockIdx.x * nitems / gridDim.x);
  const int it1 = (int)((long long)(blockIdx.x + 1) * nitems / gridDim.x);
  const float rW = 1.f / W, rTRW = 1.f / TRW, rIR = 1.f / IR;

  for (int i = tid; i < O; i += 512) bs[i] = bias ? bias[i] : 0.f;

  // lane geometry (the same for every tile): B-read byte offsets for kx = 0..2, and (s, r, xx)
  int xoff[GPW][3], pos[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int p = (wp + 4 * j) * 16 + r16;
    const int sN = fdivi(p, TRW, rTRW), rem = p - sN * TRW;
    const int r = fdivi(rem, W, rW), xx = rem - r * W;
    const int base = (sN * IR + r) * IW8 + xx;
    pos[j] = p < TP ? (sN << 16) | (r << 8) | xx : -1;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int row = p < TP ? base + kx : kx;
      xoff[j][kx] = row * 64 + ((g ^ ((row >> 1) & 2)) << 4);
    }
  }
  const int aoff = (16 * NTW * wt + r16) * 64 + ((g ^ ((r16 >> 1) & 2)) << 4);

  auto stage = [&](int item, int c, int b) {
    bf16* xb = buf + b * bufE;
    bf16* wb = xb + xrows * CH;
    const int og = item / tiles, ti = item - og * tiles;
    const int sg = ti / tilesPS, tt = ti - sg * tilesPS;
    const int n0 = sg * NS, y0 = tt * TR, o0 = og * BO, c0 = c * CH;
    // input: rows of IW8 * 4 slots (a multiple of 64: whole wave instructions)
    const int nin = NS * IR * IW8 / 16;
    for (int k = wave_u; k < nin; k += 8) {
      const int row = (64 * k) / (IW8 * 4);
      const int ls = 64 * k - row * (IW8 * 4) + lane;
      const int px = ls >> 2, q = (ls & 3) ^ ((px >> 1) & 2);
      const int sN = fdivi(row, IR, rIR), iy = y0 + row - sN * IR - 1, n = n0 + sN, ix = px - 1;
      const bool ok = n < N && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      glds16(ok ? (const void*)(x + (((size_t)n * H + iy) * W + ix) * C + c0 + 8 * q)
                : (const void*)&kZero3, xb + 64 * k * 8);
    }
    for (int k = wave_u; k < WROWS / 16; k += 8) {
      const int sl = 64 * k + lane, row = sl >> 2, q = (sl & 3) ^ ((row >> 1) & 2);
      const int tap = row / BO, m = row - tap * BO;
      // A row (tile T, m) holds channel T*16+m, or with two tiles per wave the channel that puts
      // 8 consecutive channels into each lane's two accumulators (one 16-byte store)
      const int T = m >> 4, mm = m & 15;
      const int o = NTW == 2 ? 32 * (T >> 1) + 8 * (mm >> 2) + 4 * (T & 1) + (mm & 3) : m;
      glds16(wk + (size_t)(o0 + o) * (9 * C) + tap * C + c0 + 8 * q, wb + 64 * k * 8);
    }
  };

  f4 acc[GPW][NTW];
#pragma unroll
  for (int j = 0; j < GPW; ++j)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};

  // BatchNorm partial sums: rows [blockIdx.x * 4 + wp] of R = gridDim.x * 4 per group
  float run_s[NTW][4], run_q[NTW][4];
  int cur_pair = -1;
  const int srow = blockIdx.x * 4 + wp, R = gridDim.x * 4;
  auto coff = [](int t, int i) { return (NTW == 2 ? 4 * t : 0) + i; };
  auto flush = [&](int pr) {
    if (r16) return;
    const int ogp = pr / G, gp = pr - ogp * G;
    const int cwp = ogp * BO + 16 * NTW * wt + 4 * NTW * g;
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t o = (((size_t)(cwp + coff(t, i)) * G + gp) * R + srow) * 2;
        *reinterpret_cast<float2*>(stats + o) = make_float2(run_s[t][i], run_q[t][i]);
      }
  };

  // units u = (item, chunk) in order; the barrier after unit u's MFMAs retires unit u+1's
  // DMA (issued before those MFMAs) and the previous epilogue's stores, so neither is waited
  // for right after being issued; unit u+2's DMA then refills the buffer unit u just left
  const int nunits = (it1 - it0) * nch;
  if (nunits > 0) stage(it0, 0, 0);
  __syncthreads();
  if (nunits > 1) stage(it0 + (nch == 1), nch == 1 ? 0 : 1, 1);
  for (int u = 0; u < nunits; ++u) {
    const int item = it0 + u / nch, c = u - (u / nch) * nch;
    // ---- 9 taps x NTW x GPW MFMAs; 32-bit LDS addresses with immediate tap offsets, the
    // next tap's fragments read while this tap's MFMAs run
    {
      const uint32_t xb = lds_addr(buf + (u & 1) * bufE);
      const uint32_t ab = xb + xrows * CH * 2 + aoff;
      uint32_t bp[GPW][3];
#pragma unroll
      for (int j = 0; j < GPW; ++j)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) bp[j][kx] = xb + xoff[j][kx];
      bf16x8 a[2][NTW], bv[2][GPW];
#pragma unroll
      for (int t = 0; t < NTW; ++t) a[0][t] = lds16(ab + 16 * t * 64);
#pragma unroll
      for (int j = 0; j < GPW; ++j) bv[0][j] = lds16(bp[j][0]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int cur = tap & 1, nxt = cur ^ 1;
        if (tap < 8) {
          const int ky = (tap + 1) / 3, kx = (tap + 1) % 3;
#pragma unroll
          for (int t = 0; t < NTW; ++t) a[nxt][t] = lds16(ab + ((tap + 1) * BO + 16 * t) * 64);
#pragma unroll
          for (int j = 0; j < GPW; ++j) bv[nxt][j] = lds16(bp[j][kx] + ky * IW8 * 64);
        }
        __builtin_amdgcn_sched_barrier(0);     // keep the prefetch ahead of this tap's MFMAs
#pragma unroll
        for (int j = 0; j < GPW; ++j)
#pragma unroll
          for (int t = 0; t < NTW; ++t)
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cur][t], bv[cur][j], acc[j][t], 0, 0, 0);
      }
    }
    __syncthreads();
    if (u + 2 < nunits) stage(it0 + (u + 2) / nch, (u + 2) % nch, u & 1);
    if (c == nch - 1) {
      // ---- epilogue: bias, bf16 rounding, NHWC store, BN sums of the stored values
      const int og = item / tiles, ti = item - og * tiles;
      const int sg = ti / tilesPS, tt = ti - sg * tilesPS;
      const int n0 = sg * NS, y0 = tt * TR;
      const int cw = og * BO + 16 * NTW * wt + 4 * NTW * g;
      float bv[NTW][4], ss[NTW][4], sq[NTW][4];
#pragma unroll
      for (int t = 0; t < NTW; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bv[t][i] = bs[cw + coff(t, i)];
          ss[t][i] = 0.f;
          sq[t][i] = 0.f;
        }
#pragma unroll
      for (int j = 0; j < GPW; ++j) {
        const int ps = pos[j];
        const int sN = ps >> 16, r = (ps >> 8) & 255, xx = ps & 255;
        if (ps < 0 || y0 + r >= H) continue;
        bf16* yp = y + ((((size_t)(n0 + sN) * H + y0 + r) * W + xx) * O + cw);
        uint32_t pk[NTW][2];
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const uint32_t lo = pack_bf16x2(acc[j][t][0] + bv[t][0], acc[j][t][1] + bv[t][1]);
          const uint32_t hi = pack_bf16x2(acc[j][t][2] + bv[t][2], acc[j][t][3] + bv[t][3]);
          const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                              __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            ss[t][i] += v[i];
            sq[t][i] = fmaf(v[i], v[i], sq[t][i]);
          }
          pk[t][0] = lo;
          pk[t][1] = hi;
        }
        if constexpr (NTW == 2)
          *reinterpret_cast<u4*>(yp) = u4{pk[0][0], pk[0][1], pk[1][0], pk[1][1]};
        else
          *reinterpret_cast<uint2*>(yp) = make_uint2(pk[0][0], pk[0][1]);
      }
      if (stats) {
        // per-block running sums over the tiles of one (og, BatchNorm group): written once per
        // such run (and zeros for the pairs the block never reaches) into row blockIdx*4 + wp
        const int pair = og * G + ti / tilesPG;
        if (pair != cur_pair) {
          if (cur_pair >= 0) flush(cur_pair);
          cur_pair = pair;
#pragma unroll
          for (int t = 0; t < NTW; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) { run_s[t][i] = 0.f; run_q[t][i] = 0.f; }
        }
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            run_s[t][i] += row16_sum(ss[t][i]);
            run_q[t][i] += row16_sum(sq[t][i]);
          }
      }
#pragma unroll
      for (int j = 0; j < GPW; ++j)
#pragma unroll
        for (int t = 0; t < NTW; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (stats) {
    if (cur_pair >= 0) flush(cur_pair);
    // the (og, group) pairs this block never reached: zero rows.  The reached pairs are the
    // contiguous interval [first, last] of the og-major order.
    int first = 0, last = -1;
    if (it0 < it1) {
      first = (it0 / tiles) * G + (it0 % tiles) / tilesPG;
      last = ((it1 - 1) / tiles) * G + ((it1 - 1) % tiles) / tilesPG;
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) { run_s[t][i] = 0.f; run_q[t][i] = 0.f; }
    for (int pr = 0; pr < ngo * G; ++pr)
      if (pr < first || pr > last) flush(pr);
  }
}

struct Plan3 { int TR, NS, GPW, tilesPS, IW8, xrows; };

int iw8_of(int W) { return (W + 2 + XPAD - 1) / XPAD * XPAD; }

// The tile with the best utilisation of GPW*64 pixel slots (ties: more pixels); whole small
// maps are packed NS per block with NS | B (a tile never straddles two BatchNorm groups); the
// two LDS buffers (input rows + a 64-channel weight slice) and the bias fit 160 KB.
Plan3 plan3(int H, int W, int B) {
  Plan3 best{0, 0, 0, 0, 0, 0};
  double bu = -1;
  const int IW8 = iw8_of(W);
  for (int gpw : {4, 7}) {
    const int cap = gpw * 64;
    auto consider = [&](int TR, int NS) {
      if (TR <= 0 || NS <= 0 || TR * W * NS > cap || TR > 255) return;
      const int xrows = NS * (TR + 2) * IW8;
      if (2 * (xrows + 9 * 64) * ROWB + 1024 > 160 * 1024) return;
      const int tps = avd_cdiv(H, TR);
      const double u = (double)H * W * NS / ((double)tps * cap);
      if (u > bu + 1e-9 || (u > bu - 1e-9 && TR * NS > best.TR * best.NS)) {
        bu = u;
        best = Plan3{TR, NS, gpw, tps, IW8, xrows};
      }
    };
    if (H * W <= cap)
      for (int ns = cap / (H * W); ns >= 1; --ns)
        if (B % ns == 0) consider(H, ns);
    for (int tr = 1; tr <= H && tr * W <= cap; ++tr) consider(tr, 1);
  }
  return best;
}

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int BO, int GPW, int IW8>
int launch3(const Plan3& p, const void* x, const void* wk, const float* bias, void* y, float* stats,
            int N, int B, int H, int W, int C, int O, hipStream_t st) {
  const size_t lds = 1024 + 2 * (size_t)(p.xrows + 9 * BO) * ROWB;
  const int tiles = (N / p.NS) * p.tilesPS;
  const int nitems = tiles * (O / BO);
  // with statistics every CU's block owns 4 partial rows per group (avd_c3_stat_rows)
  const int grid = stats ? num_cus() : std::min(nitems, num_cus());
  conv3p_kernel<BO, GPW, IW8><<<grid, 512, lds, st>>>(
      (const bf16*)x, (const bf16*)wk, bias, (bf16*)y, stats, N, H, W, C, O, p.TR, p.NS,
      p.tilesPS, p.xrows, nitems, N / B);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // namespace

// Served: bf16, 3x3, pad 1, C (input channels of the executed conv) % 32 == 0, O % 32 == 0,
// O <= 256, maps up to 62 pixels wide.
bool avd_c3_serves(int dt, int C, int O, int K, int pad) {
  return dt == AVD_BF16 && K == 3 && pad == 1 && C % CH == 0 && C >= CH && O % 32 == 0 && O <= 256;
}

// BN partial rows per group of avd_c3_conv (fwd): 4 per CU (each block's running sums)
int avd_c3_stat_rows(int H, int W, int B) {
  const Plan3 p = plan3(H, W, B);
  return p.NS ? 4 * num_cus() : 0;
}

// y = conv3x3(x) (+ bias, + stats) over NHWC bf16 maps; x [N][H][W][C], wk the avd_cl weight
// layout ([O][9*C], tap-major) of the executed conv (the dgrad layout for an input gradient).
int avd_c3_conv(const void* x, const void* wk, const float* bias, void* y, float* stats, int N,
                int B, int H, int W, int C, int O, hipStream_t st) {
  const Plan3 p = plan3(H, W, B);
  if (!p.NS || N % p.NS || N % B || B % p.NS || O > 256) return AVD_ERR_SHAPE;
#define AVD_L(BO_, G, I)                                                                     \
  if (O % BO_ == 0 && p.GPW == G && p.IW8 == I)                                              \
    return launch3<BO_, G, I>(p, x, wk, bias, y, stats, N, B, H, W, C, O, st);
  AVD_L(64, 7, 64) AVD_L(64, 7, 32) AVD_L(64, 7, 16) AVD_L(64, 4, 64) AVD_L(64, 4, 32)
  AVD_L(64, 4, 16) AVD_L(32, 7, 64) AVD_L(32, 7, 32) AVD_L(32, 7, 16) AVD_L(32, 4, 64)
  AVD_L(32, 4, 32) AVD_L(32, 4, 16)
#undef AVD_L
  return AVD_ERR_SHAPE;
}

// ============================================================================ weight gradient
// dW[co][ci][tap] = sum_p dY[p][co] * X[p + tap][ci] for the same 3x3 layers, as a GEMM
// M = co (a group of BO), N = (tap, ci) of one 32-channel input group = 18 column tiles,
// K = output pixels, split over pixel chunks (deterministic slabs, summed by avd_sum_rows).
// A block stages one strip (TR output rows of one sample) at a time: dY [pixels][BO] and
// X [halo rows][halo cols][32]; both MFMA operands are pixel-major there, so their fragments
// come from ds_read_b64_tr_b16 (4 pixels x 4 channels per read, two reads per fragment; the
// k-step's 32 pixels are ordered so that each half-wave reads 8 consecutive pixels: the
// wgrad_ws.hip scheme).  Pixel rows are padded to WO8 (multiple of 8) so a 4-pixel run never
// crosses a row; the pad pixels' dY stays zero.  The groups (co, ci) of one pixel chunk are
// consecutive logical blocks mapped onto one XCD, so its strips are re-read from that XCD's L2.
namespace {

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

constexpr int XS3 = CH + 16;     // X LDS pixel stride (elements)

template <int BO>
__global__ __launch_bounds__(256, 2) void wgrad3_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ parts, int N,
    int H, int W, int Cin, int Cout, int TR, int nchunk, int ngroup) {
  constexpr int DYS = BO + 16;               // dY LDS pixel stride (elements)
  constexpr int MTW = BO / 32;               // o-tiles per wave (2 wave rows)
  constexpr int NW = 9;                      // column tiles per wave (2 wave columns of 9)
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int g = lane >> 4, r16 = lane & 15, q4 = r16 >> 2, p4 = r16 & 3;
  const int wo = wave & 1, wc = wave >> 1;
  // XCD-aware: logical block L = (hw block % 8) * (grid / 8) + hw block / 8 (grid % 8 == 0)
  const int nb = gridDim.x;
  const int L = (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  const int chunk = L / ngroup, grp = L - chunk * ngroup;
  const int ngo = Cout / BO;
  const int o0 = (grp % ngo) * BO, c0 = (grp / ngo) * CH;
  const int WO8 = (W + 7) & ~7, XW = WO8 + 2, XR = TR + 2;
  const int SP = TR * WO8;                   // strip pixels (incl. row pads)
  const int KST = (SP + 31) / 32;
  bf16* dys = smem;                          // [KST*32][DYS]
  bf16* xs = smem + KST * 32 * DYS;          // [XR][XW][XS3]
  const int sps = H / TR;
  const int nstrip = N * sps;
  const int st0 = (int)((long long)chunk * nstrip / nchunk);
  const int st1 = (int)((long long)(chunk + 1) * nstrip / nchunk);

  // pad pixels (ox >= W, and the k tail) of dY stay zero for the whole launch
  for (int i = tid; i < KST * 32 * (DYS / 8); i += 256) {
    const int pix = i / (DYS / 8), ox = pix % WO8;
    if (ox >= W || pix >= SP) *reinterpret_cast<u4*>(dys + (size_t)i * 8) = u4{0u, 0u, 0u, 0u};
  }
  // this lane's column tiles: ct = wc*9 + j -> tap = ct >> 1, ci tile = ct & 1
  int xo[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int ct = wc * NW + j, tap = ct >> 1;
    xo[j] = ((tap / 3) * XW + tap % 3) * XS3 + 16 * (ct & 1) + 4 * p4;
  }
  f4 acc[MTW][NW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[m][j] = f4{0.f, 0.f, 0.f, 0.f};

  for (int st = st0; st < st1; ++st) {
    const int n = st / sps, y0 = (st - n * sps) * TR;
    __syncthreads();
    // dY strip [TR rows x W pixels][BO channels] and X strip + halo (rows y0-1 .. y0+TR, cols
    // -1 .. WO8, zero outside the image) by LDS-DMA: a wave instruction fills 64 consecutive
    // 16-byte slots of the padded image; the slots of row pads (and dY's pad pixels) are skipped
    constexpr int DSP = DYS / 8, XSP = XS3 / 8;
    for (int s0 = 64 * wave_u; s0 < SP * DSP; s0 += 256) {
      const int sl = s0 + lane, pix = sl / DSP, q = sl - pix * DSP;
      const int r = pix / WO8, ox = pix - r * WO8;
      if (q < BO / 8 && ox < W && pix < SP)
        glds16(dy + (((size_t)n * H + y0 + r) * W + ox) * Cout + o0 + 8 * q, dys + s0 * 8);
    }
    for (int s0 = 64 * wave_u; s0 < XR * XW * XSP; s0 += 256) {
      const int sl = s0 + lane, pix = sl / XSP, q = sl - pix * XSP;
      const int r = pix / XW, c = pix - r * XW;
      const int iy = y0 - 1 + r, ix = c - 1;
      const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      if (q < CH / 8 && pix < XR * XW)
        glds16(ok ? (const void*)(x + (((size_t)n * H + iy) * W + ix) * Cin + c0 + 8 * q)
                  : (const void*)&kZero3, xs + s0 * 8);
    }
    __syncthreads();
    for (int ks = 0; ks < KST; ++ks) {
      const int P0 = 32 * ks;
      bf16x8 a[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const int co = 16 * (wo * MTW + m) + 4 * p4;
        a[m] = fr8(trd(dys + (P0 + kpx(g, 0, q4)) * DYS + co),
                   trd(dys + (P0 + kpx(g, 1, q4)) * DYS + co));
      }
      int xb[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int P = min(P0 + kpx(g, h, q4), SP - 1);     // k tail: dY is 0 there
        const int r = P / WO8, ox = P - r * WO8;
        xb[h] = (r * XW + ox) * XS3;
      }
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const bf16x8 b = fr8(trd(xs + xb[0] + xo[j]), trd(xs + xb[1] + xo[j]));
#pragma unroll
        for (int m = 0; m < MTW; ++m)
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b, acc[m][j], 0, 0, 0);
      }
    }
  }

  // slab write [co][ci][tap] through LDS, one o-tile per wave row per pass (32 rows of
  // 32 x 9 floats), so the rows leave as contiguous float4 stores
  float* tb = reinterpret_cast<float*>(smem);   // [32][32 * 9]
  constexpr int PER = CH * 9;
  float* out = parts + (size_t)chunk * Cout * Cin * 9;
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int ct = wc * NW + j, tap = ct >> 1, ci = 16 * (ct & 1) + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) tb[(16 * wo + 4 * g + i) * PER + ci * 9 + tap] = acc[m][j][i];
    }
    __syncthreads();
    for (int e = tid; e < 32 * PER / 4; e += 256) {
      const int row = e / (PER / 4), c4 = e - row * (PER / 4);
      const int co = 16 * ((row >> 4) * MTW + m) + (row & 15);
      reinterpret_cast<float4*>(out + ((size_t)(o0 + co) * Cin + c0) * 9)[c4] =
          reinterpret_cast<const float4*>(tb)[e];
    }
  }
}

size_t wg3_lds(int TR, int W, int BO) {
  const int wo8 = (W + 7) & ~7, kst = (TR * wo8 + 31) / 32;
  return std::max((size_t)kst * 32 * (BO + 16) * 2 + (size_t)(TR + 2) * (wo8 + 2) * XS3 * 2,
                  (size_t)32 * CH * 9 * 4);
}

// strip rows for a map of H x W: the largest divisor of H whose strip fits 72 KB of LDS
// (two blocks per CU) within 256 pixels
int tr3(int H, int W, int BO) {
  const int wo8 = (W + 7) & ~7;
  int best = 1;
  for (int tr = 1; tr <= H; ++tr)
    if (H % tr == 0 && tr * wo8 <= 256 && wg3_lds(tr, W, BO) <= 72 * 1024) best = tr;
  return best;
}

int wg3_bo(int Cout) { return Cout % 128 == 0 ? 128 : 64; }

}  // namespace

// Slabs of avd_c3_wgrad for (N, Cout, Cin), or 0 if not served.
int avd_c3_wgrad_chunks(int N, int Cout, int Cin, int K) {
  if (K != 3 || Cin % CH || Cout % 64) return 0;
  const int groups = (Cout / wg3_bo(Cout)) * (Cin / CH);
  constexpr int target = 512;
  int nchunk = std::max(1, target / groups);
  nchunk = std::min(nchunk, N);
  // the grid (nchunk * groups) must be a multiple of 8 for the XCD remap
  while ((nchunk * groups) % 8) ++nchunk;
  return nchunk;
}

// 1 = launched, 0 = not served, < 0 = error.  parts holds avd_c3_wgrad_chunks slabs.
int avd_c3_wgrad(const void* x, const void* dy, int dt, float* parts, int N, int Cin, int H, int W,
                 int Cout, int K, int pad, hipStream_t st) {
  if (dt != AVD_BF16 || pad != 1) return 0;
  const int nchunk = avd_c3_wgrad_chunks(N, Cout, Cin, K);
  if (!nchunk) return 0;
  const int BO = wg3_bo(Cout), TR = tr3(H, W, BO);
  const int groups = (Cout / BO) * (Cin / CH);
  const size_t lds = wg3_lds(TR, W, BO);
  if (lds > 80 * 1024) return 0;
  const int grid = nchunk * groups;
  if (BO == 128)
    wgrad3_kernel<128><<<grid, 256, lds, st>>>((const bf16*)x, (const bf16*)dy, parts, N, H, W,
                                               Cin, Cout, TR, nchunk, groups);
  else
    wgrad3_kernel<64><<<grid, 256, lds, st>>>((const bf16*)x, (const bf16*)dy, parts, N, H, W,
                                              Cin, Cout, TR, nchunk, groups);
  AVD_CHECK_LAUNCH();
  return 1;
}
