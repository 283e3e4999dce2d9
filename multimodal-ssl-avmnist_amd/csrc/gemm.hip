// Dense layers: f32 GEMM with arbitrary strides for nn.Linear forward (x W^T + b), input
// gradient (dy W) and weight gradient (dy^T x, with the bias gradient = row sums of dy^T
// produced by the same launch).  Layers: CentralMultiModalEncoder's image/audio Linear and
// fusion MLP (dino.py:222-227, 459-468), ProjectionHead (dino.py:1240-1254).
//
// v1: LDS-tiled 64x64x16 tiles, 256 threads, 4x4 outputs per thread, fp32 FMA (bitwise
// deterministic: no split-K).
#include <algorithm>

#include "common.h"

using namespace avd;

namespace {

constexpr int BM = 64, BN = 64, BK = 16;

__global__ __launch_bounds__(256) void sgemm_kernel(int M, int N, int K, const float* __restrict__ A,
                                                    long long sam, long long sak,
                                                    const float* __restrict__ B, long long sbk,
                                                    long long sbn, float* __restrict__ C,
                                                    long long ldc, const float* __restrict__ bias,
                                                    float alpha, float beta, float* a_rowsum) {
  __shared__ float As[BK][BM + 4];
  __shared__ float Bs[BK][BN + 4];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const bool a_kfast = (sak == 1);
  const bool b_nfast = (sbn == 1);
  const bool want_rs = a_rowsum && blockIdx.x == 0;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  float rs = 0.f;

  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      int mm, kk;
      if (a_kfast) { kk = e & 15; mm = e >> 4; } else { mm = e & 63; kk = e >> 6; }
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? A[(size_t)gm * sam + (size_t)gk * sak] : 0.f;
      int nn;
      if (b_nfast) { nn = e & 63; kk = e >> 6; } else { kk = e & 15; nn = e >> 4; }
      const int gn = n0 + nn;
      const int gk2 = k0 + kk;
      Bs[kk][nn] = (gn < N && gk2 < K) ? B[(size_t)gk2 * sbk + (size_t)gn * sbn] : 0.f;
    }
    __syncthreads();
    if (want_rs && tid < BM) {
#pragma unroll
      for (int kk = 0; kk < BK; ++kk) rs += As[kk][tid];
    }
#pragma unroll
    for (int kk = 0; kk < BK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty + 16 * i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx + 16 * j;
      if (n >= N) continue;
      float v = alpha * acc[i][j];
      if (bias) v += bias[n];
      float* c = C + (size_t)m * ldc + n;
      if (beta != 0.f) v += beta * *c;
      *c = v;
    }
  }
  if (want_rs && tid < BM && m0 + tid < M) a_rowsum[m0 + tid] = rs;
}

// ---------------------------------------------------------------------------------------
// MFMA GEMM.  MODE 1: v_mfma_f32_16x16x4_f32 (f32 operands: exact f32 FMA chains, the fp32
// parity mode); MODE 2: v_mfma_f32_16x16x32_bf16 (operands rounded to bf16 while staging,
// fp32 accumulate: the bf16 training mode, like the reference's fp16 autocast Linear).
//
// Block tile BM x BN (128x128, 128x64 or 64x64), BK 32, 4 waves in a 2x2 grid, each wave
// (BM/2)x(BN/2) = TI x TJ MFMA 16x16 tiles.  Operands live in LDS k-contiguous ([m][k] for A,
// [n][k] for B) so every fragment is one LDS read.  Software pipeline: the next k-tile is
// loaded into registers (float4 whenever a stride is 1) while the current one feeds the
// MFMAs, then written to the other half of a double-buffered LDS ring -> one barrier per
// k-tile.  Split-K (blockIdx.z) writes raw partial tiles to a workspace that a second kernel
// sums in fixed split order: deterministic, no atomics.
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;

template <int MODE>
struct GemmT { typedef float T; static constexpr int LDK = 33; };
template <>
struct GemmT<2> { typedef bf16 T; static constexpr int LDK = 40; };

// Operand layouts of a (rows x 32) tile of X with element (r, k) at X[r*sr + k*sk]:
// LAY_K: k contiguous & 16B aligned rows (float4 along k); LAY_R: rows contiguous (float4 along
// r); LAY_S: anything else (scalar).
enum { LAY_K = 0, LAY_R = 1, LAY_S = 2 };

template <int ROWS>
struct TileRegs { float v[ROWS / 8 > 16 ? ROWS / 8 : 16]; };   // ROWS*32 elements over 256 threads

template <int ROWS, int LAY, bool EX = false>
__device__ __forceinline__ void load_tile(const float* __restrict__ X, long long sr, long long sk,
                                          int r0, int k0, int rows, int kend, TileRegs<ROWS>& t) {
  const int tid = threadIdx.x;
  if constexpr (EX && LAY == LAY_K) {
    // whole tiles (the caller checked): unconditional loads, so the wait for one register stage
    // leaves the younger stages' loads in flight (no branch for the waitcnt pass to merge over)
#pragma unroll
    for (int i = 0; i < ROWS / 32; ++i) {
      const int e4 = tid + 256 * i;
      const int r = e4 >> 3, k = (e4 & 7) * 4;
      const float4 v = *reinterpret_cast<const float4*>(X + (size_t)(r0 + r) * sr + k0 + k);
      t.v[4 * i] = v.x; t.v[4 * i + 1] = v.y; t.v[4 * i + 2] = v.z; t.v[4 * i + 3] = v.w;
    }
  } else if constexpr (EX && LAY == LAY_R) {
#pragma unroll
    for (int i = 0; i < (ROWS + 127) / 128; ++i) {
      const int b = tid + 256 * i;
      const int kb = b / (ROWS / 4), r = (b % (ROWS / 4)) * 4;
      if (ROWS >= 128 || b < 2 * ROWS) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const float4 v = *reinterpret_cast<const float4*>(X + (size_t)(k0 + 4 * kb + kk) * sk + r0 + r);
          t.v[16 * i + kk] = v.x; t.v[16 * i + 4 + kk] = v.y;
          t.v[16 * i + 8 + kk] = v.z; t.v[16 * i + 12 + kk] = v.w;
        }
      }
    }
  } else if constexpr (LAY == LAY_K) {
#pragma unroll
    for (int i = 0; i < ROWS / 32; ++i) {
      const int e4 = tid + 256 * i;
      const int r = e4 >> 3, k = (e4 & 7) * 4;
      const int gr = r0 + r, gk = k0 + k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gr < rows) {
        const float* p = X + (size_t)gr * sr + gk;
        if (gk + 3 < kend) v = *reinterpret_cast<const float4*>(p);
        else {
          if (gk < kend) v.x = p[0];
          if (gk + 1 < kend) v.y = p[1];
          if (gk + 2 < kend) v.z = p[2];
        }
      }
      t.v[4 * i] = v.x; t.v[4 * i + 1] = v.y; t.v[4 * i + 2] = v.z; t.v[4 * i + 3] = v.w;
    }
  } else if constexpr (LAY == LAY_R) {
    // a 4 (k) x 4 (rows) block per thread: four float4 loads along the rows, transposed in
    // registers so store_tile writes 4 consecutive k of a row at once
#pragma unroll
    for (int i = 0; i < (ROWS + 127) / 128; ++i) {
      const int b = tid + 256 * i;
      const int kb = b / (ROWS / 4), r = (b % (ROWS / 4)) * 4;
      const int gr = r0 + r;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int gk = k0 + 4 * kb + kk;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (b < 2 * ROWS && gk < kend) {
          const float* p = X + (size_t)gk * sk + gr;
          if (gr + 3 < rows) v = *reinterpret_cast<const float4*>(p);
          else {
            if (gr < rows) v.x = p[0];
            if (gr + 1 < rows) v.y = p[1];
            if (gr + 2 < rows) v.z = p[2];
          }
        }
        t.v[16 * i + kk] = v.x; t.v[16 * i + 4 + kk] = v.y;
        t.v[16 * i + 8 + kk] = v.z; t.v[16 * i + 12 + kk] = v.w;
      }
    }
  } else {
    const bool kfast = sk <= sr;
#pragma unroll
    for (int i = 0; i < ROWS / 8; ++i) {
      const int e = tid + 256 * i;
      int r, k;
      if (kfast) { r = e >> 5; k = e & 31; } else { k = e / ROWS; r = e % ROWS; }
      const int gr = r0 + r, gk = k0 + k;
      t.v[i] = (gr < rows && gk < kend) ? X[(size_t)gr * sr + (size_t)gk * sk] : 0.f;
    }
  }
}

template <int MODE>
__device__ __forceinline__ void lds_put(typename GemmT<MODE>::T* p, float v) {
  if constexpr (MODE == 2) *p = f2bf(v); else *p = v;
}

template <int MODE, int ROWS, int LAY>
__device__ __forceinline__ void store_tile(const TileRegs<ROWS>& t, long long sr, long long sk,
                                           typename GemmT<MODE>::T* S) {
  constexpr int LDK = GemmT<MODE>::LDK;
  const int tid = threadIdx.x;
  if constexpr (LAY == LAY_K) {
#pragma unroll
    for (int i = 0; i < ROWS / 32; ++i) {
      const int e4 = tid + 256 * i;
      const int r = e4 >> 3, k = (e4 & 7) * 4;
      typename GemmT<MODE>::T* d = S + r * LDK + k;
      if constexpr (MODE == 2) {
        // 4 bf16 = one 8-byte LDS store
        const unsigned lo = pack_bf16x2(t.v[4 * i], t.v[4 * i + 1]);
        const unsigned hi = pack_bf16x2(t.v[4 * i + 2], t.v[4 * i + 3]);
        *reinterpret_cast<uint2*>(d) = make_uint2(lo, hi);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = t.v[4 * i + j];
      }
    }
  } else if constexpr (LAY == LAY_R) {
#pragma unroll
    for (int i = 0; i < (ROWS + 127) / 128; ++i) {
      const int b = tid + 256 * i;
      if (b >= 2 * ROWS) continue;
      const int kb = b / (ROWS / 4), r = (b % (ROWS / 4)) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        typename GemmT<MODE>::T* d = S + (r + j) * LDK + 4 * kb;
        const float* v = &t.v[16 * i + 4 * j];
        if constexpr (MODE == 2) {
          *reinterpret_cast<uint2*>(d) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        } else {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) d[kk] = v[kk];
        }
      }
    }
  } else {
    const bool kfast = sk <= sr;
#pragma unroll
    for (int i = 0; i < ROWS / 8; ++i) {
      const int e = tid + 256 * i;
      int r, k;
      if (kfast) { r = e >> 5; k = e & 31; } else { k = e / ROWS; r = e % ROWS; }
      lds_put<MODE>(S + r * LDK + k, t.v[i]);
    }
  }
}

// register prefetch depth: deeper for the small tiles (the heads' latency-bound GEMMs), within
// the VGPR budget of the large ones (128x256: 48 + 128 accumulator registers per stage set)
template <int BM, int BN>
struct Depth { static constexpr int P = BM * BN >= 128 * 256 ? 1 : (BM * BN >= 128 * 64 ? 2 : 4); };

template <int MODE, int BM, int BN, int LA, int LB, bool EX = false,
          int P = EX ? Depth<BM, BN>::P : 1>
__global__ __launch_bounds__(256) void gemm_mfma_kernel(
    int M, int N, int K, int kchunk, const float* __restrict__ A, long long sam, long long sak,
    const float* __restrict__ B, long long sbk, long long sbn, float* __restrict__ C, long long ldc,
    const float* __restrict__ bias, float alpha, float beta, float* __restrict__ ws) {
  typedef typename GemmT<MODE>::T T;
  constexpr int LDK = GemmT<MODE>::LDK;
  constexpr int TI = BM / 32, TJ = BN / 32;   // MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) T As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LDK];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  f4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // P register stages of k-tiles in flight: tile kt+P is loaded while tile kt is stored to LDS
  // and multiplied (the loop is latency-bound otherwise: one HBM round trip per 32-deep k-tile)
  TileRegs<BM> ta[P];
  TileRegs<BN> tb[P];
  const int nk = (kend - kbeg + 31) / 32;
  // EX: every tile whole; loads past the last k-tile re-read the last one (clamped, never used)
  auto kt_at = [&](int kt) { return kbeg + 32 * (EX ? min(kt, nk - 1) : kt); };
#pragma unroll
  for (int p = 0; p < P; ++p)
    if (EX || p < nk) {
      load_tile<BM, LA, EX>(A, sam, sak, m0, kt_at(p), M, kend, ta[p]);
      load_tile<BN, LB, EX>(B, sbn, sbk, n0, kt_at(p), N, kend, tb[p]);   // B^T tile: rows = n
    }
  for (int kt0 = 0; kt0 < nk; kt0 += P) {
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int kt = kt0 + p;
    if (kt >= nk) break;
    const int cur = kt & 1;
    // buffer cur was last read by tile kt-2's MFMAs, which every wave finished before the
    // barrier of tile kt-1
    store_tile<MODE, BM, LA>(ta[p], sam, sak, As[cur]);
    store_tile<MODE, BN, LB>(tb[p], sbn, sbk, Bs[cur]);
    __syncthreads();
    if (EX || kt + P < nk) {
      load_tile<BM, LA, EX>(A, sam, sak, m0, kt_at(kt + P), M, kend, ta[p]);
      load_tile<BN, LB, EX>(B, sbn, sbk, n0, kt_at(kt + P), N, kend, tb[p]);
    }
    const T* as = As[cur] + (BM / 2 * wm + r16) * LDK;
    const T* bs = Bs[cur] + (BN / 2 * wn + r16) * LDK;
    if constexpr (MODE == 2) {
      bf16x8 a[TI], b[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(as + 16 * i * LDK + 8 * g);
#pragma unroll
      for (int j = 0; j < TJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bs + 16 * j * LDK + 8 * g);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        float a[TI], b[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) a[i] = as[16 * i * LDK + 4 * ks + g];
#pragma unroll
        for (int j = 0; j < TJ; ++j) b[j] = bs[16 * j * LDK + 4 * ks + g];
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  }
  float* part = ws ? ws + (size_t)blockIdx.z * M * N : nullptr;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = n0 + BN / 2 * wn + 16 * j + r16;
      if (n >= N) continue;
      const float bv = (!part && bias) ? bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + BM / 2 * wm + 16 * i + 4 * g + e;
        if (m >= M) continue;
        if (part) {
          part[(size_t)m * N + n] = acc[i][j][e];
        } else {
          float* c = C + (size_t)m * ldc + n;
          float v = alpha * acc[i][j][e] + bv;
          if (beta != 0.f) v += beta * *c;
          *c = v;
        }
      }
    }
}

// C = alpha * sum_{z < S} ws[z] (+bias) (+beta C), fixed split order
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S,
                                                            int M, int N, float* __restrict__ C,
                                                            long long ldc,
                                                            const float* __restrict__ bias,
                                                            float alpha, float beta) {
  const long long MN = (long long)M * N;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < MN; i += (long long)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += ws[(size_t)z * MN + i];
    const int m = (int)(i / N), n = (int)(i % N);
    float* c = C + (size_t)m * ldc + n;
    float v = alpha * s + (bias ? bias[n] : 0.f);
    if (beta != 0.f) v += beta * *c;
    *c = v;
  }
}

int lay_of(const float* p, long long s_rows, long long s_k) {
  const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  if (s_k == 1 && s_rows % 4 == 0 && al) return LAY_K;
  if (s_rows == 1 && s_k % 4 == 0 && al) return LAY_R;
  return LAY_S;
}

// Launch plan: the largest tile whose grid still covers the chip; deep-K products with few
// tiles (weight gradients: K = batch rows) split K so >= ~2 blocks per CU run.
struct Plan { int bm, bn, splits, kchunk; };

Plan plan_for(int M, int N, int K) {
  auto tiles = [&](int bm, int bn) { return (long long)avd_cdiv(M, bm) * avd_cdiv(N, bn); };
  // encoder Linear forward (x [rows, 1600 / 3136] x W^T, N = 256): one 256-wide column tile so
  // the f32 activations stream from HBM once (128x64 tiles re-read them 4x), split-K for blocks
  if (N > 128 && N <= 256 && K >= 1024 && M >= 4096) {
    Plan p{128, 256, 1, K};
    const long long t = tiles(128, 256);
    const int s = (int)std::max(1ll, std::min<long long>(avd_cdiv(224, t), K / 128));
    if (s > 1) {
      p.kchunk = avd_cdiv(avd_cdiv(K, s), 32) * 32;
      p.splits = avd_cdiv(K, p.kchunk);
    }
    return p;
  }
  Plan p{64, 64, 1, K};
  if (tiles(128, 128) >= 224) p = {128, 128, 1, K};
  else if (tiles(128, 64) >= 224) p = {128, 64, 1, K};
  else if (K >= 1024)   // deep K: the split below restores the block count
    p = (M >= 128 && N >= 128) ? Plan{128, 128, 1, K} : (M >= 128 ? Plan{128, 64, 1, K} : p);
  const long long t = tiles(p.bm, p.bn);
  // split target (blocks) and minimum K rows per split: AVDINO_GEMM_SPLIT / AVDINO_GEMM_KMIN
  static const int target = getenv("AVDINO_GEMM_SPLIT") ? atoi(getenv("AVDINO_GEMM_SPLIT")) : 512;
  static const int kmin = getenv("AVDINO_GEMM_KMIN") ? atoi(getenv("AVDINO_GEMM_KMIN")) : 256;
  if (t < 224 && K >= 512) {
    int s = (int)std::min<long long>(avd_cdiv(target, t), K / kmin);
    s = std::max(1, std::min(s, 128));
    if (s > 1) {
      p.kchunk = avd_cdiv(avd_cdiv(K, s), 32) * 32;
      p.splits = avd_cdiv(K, p.kchunk);
    }
  }
  return p;
}

template <int MODE, int LA, int LB>
void launch_gemm(const Plan& pl, int M, int N, int K, const float* A, long long sam, long long sak,
                 const float* B, long long sbk, long long sbn, float* C, long long ldc,
                 const float* bias, float alpha, float beta, float* ws, hipStream_t st) {
  dim3 grid(avd_cdiv(N, pl.bn), avd_cdiv(M, pl.bm), pl.splits);
  float* w = pl.splits > 1 ? ws : nullptr;
  // whole tiles in every dimension (vector layouts, 16-byte aligned strides): the deep
  // register-prefetch variant (AVDINO_GEMM_EX=1)
  // (measured no faster than the checked variant at the step's shapes, profiles/r3_gemm_ab.txt: off)
  static const bool ex_on = getenv("AVDINO_GEMM_EX") && atoi(getenv("AVDINO_GEMM_EX")) != 0;
  const bool ex = ex_on && LA != LAY_S && LB != LAY_S && M % pl.bm == 0 && N % pl.bn == 0 &&
                  K % 32 == 0 && pl.kchunk % 32 == 0;
#define AVD_G(BM_, BN_)                                                                        \
  if (pl.bm == BM_ && pl.bn == BN_) {                                                          \
    if (ex)                                                                                    \
      gemm_mfma_kernel<MODE, BM_, BN_, LA, LB, true><<<grid, 256, 0, st>>>(                    \
          M, N, K, pl.kchunk, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha, beta, w);         \
    else                                                                                       \
      gemm_mfma_kernel<MODE, BM_, BN_, LA, LB, false><<<grid, 256, 0, st>>>(                   \
          M, N, K, pl.kchunk, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha, beta, w);         \
  }
  AVD_G(128, 256) else AVD_G(128, 128) else AVD_G(128, 64) else AVD_G(64, 64)
#undef AVD_G
  if (pl.splits > 1) {
    const long long MN = (long long)M * N;
    const int blocks = (int)std::min<long long>(avd_cdiv(MN, 256), 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>(ws, pl.splits, M, N, C, ldc, bias, alpha, beta);
  }
}

// operand layouts are template parameters (the index math of the others would otherwise sit in
// registers): K/R combinations get vector loads, anything with a scalar operand the generic path
template <int MODE>
void dispatch_gemm(const Plan& pl, int lA, int lB, int M, int N, int K, const float* A,
                   long long sam, long long sak, const float* B, long long sbk, long long sbn,
                   float* C, long long ldc, const float* bias, float alpha, float beta, float* ws,
                   hipStream_t st) {
#define AVD_L(LA_, LB_) launch_gemm<MODE, LA_, LB_>(pl, M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, \
                                                   bias, alpha, beta, ws, st)
  if (lA == LAY_K && lB == LAY_K) AVD_L(LAY_K, LAY_K);
  else if (lA == LAY_K && lB == LAY_R) AVD_L(LAY_K, LAY_R);
  else if (lA == LAY_R && lB == LAY_R) AVD_L(LAY_R, LAY_R);
  else if (lA == LAY_R && lB == LAY_K) AVD_L(LAY_R, LAY_K);
  else AVD_L(LAY_S, LAY_S);
#undef AVD_L
}

}  // namespace

extern "C" {

long long avd_gemm_ws_elems(int M, int N, int K, int mode) {
  if (mode != 1 && mode != 2) return 0;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const Plan p = plan_for(M, N, K);
  return p.splits > 1 ? (long long)p.splits * M * N : 0;
}

int avd_gemm(int M, int N, int K, const float* A, long long sam, long long sak, const float* B,
             long long sbk, long long sbn, float* C, long long ldc, const float* bias, float alpha,
             float beta, int mode, float* ws, long long ws_elems, void* stream) {
  if (!A || !B || !C) return AVD_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
  if (mode == 0) {
    dim3 grid(avd_cdiv(N, 64), avd_cdiv(M, 64));
    sgemm_kernel<<<grid, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha,
                                        beta, nullptr);
  } else if (mode == 1 || mode == 2) {
    Plan pl = plan_for(M, N, K);
    if (pl.splits > 1 && (!ws || ws_elems < (long long)pl.splits * M * N)) {
      pl.splits = 1;   // no (or too small a) workspace: single pass over K
      pl.kchunk = K;
    }
    const int lA = lay_of(A, sam, sak);
    const int lB = lay_of(B, sbn, sbk);
    if (mode == 1)
      dispatch_gemm<1>(pl, lA, lB, M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha, beta, ws, st);
    else
      dispatch_gemm<2>(pl, lA, lB, M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha, beta, ws, st);
  } else {
    return AVD_ERR_ARG;
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
