// Dense layers: f32 GEMM with arbitrary strides for nn.Linear forward (x W^T + b), input
// gradient (dy W) and weight gradient (dy^T x, with the bias gradient = row sums of dy^T
// produced by the same launch).  Layers: CentralMultiModalEncoder's image/audio Linear and
// fusion MLP (dino.py:222-227, 459-468), ProjectionHead (dino.py:1240-1254).
//
// v1: LDS-tiled 64x64x16 tiles, 256 threads, 4x4 outputs per thread, fp32 FMA (bitwise
// deterministic: no split-K).
#include <algorithm>
#include <type_traits>

#include "common.h"

using namespace avd;

namespace {

__device__ __forceinline__ int avd_cdiv_d(int a, int b) { return (a + b - 1) / b; }

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
// Block tile BM x BN (128x128, 128x64 or 64x64), BK 32 (f32) / 64 (bf16), 4 waves in a 2x2 grid, each wave
// (BM/2)x(BN/2) = TI x TJ MFMA 16x16 tiles.  Operands live in LDS k-contiguous ([m][k] for A,
// [n][k] for B) so every fragment is one LDS read.  Software pipeline: the next k-tile is
// loaded into registers (float4 whenever a stride is 1) while the current one feeds the
// MFMAs, then written to the other half of a double-buffered LDS ring -> one barrier per
// k-tile.  Split-K (blockIdx.z) writes raw partial tiles to a workspace that a second kernel
// sums in fixed split order: deterministic, no atomics.
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;

template <int MODE>
struct GemmT { typedef float T; static constexpr int LDK = 33, BK = 32; };
template <>
struct GemmT<2> { typedef bf16 T; static constexpr int LDK = 64, BK = 64; };

// bf16 tiles (BK 64): 128-byte rows, the 16-byte chunk c of row r stored at chunk c ^ ((r >> 1) & 7).
// The MFMA fragment reads (16 rows x one chunk per 16 lanes, ds_read_b128) and the staging
// writes are then bank-conflict free (tools/lds_conflicts.py gemm).
__device__ __forceinline__ int gsw(int r, int k) { return r * 64 + (((k >> 3) ^ ((r >> 1) & 7)) << 3) + (k & 7); }

// Operand layouts of a (rows x BK) tile of X with element (r, k) at X[r*sr + k*sk]:
// LAY_K: k contiguous & 16B aligned rows (float4 along k); LAY_R: rows contiguous (float4 along
// r); LAY_S: anything else (scalar).
enum { LAY_K = 0, LAY_R = 1, LAY_S = 2 };

// f32 staging registers of a ROWS x BK tile over 256 threads (LAY_R: 4x4 blocks, 16 per pass)
template <int ROWS, int BK>
struct TileRegs {
  static constexpr int NK = ROWS * BK / 256;
  static constexpr int NR = 16 * ((ROWS * BK / 16 + 255) / 256);
  float v[NK > NR ? NK : NR];
};

// f32 operand loads (bf16 operands go through the raw Stage specialisations below)
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// 16 zero bytes the out-of-range lanes of a k-tile load read instead of their operand: the
// loads then need neither a per-lane branch nor a select on the loaded value (either makes the
// compiler wait for the load right where it is issued)
__device__ uint4 g_zero16 = {0u, 0u, 0u, 0u};   // (global, not constant, address space: loads stay global_load)
template <typename S>
__device__ __forceinline__ const S* zero16() { return reinterpret_cast<const S*>(&g_zero16); }
__device__ __forceinline__ float ld1(const float* p) { return *p; }

// LAY_R row-block order: bits 0 and 1 swapped (row blocks 2m, 2m + 1 of the lane order sit
// 8 rows apart)
__device__ __forceinline__ int lrb(int q) { return (q & ~3) | ((q & 1) << 1) | ((q >> 1) & 1); }

template <int ROWS, int BK, int LAY, typename S = float>
__device__ __forceinline__ void load_tile(const S* __restrict__ X, long long sr, long long sk,
                                          int r0, int k0, int rows, int kend, TileRegs<ROWS, BK>& t) {
  const int tid = threadIdx.x;
  if constexpr (LAY == LAY_K) {
    constexpr int KV = BK / 4;                        // float4 per tile row
#pragma unroll
    for (int i = 0; i < ROWS * KV / 256; ++i) {
      const int e4 = tid + 256 * i;
      const int r = e4 / KV, k = (e4 % KV) * 4;
      const int gr = r0 + r, gk = k0 + k;
      // whole-vector bounds (the host serves LAY_K only for k extents % 4 == 0): an
      // out-of-range lane reads g_zero16 -- no per-lane branch, so the compiler can count the
      // k-tile's loads exactly (s_waitcnt vmcnt(n), not vmcnt(0))
      const bool ok = gr < rows && gk < kend;
      const float4 v = ld4(ok ? X + (size_t)gr * sr + gk : zero16<S>());
      t.v[4 * i] = v.x; t.v[4 * i + 1] = v.y; t.v[4 * i + 2] = v.z; t.v[4 * i + 3] = v.w;
    }
  } else if constexpr (LAY == LAY_R) {
    // a 4 (k) x 4 (rows) block per thread: four float4 loads along the rows, transposed in
    // registers so store_tile writes 4 consecutive k of a row at once.  Block b: k-block
    // b & 7 of the 32-k half b / (8 * ROWS / 4), row block lrb((b >> 3) % (ROWS / 4)): 8 lanes
    // cover one row's 32 k and the next 8 lanes rows 8 further on (lrb swaps bits 0 and 1), so a
    // 16-lane group of 8-byte LDS writes covers both 64-byte halves of the 128-byte bank row
    // (tools/lds_conflicts.py gemm); a wave still reads whole 128-byte row segments
    constexpr int NB = ROWS * BK / 16;
#pragma unroll
    for (int i = 0; i < (NB + 255) / 256; ++i) {
      const int b = tid + 256 * i;
      const int kb = b & 7, rest = b >> 3;
      const int r = lrb(rest % (ROWS / 4)) * 4, kh = rest / (ROWS / 4);
      const int gr = r0 + r;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int gk = k0 + 32 * kh + 4 * kb + kk;
        // whole-vector bounds (LAY_R only for row extents % 4 == 0), branch-free as LAY_K
        const bool ok = b < NB && gk < kend && gr < rows;
        const float4 v = ld4(ok ? X + (size_t)gk * sk + gr : zero16<S>());
        t.v[16 * i + kk] = v.x; t.v[16 * i + 4 + kk] = v.y;
        t.v[16 * i + 8 + kk] = v.z; t.v[16 * i + 12 + kk] = v.w;
      }
    }
  } else {
    const bool kfast = sk <= sr;
#pragma unroll
    for (int i = 0; i < ROWS * BK / 256; ++i) {
      const int e = tid + 256 * i;
      int r, k;
      if (kfast) { r = e / BK; k = e % BK; } else { k = e / ROWS; r = e % ROWS; }
      const int gr = r0 + r, gk = k0 + k;
      t.v[i] = (gr < rows && gk < kend) ? ld1(X + (size_t)gr * sr + (size_t)gk * sk) : 0.f;
    }
  }
}

template <int MODE>
__device__ __forceinline__ void lds_put(typename GemmT<MODE>::T* p, float v) {
  if constexpr (MODE == 2) *p = f2bf(v); else *p = v;
}

template <int MODE, int ROWS, int LAY>
__device__ __forceinline__ void store_tile(const TileRegs<ROWS, GemmT<MODE>::BK>& t, long long sr,
                                           long long sk, typename GemmT<MODE>::T* S) {
  constexpr int LDK = GemmT<MODE>::LDK, BK = GemmT<MODE>::BK;
  const int tid = threadIdx.x;
  if constexpr (LAY == LAY_K) {
    constexpr int KV = BK / 4;
#pragma unroll
    for (int i = 0; i < ROWS * KV / 256; ++i) {
      const int e4 = tid + 256 * i;
      const int r = e4 / KV, k = (e4 % KV) * 4;
      typename GemmT<MODE>::T* d = S + (MODE == 2 ? gsw(r, k) : r * LDK + k);
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
    constexpr int NB = ROWS * BK / 16;
#pragma unroll
    for (int i = 0; i < (NB + 255) / 256; ++i) {
      const int b = tid + 256 * i;
      // (wave-uniform: a scalar branch keeps the k-tile's load counting exact)
      if (NB % 256 != 0 && __builtin_amdgcn_readfirstlane(b) >= NB) continue;
      const int kb = b & 7, rest = b >> 3;                      // as load_tile<LAY_R>
      const int r = lrb(rest % (ROWS / 4)) * 4, k = 32 * (rest / (ROWS / 4)) + 4 * kb;
      if constexpr (MODE == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float* v = &t.v[16 * i + 4 * j];
          *reinterpret_cast<uint2*>(S + gsw(r + j, k)) =
              make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          typename GemmT<MODE>::T* d = S + (r + j) * LDK + k;
          const float* v = &t.v[16 * i + 4 * j];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) d[kk] = v[kk];
        }
      }
    }
  } else {
    const bool kfast = sk <= sr;
#pragma unroll
    for (int i = 0; i < ROWS * BK / 256; ++i) {
      const int e = tid + 256 * i;
      int r, k;
      if (kfast) { r = e / BK; k = e % BK; } else { k = e / ROWS; r = e % ROWS; }
      lds_put<MODE>(S + (MODE == 2 ? gsw(r, k) : r * LDK + k), t.v[i]);
    }
  }
}

// Staging of one operand tile (ROWS x BK k) from HBM through registers into the LDS ring.  f32
// sources (and bf16 ones in the f32 MFMA mode) go through TileRegs as floats; bf16 sources in the
// bf16 mode are copied raw, 16 bytes per load (8-byte accesses run at 0.54-0.70x the 16-byte rate,
// MI355X_MICROARCH.md): k-contiguous rows as 16-byte chunks straight into their swizzled LDS
// chunk, row-contiguous (LAY_R) ones as 8 rows x 4 k per thread transposed in registers.
template <int MODE, int ROWS, int LAY, typename S,
          bool RAW = (MODE == 2 && std::is_same<S, bf16>::value && LAY != LAY_S)>
struct Stage {
  TileRegs<ROWS, GemmT<MODE>::BK> t;
  __device__ __forceinline__ void load(const S* __restrict__ X, long long sr, long long sk, int r0,
                                       int k0, int rows, int kend) {
    load_tile<ROWS, GemmT<MODE>::BK, LAY, S>(X, sr, sk, r0, k0, rows, kend, t);
  }
  __device__ __forceinline__ void store(long long sr, long long sk, typename GemmT<MODE>::T* dst) {
    store_tile<MODE, ROWS, LAY>(t, sr, sk, dst);
  }
};

// raw bf16 staging registers: a native vector (HIP's uint4 class copies through memory when
// loaded from a selected pointer)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned hw16(const u32x4& v, int j) {
  const unsigned w = j < 2 ? v.x : j < 4 ? v.y : j < 6 ? v.z : v.w;
  return (j & 1) ? (w >> 16) : (w & 0xffffu);
}

// (raw stages exist in the bf16 mode only: BK 64, 8 chunks per tile row)
template <int MODE, int ROWS, typename S>
struct Stage<MODE, ROWS, LAY_K, S, true> {
  static constexpr int NV = ROWS * 8 / 256 > 0 ? ROWS * 8 / 256 : 1;   // 16-byte chunks per thread
  u32x4 v[NV];
  __device__ __forceinline__ void load(const S* __restrict__ X, long long sr, long long, int r0,
                                       int k0, int rows, int kend) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = (int)threadIdx.x + 256 * i;
      const int r = e >> 3, kc = e & 7;
      const int gr = r0 + r, gk = k0 + 8 * kc;
      // whole 16-byte chunks (bf16 operands need k extents % 8 == 0), branch-free
      const bool ok = r < ROWS && gr < rows && gk < kend;
      const bf16* p = ok ? reinterpret_cast<const bf16*>(X) + (size_t)gr * sr + gk : zero16<bf16>();
      v[i] = *reinterpret_cast<const u32x4*>(p);
    }
  }
  __device__ __forceinline__ void store(long long, long long, typename GemmT<MODE>::T* dst) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = (int)threadIdx.x + 256 * i;
      const int r = e >> 3, kc = e & 7;
      if (ROWS >= 32 || r < ROWS) *reinterpret_cast<u32x4*>(dst + gsw(r, 8 * kc)) = v[i];
    }
  }
};

template <int MODE, int ROWS, typename S>
struct Stage<MODE, ROWS, LAY_R, S, true> {
  static_assert(ROWS <= 256 && ROWS % 64 == 0, "LAY_R raw tile");
  static constexpr int RG = ROWS / 8;                 // 8-row groups; thread = (kq, rg), kq < 16
  static constexpr int IT = (16 * RG + 255) / 256;    // passes over the 256 threads
  static constexpr int LG = RG == 8 ? 0 : RG == 16 ? 1 : 2;
  u32x4 v[4 * IT];
  // thread b: row group (b & 7) | (b >> 4 & (RG / 8 - 1)) << 3, k-quad (b >> 3 & 1) | (b >> (4 + LG)) << 1:
  // a 16-lane group writes 8 row groups x both 8-byte halves of one k chunk, which the rotated
  // row order spreads over all 32 banks (tools/lds_conflicts.py gemm); a wave reads 16 row
  // groups' 16 bytes = 256 contiguous bytes per k row
  __device__ __forceinline__ static int rg_of(int b) { return (b & 7) | (((b >> 4) & (RG / 8 - 1)) << 3); }
  __device__ __forceinline__ static int kq_of(int b) { return ((b >> 3) & 1) | ((b >> (4 + LG)) << 1); }
  __device__ __forceinline__ void load(const S* __restrict__ X, long long, long long sk, int r0,
                                       int k0, int rows, int kend) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int b = (int)threadIdx.x + 256 * it;
      const int rg = rg_of(b), kq = kq_of(b);
      const int gr = r0 + 8 * rg;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int gk = k0 + 4 * kq + kk;
        // whole 16-byte chunks (row extents % 8 == 0), branch-free
        const bool ok = b < 16 * RG && gk < kend && gr < rows;
        const bf16* p = ok ? reinterpret_cast<const bf16*>(X) + (size_t)gk * sk + gr : zero16<bf16>();
        v[4 * it + kk] = *reinterpret_cast<const u32x4*>(p);
      }
    }
  }
  __device__ __forceinline__ void store(long long, long long, typename GemmT<MODE>::T* dst) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int b = (int)threadIdx.x + 256 * it;
      if ((16 * RG) % 256 != 0 && __builtin_amdgcn_readfirstlane(b) >= 16 * RG) continue;   // whole waves
      const int rg = rg_of(b), kq = kq_of(b);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = (jj + rg) & 7;            // rotated per row group: the 16-lane write groups
        const unsigned lo = hw16(v[4 * it], j) | hw16(v[4 * it + 1], j) << 16;   // spread over the banks
        const unsigned hi = hw16(v[4 * it + 2], j) | hw16(v[4 * it + 3], j) << 16;
        *reinterpret_cast<uint2*>(dst + gsw(8 * rg + j, 4 * kq)) = make_uint2(lo, hi);
      }
    }
  }
};

// One GEMM problem of a launch (the paired launch carries two).
struct GemmArgs {
  int M, N, K, kchunk;
  const void* A;      // f32 or bf16 (the kernel's SA / SB template types)
  long long sam, sak;
  const void* B;
  long long sbk, sbn;
  void* C;            // f32, or bf16 when c_bf16
  long long ldc;
  const float* bias;
  float alpha, beta;
  float* ws;      // split-K partial tiles (nullptr: one pass over K)
  int c_bf16;     // C stored as bf16 (beta must be 0)
  int map_c;      // > 0: output column n lands at (n % map_c) * map_hw + n / map_c (an NHWC
  int map_hw;     //      (h, w, c) feature index -> the reference's (c, h, w) flatten index)
};

// the output element (m, n) of a problem: bias, alpha / beta, bf16 or f32, optional column map
__device__ __forceinline__ void gemm_out(const GemmArgs& p, int m, int n, float acc) {
  const float bv = p.bias ? p.bias[n] : 0.f;
  const int cn = p.map_c > 0 ? (n % p.map_c) * p.map_hw + n / p.map_c : n;
  if (p.c_bf16) {
    reinterpret_cast<bf16*>(p.C)[(size_t)m * p.ldc + cn] = f2bf(p.alpha * acc + bv);
  } else {
    float* c = reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + cn;
    float v = p.alpha * acc + bv;
    if (p.beta != 0.f) v += p.beta * *c;
    *c = v;
  }
}

// LDS bytes of one tile body: double-buffered A and B k-tiles
template <int MODE, int BM, int BN>
struct GemmLds {
  static constexpr int BYTES = 2 * (BM + BN) * GemmT<MODE>::LDK * (int)sizeof(typename GemmT<MODE>::T);
};

// One BM x BN output tile (tile column tn, tile row tm) over the k-chunk tz of problem p, staged
// through the LDS block `smem` (GemmLds bytes).
template <int MODE, int BM, int BN, int LA, int LB, typename SA = float, typename SB = float>
__device__ __forceinline__ void gemm_tile(const GemmArgs& p, int tn, int tm, int tz, char* smem) {
  typedef typename GemmT<MODE>::T T;
  constexpr int LDK = GemmT<MODE>::LDK, BK = GemmT<MODE>::BK;
  constexpr int TI = BM / 32, TJ = BN / 32;   // MFMA tiles per wave
  T (*As)[BM * LDK] = reinterpret_cast<T (*)[BM * LDK]>(smem);
  T (*Bs)[BN * LDK] = reinterpret_cast<T (*)[BN * LDK]>(smem + 2 * BM * LDK * sizeof(T));
  const int M = p.M, N = p.N, K = p.K;
  const SA* __restrict__ A = static_cast<const SA*>(p.A);
  const SB* __restrict__ B = static_cast<const SB*>(p.B);
  const long long sam = p.sam, sak = p.sak, sbk = p.sbk, sbn = p.sbn;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = tz * p.kchunk;
  const int kend = min(K, kbeg + p.kchunk);
  f4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  Stage<MODE, BM, LA, SA> ta;
  Stage<MODE, BN, LB, SB> tb;
  const int nk = (kend - kbeg + BK - 1) / BK;
  ta.load(A, sam, sak, m0, kbeg, M, kend);
  tb.load(B, sbn, sbk, n0, kbeg, N, kend);   // B^T tile: rows = n
  ta.store(sam, sak, As[0]);
  tb.store(sbn, sbk, Bs[0]);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      ta.load(A, sam, sak, m0, kbeg + BK * (kt + 1), M, kend);
      tb.load(B, sbn, sbk, n0, kbeg + BK * (kt + 1), N, kend);
    }
    const T* as = As[cur] + (BM / 2 * wm + r16) * LDK;
    const T* bs = Bs[cur] + (BN / 2 * wn + r16) * LDK;
    if constexpr (MODE == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 a[TI], b[TJ];
        // the swizzled chunk of k-chunk 4 ks + g (tile rows are r16 mod 16)
        const int gc = 8 * ((4 * ks + g) ^ ((r16 >> 1) & 7));
#pragma unroll
        for (int i = 0; i < TI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(as + 16 * i * LDK + gc);
#pragma unroll
        for (int j = 0; j < TJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bs + 16 * j * LDK + gc);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
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
    if (more) {
      ta.store(sam, sak, As[cur ^ 1]);
      tb.store(sbn, sbk, Bs[cur ^ 1]);
    }
    __syncthreads();
  }
  float* part = p.ws ? p.ws + (size_t)tz * M * N : nullptr;
  if constexpr (MODE == 2 && BM * BN * 2 <= GemmLds<MODE, BM, BN>::BYTES) {
    if (!part && p.c_bf16 && p.map_c == 0) {
      // bf16 output tile: staged in the (now idle) operand LDS as [BM][BN] with 16-byte chunks
      // XOR-swizzled by row, then written as 16-byte row segments (the MFMA layout would store
      // 2 bytes per lane, 32-byte segments per row)
      bf16* ts = reinterpret_cast<bf16*>(smem);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int nl = BN / 2 * wn + 16 * j + r16;
          const float bv = p.bias && n0 + nl < N ? p.bias[n0 + nl] : 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ml = BM / 2 * wm + 16 * i + 4 * g + e;
            ts[ml * BN + ((((nl >> 3) ^ (ml & 7)) << 3) | (nl & 7))] = f2bf(p.alpha * acc[i][j][e] + bv);
          }
        }
      __syncthreads();
      bf16* C = reinterpret_cast<bf16*>(p.C);
      for (int c = tid; c < BM * BN / 8; c += 256) {
        const int ml = c / (BN / 8), ch = c % (BN / 8);
        const int m = m0 + ml, n = n0 + 8 * ch;
        if (m >= M || n >= N) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(ts + ml * BN + ((ch ^ (ml & 7)) << 3));
        bf16* dst = C + (size_t)m * p.ldc + n;
        if (n + 7 < N && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
          *reinterpret_cast<uint4*>(dst) = v;
        } else {
          const unsigned w[4] = {v.x, v.y, v.z, v.w};
          for (int k = 0; k < 8 && n + k < N; ++k) dst[k] = (bf16)((w[k >> 1] >> (16 * (k & 1))) & 0xffffu);
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = n0 + BN / 2 * wn + 16 * j + r16;
      if (n >= N) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + BM / 2 * wm + 16 * i + 4 * g + e;
        if (m >= M) continue;
        if (part)
          part[(size_t)m * N + n] = acc[i][j][e];
        else
          gemm_out(p, m, n, acc[i][j][e]);
      }
    }
}

template <int MODE, int BM, int BN, int LA, int LB, typename SA = float, typename SB = float>
__global__ __launch_bounds__(256) void gemm_mfma_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[GemmLds<MODE, BM, BN>::BYTES];
  gemm_tile<MODE, BM, BN, LA, LB, SA, SB>(p, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// The bias gradient db[o] = sum_r dout[r, o] of a Linear backward, riding on the launches the
// weight gradient makes anyway: the paired GEMM launch's extra blocks write column partial sums
// of row chunks (block (chunk, 256-column strip)), the split-K reduce launch's extra blocks fold
// them in fixed chunk order.  Deterministic; two launches fewer per layer than avd_sum_rows_split.
struct DbArgs {
  const float* dout;
  long long ld;
  int rows, O, chunk, nrc, strips;
  float* part;   // [nrc][O]
  float* db;     // nullptr: no bias gradient in these launches
};

__device__ __forceinline__ void db_partial(const DbArgs& d, int b) {
  const int strip = b % d.strips, rc = b / d.strips, c = strip * 256 + (int)threadIdx.x;
  if (c >= d.O) return;
  const int r0 = rc * d.chunk, r1 = min(d.rows, r0 + d.chunk);
  const float* p = d.dout + (size_t)r0 * d.ld + c;
  float s = 0.f;
  for (int r = r0; r < r1; ++r, p += d.ld) s += *p;
  d.part[(size_t)rc * d.O + c] = s;
}

__device__ __forceinline__ void db_final(const DbArgs& d, int b) {
  const int c = b * 256 + (int)threadIdx.x;
  if (c >= d.O) return;
  // fixed chunk order; 4 loads in flight per step (the sum stays sequential)
  float s = 0.f;
  int rc = 0;
  for (; rc + 4 <= d.nrc; rc += 4) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = d.part[(size_t)(rc + u) * d.O + c];
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u];
  }
  for (; rc < d.nrc; ++rc) s += d.part[(size_t)rc * d.O + c];
  d.db[c] = s;
}

// Two independent problems in one grid (a Linear layer's weight gradient and input gradient
// both read dout): blocks [0, nb1) run problem 1 on its (n1 x m1 x z1) tile grid, the next nb2
// problem 2, and the last (when d.db) the bias gradient's chunk partials.  One launch boundary
// instead of three, and the small grids fill the chip together.
template <int MODE, int BM1, int BN1, int LA1, int LB1, int BM2, int BN2, int LA2, int LB2,
          typename SB = float>
__global__ __launch_bounds__(256) void gemm_pair_kernel(GemmArgs p1, int n1, int m1, GemmArgs p2,
                                                        int n2, int m2, DbArgs d) {
  constexpr int L1 = GemmLds<MODE, BM1, BN1>::BYTES, L2 = GemmLds<MODE, BM2, BN2>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[L1 > L2 ? L1 : L2];
  int b = blockIdx.x;
  const int nb1 = n1 * m1 * (p1.ws ? avd_cdiv_d(p1.K, p1.kchunk) : 1);
  const int nb2 = n2 * m2 * (p2.ws ? avd_cdiv_d(p2.K, p2.kchunk) : 1);
  if (b < nb1) {
    gemm_tile<MODE, BM1, BN1, LA1, LB1, float, SB>(p1, b % n1, (b / n1) % m1, b / (n1 * m1), smem);
  } else if (b < nb1 + nb2) {
    b -= nb1;
    gemm_tile<MODE, BM2, BN2, LA2, LB2, float, SB>(p2, b % n2, (b / n2) % m2, b / (n2 * m2), smem);
  } else {
    db_partial(d, b - nb1 - nb2);
  }
}

// C = alpha * sum_{z < S} ws[z] (+bias) (+beta C), fixed split order; blocks >= nmain (when
// the launch carries a bias gradient) fold its chunk partials instead.  A thread owns 4
// consecutive outputs (16-byte partial loads when N % 4 == 0) and keeps 4 splits' loads in
// flight; each output's sum still runs z = 0, 1, ... in order (bit-identical to one at a time).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs a, int S, int nmain, DbArgs d) {
  if ((int)blockIdx.x >= nmain) {
    db_final(d, (int)blockIdx.x - nmain);
    return;
  }
  const float* __restrict__ ws = a.ws;
  const int M = a.M, N = a.N;
  const long long MN = (long long)M * N;
  if ((N & 3) == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0) {
    for (long long i = 4 * (blockIdx.x * 256ll + threadIdx.x); i < MN; i += 4ll * nmain * 256) {
      f4 s = f4{0.f, 0.f, 0.f, 0.f};
      int z = 0;
      for (; z + 4 <= S; z += 4) {
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f4*>(ws + (size_t)(z + u) * MN + i);
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u];
      }
      for (; z < S; ++z) s += *reinterpret_cast<const f4*>(ws + (size_t)z * MN + i);
      const int m = (int)(i / N), n = (int)(i % N);
#pragma unroll
      for (int e = 0; e < 4; ++e) gemm_out(a, m, n + e, s[e]);
    }
    return;
  }
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < MN; i += (long long)nmain * 256) {
    float s = 0.f;
    int z = 0;
    for (; z + 4 <= S; z += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ws[(size_t)(z + u) * MN + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; z < S; ++z) s += ws[(size_t)z * MN + i];
    gemm_out(a, (int)(i / N), (int)(i % N), s);
  }
}

// (the vector layouts also need the bounded extent to be whole vectors: the loads test bounds
// per float4, not per element -- n_k for LAY_K, n_rows for LAY_R)
int lay_of(const float* p, long long s_rows, long long s_k, long long n_rows, long long n_k) {
  const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  if (s_k == 1 && s_rows % 4 == 0 && n_k % 4 == 0 && al) return LAY_K;
  if (s_rows == 1 && s_k % 4 == 0 && n_rows % 4 == 0 && al) return LAY_R;
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
    // split target in blocks (112 / 448 / 896 measured slower, profiles/r3_gemm_ab_n256.txt)
    constexpr int target256 = 224;
    const int s = (int)std::max(1ll, std::min<long long>(avd_cdiv(target256, t), K / 128));
    if (s > 1) {
      p.kchunk = avd_cdiv(avd_cdiv(K, s), 64) * 64;   // whole k-tiles of either mode
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
  // split target (blocks) and minimum K rows per split (512 / 256: the best of 128-2048 /
  // 64-256, profiles/r3_gemm_ab.txt; re-measured with 64-wide k-tiles against kmin 128 / 512
  // and target 1024, profiles/r5j_gemm_plan_ab.txt)
  constexpr int target = 512, kmin = 256;
  if (t < 224 && K >= 512) {
    int s = (int)std::min<long long>(avd_cdiv(target, t), K / kmin);
    s = std::max(1, std::min(s, 128));
    if (s > 1) {
      p.kchunk = avd_cdiv(avd_cdiv(K, s), 64) * 64;   // whole k-tiles of either mode
      p.splits = avd_cdiv(K, p.kchunk);
    }
  }
  return p;
}

GemmArgs make_args(const Plan& pl, int M, int N, int K, const void* A, long long sam,
                   long long sak, const void* B, long long sbk, long long sbn, void* C,
                   long long ldc, const float* bias, float alpha, float beta, float* ws,
                   int c_bf16 = 0, int map_c = 0, int map_hw = 0) {
  return GemmArgs{M, N, K, pl.kchunk, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha, beta,
                  pl.splits > 1 ? ws : nullptr, c_bf16, map_c, map_hw};
}

__global__ __launch_bounds__(256) void db_final_kernel(DbArgs d) { db_final(d, (int)blockIdx.x); }

// the split-K reduce of one problem (plus, with d.db, the bias gradient's final fold); with no
// split and a bias gradient, the fold alone
void launch_splitk_reduce(const Plan& pl, const GemmArgs& a, hipStream_t st, const DbArgs* d = nullptr) {
  const int nd = (d && d->db) ? avd_cdiv(d->O, 256) : 0;
  if (pl.splits > 1) {
    const long long MN = (long long)a.M * a.N;
    const int per = (a.N & 3) == 0 ? 4 : 1;     // outputs per thread (the kernel's vector path)
    const int blocks = (int)std::min<long long>(avd_cdiv(avd_cdiv(MN, per), 256), 4096);
    splitk_reduce_kernel<<<blocks + nd, 256, 0, st>>>(a, pl.splits, blocks, d ? *d : DbArgs{});
  } else if (nd) {
    db_final_kernel<<<nd, 256, 0, st>>>(*d);
  }
}

template <int MODE, int LA, int LB, typename SA = float, typename SB = float>
void launch_gemm(const Plan& pl, const GemmArgs& a, hipStream_t st) {
  dim3 grid(avd_cdiv(a.N, pl.bn), avd_cdiv(a.M, pl.bm), pl.splits);
#define AVD_G(BM_, BN_)                                                                        \
  if (pl.bm == BM_ && pl.bn == BN_) gemm_mfma_kernel<MODE, BM_, BN_, LA, LB, SA, SB><<<grid, 256, 0, st>>>(a);
  AVD_G(128, 256) else AVD_G(128, 128) else AVD_G(128, 64) else AVD_G(64, 64)
#undef AVD_G
  launch_splitk_reduce(pl, a, st);
}

// operand layouts are template parameters (the index math of the others would otherwise sit in
// registers): K/R combinations get vector loads, anything with a scalar operand the generic path
template <int MODE>
void dispatch_gemm(const Plan& pl, int lA, int lB, const GemmArgs& a, hipStream_t st) {
#define AVD_L(LA_, LB_) launch_gemm<MODE, LA_, LB_>(pl, a, st)
  if (lA == LAY_K && lB == LAY_K) AVD_L(LAY_K, LAY_K);
  else if (lA == LAY_K && lB == LAY_R) AVD_L(LAY_K, LAY_R);
  else if (lA == LAY_R && lB == LAY_R) AVD_L(LAY_R, LAY_R);
  else if (lA == LAY_R && lB == LAY_K) AVD_L(LAY_R, LAY_K);
  else AVD_L(LAY_S, LAY_S);
#undef AVD_L
}

// The paired Linear backward launch: problem 1 = dW [O, In] = dout^T x (A rows contiguous, B
// rows contiguous), problem 2 = dX [rows, In] = dout W (A k-contiguous, B rows contiguous).
// Tile plans served: dW 128x128 (every weight-gradient plan of the step), dX any of 128x128,
// 128x64, 64x64; anything else returns false and the caller launches the two GEMMs separately.
// which: 3 = both problems; 1 = the weight gradient (+ bias gradient) only, the input-gradient
// grid empty (the caller runs dX on the critical stream and dW beside it, on another stream).
template <int MODE, typename SB = float>
bool launch_pair(const Plan& p1, const GemmArgs& a1, const Plan& p2, const GemmArgs& a2,
                 const DbArgs& d, hipStream_t st, int which = 3) {
  if (p1.bm != 128 || p1.bn != 128) return false;
  const int n1 = avd_cdiv(a1.N, p1.bn), m1 = avd_cdiv(a1.M, p1.bm);
  const int n2 = which & 2 ? avd_cdiv(a2.N, p2.bn) : 0, m2 = which & 2 ? avd_cdiv(a2.M, p2.bm) : 0;
  const int blocks = n1 * m1 * p1.splits + n2 * m2 * p2.splits + (d.db ? d.nrc * d.strips : 0);
#define AVD_P(BM2_, BN2_)                                                                      \
  if (p2.bm == BM2_ && p2.bn == BN2_) {                                                        \
    gemm_pair_kernel<MODE, 128, 128, LAY_R, LAY_R, BM2_, BN2_, LAY_K, LAY_R, SB>               \
        <<<blocks, 256, 0, st>>>(a1, n1, m1, a2, n2, m2, d);                                   \
  }
  AVD_P(128, 128) else AVD_P(128, 64) else AVD_P(64, 64) else return false;
#undef AVD_P
  launch_splitk_reduce(p1, a1, st, &d);
  if (which & 2) launch_splitk_reduce(p2, a2, st);
  return true;
}

__global__ __launch_bounds__(256) void db_partial_kernel(DbArgs d) { db_partial(d, (int)blockIdx.x); }

// bias-gradient chunking: ~128 row chunks
DbArgs db_args(const float* dout, long long ld, int rows, int O, float* part, float* db) {
  DbArgs d{};
  d.dout = dout; d.ld = ld; d.rows = rows; d.O = O;
  d.chunk = std::max(1, avd_cdiv(rows, 128));
  d.nrc = avd_cdiv(rows, d.chunk);
  d.strips = avd_cdiv(O, 256);
  d.part = part; d.db = db;
  return d;
}
long long db_ws_elems(int rows, int O) {
  const int chunk = std::max(1, avd_cdiv(rows, 128));
  return (long long)avd_cdiv(rows, chunk) * O;
}

// The encoder Linear's weight with its columns in the NHWC (h, w, c) order of the bf16 features:
// Wp[o][hw * C + c] = bf16(W[o][c * HW + hw]); up to HWCB_MAX weights per launch (blockIdx.y).
constexpr int HWCB_MAX = 4;
struct HwcBatch {
  const float* w[HWCB_MAX];
  bf16* wp[HWCB_MAX];
  int O[HWCB_MAX], C[HWCB_MAX], HW[HWCB_MAX];
};

__global__ __launch_bounds__(256) void weight_hwc_kernel(HwcBatch b) {
  const int e = blockIdx.y;
  const int C = b.C[e], HW = b.HW[e], In = C * HW;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)b.O[e] * In) return;
  const int o = (int)(i / In), j = (int)(i - (long long)o * In);    // j = hw * C + c
  const int hw = j / C, c = j - hw * C;
  b.wp[e][i] = f2bf(b.w[e][(size_t)o * In + (size_t)c * HW + hw]);
}

}  // namespace

extern "C" {

long long avd_linear_bwd_ws_elems(int rows, int O, int In, int mode) {
  return avd_gemm_ws_elems(O, In, rows, mode) + avd_gemm_ws_elems(rows, In, O, mode) +
         db_ws_elems(rows, O);
}

int avd_linear_bwd(int rows, int O, int In, const float* dout, long long dout_ld, const float* x,
                   long long x_ld, const float* W, float* dW, float* dX, long long dx_ld, float* db,
                   int mode, int which, float* ws, long long ws_elems, void* stream) {
  if (which < 1 || which > 3) return AVD_ERR_ARG;
  if (!dout || ((which & 1) && (!x || !dW)) || ((which & 2) && (!W || !dX))) return AVD_ERR_ARG;
  if (rows <= 0 || O <= 0 || In <= 0 || dout_ld < O || x_ld < In || dx_ld < In) return AVD_ERR_SHAPE;
  if (mode != 1 && mode != 2) return AVD_ERR_ARG;
  hipStream_t st = avd_stream(stream);
  Plan p1 = plan_for(O, In, rows), p2 = plan_for(rows, In, O);
  const long long w1 = p1.splits > 1 ? (long long)p1.splits * O * In : 0;
  const long long w2 = p2.splits > 1 ? (long long)p2.splits * rows * In : 0;
  const long long w3 = db_ws_elems(rows, O);
  if (db && (!ws || ws_elems < w1 + w2 + w3)) return AVD_ERR_ARG;   // the bias partials need room
  if (!ws || ws_elems < w1 + w2) {   // no (or too small a) workspace: single passes over K
    if (p1.splits > 1) { p1.splits = 1; p1.kchunk = rows; }
    if (p2.splits > 1) { p2.splits = 1; p2.kchunk = O; }
  }
  const DbArgs d = db_args(dout, dout_ld, rows, O, db ? ws + w1 + w2 : nullptr, db);
  // dW[o, i] = sum_r dout[r, o] x[r, i]; dX[r, i] = sum_o dout[r, o] W[o, i]
  const GemmArgs a1 = make_args(p1, O, In, rows, dout, 1, dout_ld, x, x_ld, 1, dW, In, nullptr,
                                1.f, 0.f, ws);
  const GemmArgs a2 = make_args(p2, rows, In, O, dout, dout_ld, 1, W, In, 1, dX, dx_ld, nullptr,
                                1.f, 0.f, p1.splits > 1 ? ws + w1 : ws);
  const bool lay = (which & 1) && lay_of(dout, 1, dout_ld, O, rows) == LAY_R &&
                   lay_of(x, 1, x_ld, In, rows) == LAY_R &&
                   (!(which & 2) || (lay_of(dout, dout_ld, 1, rows, O) == LAY_K &&
                                     lay_of(W, 1, In, In, O) == LAY_R));
  bool done = false;
  if (lay)
    done = mode == 1 ? launch_pair<1>(p1, a1, p2, a2, d, st, which)
                     : launch_pair<2>(p1, a1, p2, a2, d, st, which);
  if (!done) {
    if (db && (which & 1)) {
      db_partial_kernel<<<d.nrc * d.strips, 256, 0, st>>>(d);
      db_final_kernel<<<avd_cdiv(O, 256), 256, 0, st>>>(d);
    }
    if (which & 1) {
      const int l1a = lay_of(dout, 1, dout_ld, O, rows), l1b = lay_of(x, 1, x_ld, In, rows);
      if (mode == 1) dispatch_gemm<1>(p1, l1a, l1b, a1, st);
      else dispatch_gemm<2>(p1, l1a, l1b, a1, st);
    }
    if (which & 2) {
      const int l2a = lay_of(dout, dout_ld, 1, rows, O), l2b = lay_of(W, 1, In, In, O);
      if (mode == 1) dispatch_gemm<1>(p2, l2a, l2b, a2, st);
      else dispatch_gemm<2>(p2, l2a, l2b, a2, st);
    }
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// ---- encoder Linear over NHWC bf16 features (include/avdino.h "encoder Linear, NHWC features")
long long avd_linear_hwc_ws_elems(int rows, int O, int In) {
  if (rows <= 0 || O <= 0 || In <= 0) return 0;
  const Plan pf = plan_for(rows, O, In), p1 = plan_for(O, In, rows), p2 = plan_for(rows, In, O);
  const long long wf = pf.splits > 1 ? (long long)pf.splits * rows * O : 0;
  const long long wb = (p1.splits > 1 ? (long long)p1.splits * O * In : 0) +
                       (p2.splits > 1 ? (long long)p2.splits * rows * In : 0) + db_ws_elems(rows, O);
  return std::max(wf, wb);
}

int avd_linear_weight_hwc(int n, const float* const* W, void* const* Wp, const int* O, const int* C,
                          const int* HW, void* stream) {
  if (n <= 0 || n > HWCB_MAX || !W || !Wp || !O || !C || !HW) return AVD_ERR_ARG;
  HwcBatch b{};
  int most = 1;
  for (int e = 0; e < n; ++e) {
    if (!W[e] || !Wp[e]) return AVD_ERR_ARG;
    if (O[e] <= 0 || C[e] <= 0 || HW[e] <= 0) return AVD_ERR_SHAPE;
    b.w[e] = W[e]; b.wp[e] = (bf16*)Wp[e]; b.O[e] = O[e]; b.C[e] = C[e]; b.HW[e] = HW[e];
    most = std::max(most, O[e] * C[e] * HW[e]);
  }
  weight_hwc_kernel<<<dim3(avd_cdiv(most, 256), n), 256, 0, avd_stream(stream)>>>(b);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_linear_fwd_hwc(int rows, int O, int C, int HW, const void* feat, const void* Wp,
                       const float* bias, float* out, long long out_ld, float* ws,
                       long long ws_elems, void* stream) {
  if (!feat || !Wp || !out) return AVD_ERR_ARG;
  const int In = C * HW;
  if (rows <= 0 || O <= 0 || C <= 0 || HW <= 0 || out_ld < O || In % 8) return AVD_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(feat) & 15) || (reinterpret_cast<uintptr_t>(Wp) & 15)) return AVD_ERR_ARG;
  Plan pl = plan_for(rows, O, In);
  if (pl.splits > 1 && (!ws || ws_elems < (long long)pl.splits * rows * O)) { pl.splits = 1; pl.kchunk = In; }
  // out[r, o] = sum_i feat[r, i] Wp[o, i]: A = feat (k contiguous), B^T rows = Wp rows
  const GemmArgs a = make_args(pl, rows, O, In, feat, In, 1, Wp, 1, In, out, out_ld, bias, 1.f, 0.f, ws);
  launch_gemm<2, LAY_K, LAY_K, bf16, bf16>(pl, a, avd_stream(stream));
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_linear_bwd_hwc(int rows, int O, int C, int HW, const float* dout, long long dout_ld,
                       const void* feat, const void* Wp, float* dW, float* db, void* dX, int which,
                       float* ws, long long ws_elems, void* stream) {
  if (which < 1 || which > 3) return AVD_ERR_ARG;
  if (!dout || ((which & 1) && (!feat || !dW)) || ((which & 2) && (!Wp || !dX))) return AVD_ERR_ARG;
  const int In = C * HW;
  if (rows <= 0 || O <= 0 || C <= 0 || HW <= 0 || dout_ld < O || In % 8 || O % 4 || dout_ld % 4)
    return AVD_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(dout) & 15) || (reinterpret_cast<uintptr_t>(feat) & 15) ||
      (reinterpret_cast<uintptr_t>(Wp) & 15))
    return AVD_ERR_ARG;       // (NULL, for a part not computed, passes)
  hipStream_t st = avd_stream(stream);
  Plan p1 = plan_for(O, In, rows), p2 = plan_for(rows, In, O);
  const long long w1 = p1.splits > 1 ? (long long)p1.splits * O * In : 0;
  const long long w2 = p2.splits > 1 ? (long long)p2.splits * rows * In : 0;
  const long long w3 = db_ws_elems(rows, O);
  if (!ws || ws_elems < w1 + w2 + w3) return AVD_ERR_ARG;
  const DbArgs d = db_args(dout, dout_ld, rows, O, db ? ws + w1 + w2 : nullptr, db);
  // dW[o, (c,h,w)] = sum_r dout[r, o] feat[r, (h,w,c)]: the column map scatters the hwc index
  const GemmArgs a1 = make_args(p1, O, In, rows, dout, 1, dout_ld, feat, In, 1, dW, In, nullptr,
                                1.f, 0.f, ws, 0, C, HW);
  // dX[r, (h,w,c)] = sum_o dout[r, o] Wp[o, (h,w,c)], stored bf16 NHWC
  const GemmArgs a2 = make_args(p2, rows, In, O, dout, dout_ld, 1, Wp, In, 1, dX, In, nullptr,
                                1.f, 0.f, p1.splits > 1 ? ws + w1 : ws, 1);
  if (!(which & 1) || !launch_pair<2, bf16>(p1, a1, p2, a2, d, st, which)) {
    // dX alone, or shapes the paired launch does not serve (few rows: no 128x128 dW plan)
    if ((which & 1) && db) {
      db_partial_kernel<<<d.nrc * d.strips, 256, 0, st>>>(d);
      db_final_kernel<<<avd_cdiv(O, 256), 256, 0, st>>>(d);
    }
    if (which & 1) launch_gemm<2, LAY_R, LAY_R, float, bf16>(p1, a1, st);
    if (which & 2) launch_gemm<2, LAY_K, LAY_R, float, bf16>(p2, a2, st);
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

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
    const int lA = lay_of(A, sam, sak, M, K);
    const int lB = lay_of(B, sbn, sbk, N, K);
    const GemmArgs a = make_args(pl, M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha, beta, ws);
    if (mode == 1)
      dispatch_gemm<1>(pl, lA, lB, a, st);
    else
      dispatch_gemm<2>(pl, lA, lB, a, st);
  } else {
    return AVD_ERR_ARG;
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
