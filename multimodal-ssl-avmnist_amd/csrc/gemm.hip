// Dense layers: f32 GEMM with arbitrary strides for nn.Linear forward (x W^T + b), input
// gradient (dy W) and weight gradient (dy^T x, with the bias gradient = row sums of dy^T
// produced by the same launch).  Layers: CentralMultiModalEncoder's image/audio Linear and
// fusion MLP (dino.py:222-227, 459-468), ProjectionHead (dino.py:1240-1254).
//
// v1: LDS-tiled 64x64x16 tiles, 256 threads, 4x4 outputs per thread, fp32 FMA (bitwise
// deterministic: no split-K).
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
// Block tile 64x64, BK 32, 4 waves x (32x32 = 2x2 MFMA tiles).  Operands are staged in LDS
// with k contiguous ([m][k] for A, [n][k] for B) so every fragment is one LDS read; global
// loads are float4 whenever the contiguous stride is 1 and rows are 16-byte aligned.
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;

template <int MODE>
struct GemmT { typedef float T; static constexpr int LDK = 33; };
template <>
struct GemmT<2> { typedef bf16 T; static constexpr int LDK = 40; };

template <int MODE>
__device__ __forceinline__ void lds_put(typename GemmT<MODE>::T* p, float v) {
  if constexpr (MODE == 2) *p = f2bf(v); else *p = v;
}

// Stage a 64 (rows r) x 32 (k) tile of a matrix X with element (r, k) at X[r*sr + k*sk] into
// S[r*LDK + k].  rows/ks = valid extent.
template <int MODE>
__device__ __forceinline__ void stage_tile(const float* __restrict__ X, long long sr, long long sk,
                                           int r0, int k0, int rows, int ks, bool vec,
                                           typename GemmT<MODE>::T* S) {
  constexpr int LDK = GemmT<MODE>::LDK;
  const int tid = threadIdx.x;
  if (vec && sk == 1) {  // k contiguous: float4 along k
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e4 = tid + 256 * i;
      const int r = e4 >> 3, k = (e4 & 7) * 4;
      const int gr = r0 + r, gk = k0 + k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gr < rows) {
        const float* p = X + (size_t)gr * sr + gk;
        if (gk + 3 < ks) v = *reinterpret_cast<const float4*>(p);
        else {
          if (gk < ks) v.x = p[0];
          if (gk + 1 < ks) v.y = p[1];
          if (gk + 2 < ks) v.z = p[2];
        }
      }
      typename GemmT<MODE>::T* d = S + r * LDK + k;
      lds_put<MODE>(d, v.x); lds_put<MODE>(d + 1, v.y); lds_put<MODE>(d + 2, v.z); lds_put<MODE>(d + 3, v.w);
    }
  } else if (vec && sr == 1) {  // rows contiguous: float4 along r
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e4 = tid + 256 * i;
      const int k = e4 >> 4, r = (e4 & 15) * 4;
      const int gr = r0 + r, gk = k0 + k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk < ks) {
        const float* p = X + (size_t)gk * sk + gr;
        if (gr + 3 < rows) v = *reinterpret_cast<const float4*>(p);
        else {
          if (gr < rows) v.x = p[0];
          if (gr + 1 < rows) v.y = p[1];
          if (gr + 2 < rows) v.z = p[2];
        }
      }
      lds_put<MODE>(S + r * LDK + k, v.x);
      lds_put<MODE>(S + (r + 1) * LDK + k, v.y);
      lds_put<MODE>(S + (r + 2) * LDK + k, v.z);
      lds_put<MODE>(S + (r + 3) * LDK + k, v.w);
    }
  } else {
    const bool kfast = sk <= sr;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i;
      int r, k;
      if (kfast) { r = e >> 5; k = e & 31; } else { k = e >> 6; r = e & 63; }
      const int gr = r0 + r, gk = k0 + k;
      const float v = (gr < rows && gk < ks) ? X[(size_t)gr * sr + (size_t)gk * sk] : 0.f;
      lds_put<MODE>(S + r * LDK + k, v);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void gemm_mfma_kernel(int M, int N, int K, const float* __restrict__ A,
                                                        long long sam, long long sak,
                                                        const float* __restrict__ B, long long sbk,
                                                        long long sbn, float* __restrict__ C,
                                                        long long ldc, const float* __restrict__ bias,
                                                        float alpha, float beta, int vecA, int vecB) {
  typedef typename GemmT<MODE>::T T;
  constexpr int LDK = GemmT<MODE>::LDK;
  __shared__ __attribute__((aligned(16))) T As[64 * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[64 * LDK];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += 32) {
    stage_tile<MODE>(A, sam, sak, m0, k0, M, K, vecA, As);
    stage_tile<MODE>(B, sbn, sbk, n0, k0, N, K, vecB, Bs);   // B^T tile: rows = n
    __syncthreads();
    if constexpr (MODE == 2) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(As + (32 * wm + 16 * i + r16) * LDK + 8 * g);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + (32 * wn + 16 * j + r16) * LDK + 8 * g);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        float a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = As[(32 * wm + 16 * i + r16) * LDK + 4 * ks + g];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = Bs[(32 * wn + 16 * j + r16) * LDK + 4 * ks + g];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 32 * wn + 16 * j + r16;
      if (n >= N) continue;
      const float bv = bias ? bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 32 * wm + 16 * i + 4 * g + e;
        if (m >= M) continue;
        float* c = C + (size_t)m * ldc + n;
        float v = alpha * acc[i][j][e] + bv;
        if (beta != 0.f) v += beta * *c;
        *c = v;
      }
    }
}

bool vec_ok(const float* p, long long s_contig, long long s_other) {
  return s_contig == 1 && (s_other % 4) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

}  // namespace

extern "C" {

int avd_gemm(int M, int N, int K, const float* A, long long sam, long long sak, const float* B,
             long long sbk, long long sbn, float* C, long long ldc, const float* bias, float alpha,
             float beta, int mode, void* stream) {
  if (!A || !B || !C) return AVD_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
  dim3 grid(avd_cdiv(N, 64), avd_cdiv(M, 64));
  if (mode == 0) {
    sgemm_kernel<<<grid, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias, alpha,
                                        beta, nullptr);
  } else if (mode == 1 || mode == 2) {
    const int vA = vec_ok(A, sak == 1 ? sak : sam, sak == 1 ? sam : sak);
    const int vB = vec_ok(B, sbk == 1 ? sbk : sbn, sbk == 1 ? sbn : sbk);
    if (mode == 1)
      gemm_mfma_kernel<1><<<grid, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias,
                                                 alpha, beta, vA, vB);
    else
      gemm_mfma_kernel<2><<<grid, 256, 0, st>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias,
                                                 alpha, beta, vA, vB);
  } else {
    return AVD_ERR_ARG;
  }
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
