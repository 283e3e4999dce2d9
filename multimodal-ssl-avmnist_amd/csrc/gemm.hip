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

}  // namespace

extern "C" {

int avd_gemm(int M, int N, int K, const float* A, long long sam, long long sak, const float* B,
             long long sbk, long long sbn, float* C, long long ldc, const float* bias, float alpha,
             float beta, float* a_rowsum, void* stream) {
  if (!A || !B || !C) return AVD_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0) return AVD_ERR_SHAPE;
  dim3 grid(avd_cdiv(N, BN), avd_cdiv(M, BM));
  sgemm_kernel<<<grid, 256, 0, avd_stream(stream)>>>(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc,
                                                      bias, alpha, beta, a_rowsum);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
