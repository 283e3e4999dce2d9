// Downstream evaluation kernels: kNN neighbour selection + vote over a
// distance GEMM, and row argmax for classification metrics.
//
// Reference: training_structures/dino_train.py:349-369 train_knn_classifier
// (sklearn KNeighborsClassifier(n_neighbors=5): brute-force euclidean, uniform weights, the
// vote's ties to the smallest class label as scipy.stats.mode), 47-102
// compute_classification_metrics (torch.max(outputs, 1): first maximum).
#include "common.h"

namespace {

using namespace avd;

constexpr int KNN_T = 256;      // threads per test row
constexpr int KNN_KMAX = 16;
constexpr int KNN_CMAX = 64;

// (d, j) ordering: smaller distance first, ties to the smaller train index
__device__ __forceinline__ bool knn_less(float da, int ja, float db, int jb) {
  return da < db || (da == db && ja < jb);
}

// One workgroup per test row i.  d_j = xnorm[j] + S[i, j], with S = -2 q_i . x_j from the GEMM
// (|q_i|^2 is the same for every j of the row, so the ranking does not need it).  Each thread
// keeps a sorted top-KS of its strided columns in LDS; 8 pairwise merge rounds reduce the 256
// lists.  The GEMM form cancels |q|^2 + |x|^2 against 2 q.x, so its f32 error is relative to
// the norms, not to the distance: with Q/X given, the KS = min(16, N) candidates are re-ranked
// by their direct distance sum_k (q_k - x_jk)^2 (error relative to the distance itself, as
// sklearn's float64 path ranks them) before the first K are kept.  Thread 0 votes.
__global__ __launch_bounds__(KNN_T) void knn_select_kernel(
    const float* __restrict__ S, long long ldS, const float* __restrict__ xnorm, int N, int K,
    int KS, const float* __restrict__ Q, const float* __restrict__ X, int D,
    const int64_t* __restrict__ labels, int C, int64_t* __restrict__ nbr, int64_t* __restrict__ pred) {
  __shared__ float rd[KNN_KMAX];
  __shared__ float sd[KNN_T * KNN_KMAX];
  __shared__ int sj[KNN_T * KNN_KMAX];
  __shared__ float td[KNN_T / 2 * KNN_KMAX];   // merge outputs
  __shared__ int tj[KNN_T / 2 * KNN_KMAX];
  __shared__ int cnt[KNN_CMAX];
  const int t = threadIdx.x;
  const int i = blockIdx.x;
  float* d = sd + t * KS;
  int* jj = sj + t * KS;
  for (int k = 0; k < KS; ++k) { d[k] = INFINITY; jj[k] = 0x7fffffff; }
  float worst = INFINITY;
  int worst_j = 0x7fffffff;
  const float* row = S + (size_t)i * ldS;
  for (int j = t; j < N; j += KNN_T) {
    const float v = xnorm[j] + row[j];
    if (knn_less(v, j, worst, worst_j)) {      // insert into the sorted list, drop the last
      int p = KS - 1;
      while (p > 0 && knn_less(v, j, d[p - 1], jj[p - 1])) { d[p] = d[p - 1]; jj[p] = jj[p - 1]; --p; }
      d[p] = v; jj[p] = j;
      worst = d[KS - 1]; worst_j = jj[KS - 1];
    }
  }
  __syncthreads();
  for (int s = KNN_T / 2; s > 0; s >>= 1) {
    if (t < s) {   // merge lists t and t + s (both sorted) -> the KS smallest into list t
      float* a = sd + t * KS;   int* aj = sj + t * KS;
      const float* b = sd + (t + s) * KS; const int* bj = sj + (t + s) * KS;
      float* od = td + t * KS; int* oj = tj + t * KS;
      int x = 0, y = 0;
      for (int k = 0; k < KS; ++k) {
        if (knn_less(a[x], aj[x], b[y], bj[y])) { od[k] = a[x]; oj[k] = aj[x]; ++x; }
        else { od[k] = b[y]; oj[k] = bj[y]; ++y; }
      }
      for (int k = 0; k < KS; ++k) { a[k] = od[k]; aj[k] = oj[k]; }
    }
    __syncthreads();
  }
  if (Q) {   // re-rank the KS candidates by their direct distances: 16 lanes per candidate
    const int c = t >> 4, l = t & 15;
    float acc = 0.f;
    const int j = c < KS ? sj[c] : 0x7fffffff;
    if (c < KS && j < N) {
      const float* q = Q + (size_t)i * D;
      const float* x = X + (size_t)j * D;
      for (int k = l; k < D; k += 16) {
        const float df = q[k] - x[k];
        acc = fmaf(df, df, acc);
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
    __syncthreads();
    if (c < KS && l == 0) rd[c] = j < N ? acc : INFINITY;
    __syncthreads();
    if (t == 0) {   // insertion sort of the KS (distance, index) pairs
      for (int a = 1; a < KS; ++a) {
        const float dv = rd[a];
        const int jv = sj[a];
        int b = a;
        while (b > 0 && knn_less(dv, jv, rd[b - 1], sj[b - 1])) { rd[b] = rd[b - 1]; sj[b] = sj[b - 1]; --b; }
        rd[b] = dv; sj[b] = jv;
      }
    }
  }
  if (t < C) cnt[t] = 0;
  __syncthreads();
  if (t == 0) {
    for (int k = 0; k < K; ++k) {
      const int j = sj[k];
      if (nbr) nbr[(size_t)i * K + k] = j < N ? j : -1;
      if (j < N) {
        const long long c = labels[j];
        if (c >= 0 && c < C) ++cnt[c];
      }
    }
    int best = 0;
    for (int c = 1; c < C; ++c)
      if (cnt[c] > cnt[best]) best = c;
    pred[i] = best;
  }
}

// idx[r] = argmax_j logits[r*ld + j] (first maximum, torch.max), one wave per row
__global__ __launch_bounds__(256) void argmax_rows_kernel(const float* __restrict__ logits, long long ld,
                                                         int R, int C, int64_t* __restrict__ idx) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (r >= R) return;
  float best = -INFINITY;
  int bi = C;
  for (int j = l; j < C; j += 64) {
    const float v = logits[(size_t)r * ld + j];
    if (v > best || bi == C) { best = v; bi = j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (l == 0) idx[r] = bi;
}

// xnorm[j] = sum_k x[j*D + k]^2, one wave per row
__global__ __launch_bounds__(256) void row_sqnorm_kernel(const float* __restrict__ x, int N, int D,
                                                        float* __restrict__ out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (r >= N) return;
  float s = 0.f;
  for (int k = l; k < D; k += 64) {
    const float v = x[(size_t)r * D + k];
    s = fmaf(v, v, s);
  }
  s = wave_sum(s);
  if (l == 0) out[r] = s;
}

}  // namespace

extern "C" {

int avd_row_sqnorm(const float* x, int N, int D, float* out, void* stream) {
  if (!x || !out) return AVD_ERR_ARG;
  if (N <= 0 || D <= 0) return AVD_ERR_SHAPE;
  row_sqnorm_kernel<<<avd_cdiv(N, 4), 256, 0, avd_stream(stream)>>>(x, N, D, out);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_knn_select(const float* S, long long ldS, const float* xnorm, int M, int N, int K,
                   const float* Q, const float* X, int D, const int64_t* labels, int C,
                   int64_t* nbr, int64_t* pred, void* stream) {
  if (!S || !xnorm || !labels || !pred || (Q && !X)) return AVD_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0 || K > KNN_KMAX || K > N || C <= 0 || C > KNN_CMAX || ldS < N ||
      (Q && D <= 0))
    return AVD_ERR_SHAPE;
  const int KS = Q ? (N < KNN_KMAX ? N : KNN_KMAX) : K;
  knn_select_kernel<<<M, KNN_T, 0, avd_stream(stream)>>>(S, ldS, xnorm, N, K, KS, Q, X, D, labels, C,
                                                         nbr, pred);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_argmax_rows(const float* logits, long long ld, int R, int C, int64_t* idx, void* stream) {
  if (!logits || !idx) return AVD_ERR_ARG;
  if (R <= 0 || C <= 0 || ld < C) return AVD_ERR_SHAPE;
  argmax_rows_kernel<<<avd_cdiv(R, 4), 256, 0, avd_stream(stream)>>>(logits, ld, R, C, idx);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
