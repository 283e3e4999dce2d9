// Loss heads, forward + backward fused, one wavefront per row (projection width P <= 512,
// P/64 values per lane, shuffle reductions for norms / softmax):
//  * DINO cross-entropy over softmaxes with teacher centring + centre EMA
//    (MultiModalDINO.forward dino.py:709-720, update_center 648-653, dino_loss 822-854;
//     UniModalDINOLightning.dino_loss 1596-1635 with the per-view teacher mean subtraction)
//  * MSE between L2-normalised rows (mse_loss, dino.py:1193-1211)
//  * row L2 normalisation fwd/bwd (F.normalize) and softmax cross-entropy with integer /
//    diagonal / NT-Xent targets (infoNCE_loss dino.py:1091-1128, nt_xent_loss
//    multimodal_simclr.py:74-89, supervised_loss dino.py:1001-1025).
#include "common.h"

using namespace avd;

namespace {

constexpr int MAXV = 8;  // P <= 64*MAXV
constexpr float NORM_EPS = 1e-12f;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Teacher rows: tn = normalize(t_raw - center)   [T*B, P]
__global__ __launch_bounds__(256) void teacher_norm_kernel(const float* __restrict__ t_raw,
                                                           const float* __restrict__ center,
                                                           float* __restrict__ tn, int rows, int P) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (row >= rows) return;
  float v[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    v[j] = k < P ? t_raw[(size_t)row * P + k] - center[k] : 0.f;
    ss += v[j] * v[j];
  }
  const float inv = 1.f / fmaxf(sqrtf(wave_sum(ss)), NORM_EPS);
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    if (k < P) tn[(size_t)row * P + k] = v[j] * inv;
  }
}

// Per-view column means of tn over B rows, subtracted in place (center_teacher variant).
__global__ __launch_bounds__(256) void teacher_center_kernel(float* __restrict__ tn, int T, int B,
                                                             int P) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int t = blockIdx.y;
  if (k >= P) return;
  double s = 0.0;
  for (int b = 0; b < B; ++b) s += tn[((size_t)t * B + b) * P + k];
  const float m = (float)(s / B);
  for (int b = 0; b < B; ++b) tn[((size_t)t * B + b) * P + k] -= m;
}

// ptsum[b] = sum_t softmax(tn[t*B+b] / tau_t)
__global__ __launch_bounds__(256) void teacher_probs_kernel(const float* __restrict__ tn,
                                                            float* __restrict__ ptsum, int T, int B,
                                                            int P, float inv_tau) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (b >= B) return;
  float acc[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) acc[j] = 0.f;
  for (int t = 0; t < T; ++t) {
    float z[MAXV];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int k = l + 64 * j;
      z[j] = k < P ? tn[((size_t)t * B + b) * P + k] * inv_tau : -INFINITY;
      m = fmaxf(m, z[j]);
    }
    m = wave_max(m);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      z[j] = (l + 64 * j < P) ? expf(z[j] - m) : 0.f;
      se += z[j];
    }
    const float inv = 1.f / wave_sum(se);
#pragma unroll
    for (int j = 0; j < MAXV; ++j) acc[j] += z[j] * inv;
  }
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    if (k < P) ptsum[(size_t)b * P + k] = acc[j];
  }
}

// Student rows: loss part and d loss / d s.
__global__ __launch_bounds__(256) void student_kernel(const float* __restrict__ s,
                                                      const float* __restrict__ ptsum,
                                                      float* __restrict__ loss_parts,
                                                      float* __restrict__ ds, int V, int T, int B,
                                                      int P, float inv_tau) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (row >= V * B) return;
  const int b = row % B;
  const float norm_c = 1.f / ((float)B * V * T);
  float x[MAXV], pt[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    x[j] = k < P ? s[(size_t)row * P + k] : 0.f;
    pt[j] = k < P ? ptsum[(size_t)b * P + k] : 0.f;
    ss += x[j] * x[j];
  }
  const float nrm = sqrtf(wave_sum(ss));
  const float d = fmaxf(nrm, NORM_EPS);
  float z[MAXV], m = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    z[j] = (l + 64 * j < P) ? (x[j] / d) * inv_tau : -INFINITY;
    m = fmaxf(m, z[j]);
  }
  m = wave_max(m);
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) se += (l + 64 * j < P) ? expf(z[j] - m) : 0.f;
  se = wave_sum(se);
  const float lse = m + logf(se);
  // loss part = -sum_k pt_k (z_k - lse) / (B V T); g_k = -pt_k / (B V T)
  float lp = 0.f, gsum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (l + 64 * j < P) {
      lp += pt[j] * (z[j] - lse);
      gsum += pt[j];
    }
  lp = wave_sum(lp);
  gsum = -wave_sum(gsum) * norm_c;
  if (l == 0) loss_parts[row] = -lp * norm_c;
  // dz = g - softmax * sum(g); dsn = dz / tau; ds = (dsn - sn (sn.dsn)) / d
  float dsn[MAXV], proj = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const bool ok = l + 64 * j < P;
    const float sm = ok ? expf(z[j] - lse) : 0.f;
    dsn[j] = ok ? (-pt[j] * norm_c - sm * gsum) * inv_tau : 0.f;
    proj += dsn[j] * (x[j] / d);
  }
  proj = wave_sum(proj);
  const bool live = nrm > NORM_EPS;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    if (k < P) ds[(size_t)row * P + k] = (dsn[j] - (live ? (x[j] / d) * proj : 0.f)) / d;
  }
}

// center_new = m*center + (1-m) * mean over rows of t_raw  (fixed-order f64 column sums:
// 16 columns x 64 row phases per block)
__global__ __launch_bounds__(1024) void center_kernel(const float* __restrict__ t_raw,
                                                      const float* __restrict__ center,
                                                      float* __restrict__ center_new, int rows, int P,
                                                      float cm) {
  __shared__ double sh[64][16];
  const int lc = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int k = blockIdx.x * 16 + lc;
  double s = 0.0;
  if (k < P)
    for (int r = ph; r < rows; r += 64) s += t_raw[(size_t)r * P + k];
  sh[ph][lc] = s;
  __syncthreads();
  if (ph == 0 && k < P) {
    double t = 0.0;
    for (int i = 0; i < 64; ++i) t += sh[i][lc];
    center_new[k] = (float)((double)center[k] * cm + (t / rows) * (1.0 - (double)cm));
  }
}

__global__ __launch_bounds__(256) void mse_kernel(const float* __restrict__ a,
                                                  const float* __restrict__ bb,
                                                  float* __restrict__ loss_parts,
                                                  float* __restrict__ da, float* __restrict__ db,
                                                  int B, int P) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (row >= B) return;
  float x[MAXV], y[MAXV], sx = 0.f, sy = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    x[j] = k < P ? a[(size_t)row * P + k] : 0.f;
    y[j] = k < P ? bb[(size_t)row * P + k] : 0.f;
    sx += x[j] * x[j];
    sy += y[j] * y[j];
  }
  const float nx = sqrtf(wave_sum(sx)), ny = sqrtf(wave_sum(sy));
  const float dx = fmaxf(nx, NORM_EPS), dy = fmaxf(ny, NORM_EPS);
  const float sc = 2.f / ((float)B * P);
  float lp = 0.f, px = 0.f, py = 0.f, g[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const float d = x[j] / dx - y[j] / dy;
    lp += d * d;
    g[j] = sc * d;
    px += g[j] * (x[j] / dx);
    py += g[j] * (y[j] / dy);
  }
  lp = wave_sum(lp);
  px = wave_sum(px);
  py = wave_sum(py);
  if (l == 0) loss_parts[row] = lp / ((float)B * P);
  const bool lx = nx > NORM_EPS, ly = ny > NORM_EPS;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    if (k < P) {
      da[(size_t)row * P + k] = (g[j] - (lx ? (x[j] / dx) * px : 0.f)) / dx;
      db[(size_t)row * P + k] = (-g[j] + (ly ? (y[j] / dy) * py : 0.f)) / dy;
    }
  }
}

__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const float* __restrict__ x,
                                                         float* __restrict__ y,
                                                         float* __restrict__ norms, int rows,
                                                         int P) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (row >= rows) return;
  float v[MAXV], ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    v[j] = k < P ? x[(size_t)row * P + k] : 0.f;
    ss += v[j] * v[j];
  }
  const float n = sqrtf(wave_sum(ss));
  const float inv = 1.f / fmaxf(n, NORM_EPS);
  if (l == 0) norms[row] = n;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    if (k < P) y[(size_t)row * P + k] = v[j] * inv;
  }
}

__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ y,
                                                         const float* __restrict__ norms,
                                                         const float* dy, float* dx, int rows,
                                                         int P) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (row >= rows) return;
  float yy[MAXV], g[MAXV], pr = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    yy[j] = k < P ? y[(size_t)row * P + k] : 0.f;
    g[j] = k < P ? dy[(size_t)row * P + k] : 0.f;
    pr += yy[j] * g[j];
  }
  pr = wave_sum(pr);
  const float n = norms[row];
  const float d = fmaxf(n, NORM_EPS);
  const bool live = n > NORM_EPS;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int k = l + 64 * j;
    if (k < P) dx[(size_t)row * P + k] = (g[j] - (live ? yy[j] * pr : 0.f)) / d;
  }
}

__global__ __launch_bounds__(256) void softmax_xent_kernel(
    const float* __restrict__ logits, long long ld, int R, int C, const int64_t* __restrict__ targets,
    int target_mode, int tgt_off, int col_major, int mask_off, float gscale,
    float* __restrict__ loss_parts, float* dlogits, long long ldd, int accumulate) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (r >= R) return;
  auto at = [&](int j) -> size_t { return col_major ? (size_t)j * ld + r : (size_t)r * ld + j; };
  auto atd = [&](int j) -> size_t { return col_major ? (size_t)j * ldd + r : (size_t)r * ldd + j; };
  const int tgt = target_mode == 0 ? (int)targets[r] : target_mode == 1 ? r + tgt_off : (r + R / 2) % R;
  const int mcol = mask_off >= 0 ? r + mask_off : -1;   // excluded column (-inf logit)
  float m = -INFINITY;
  for (int j = l; j < C; j += 64)
    if (j != mcol) m = fmaxf(m, logits[at(j)]);
  m = wave_max(m);
  float se = 0.f;
  for (int j = l; j < C; j += 64)
    if (j != mcol) se += expf(logits[at(j)] - m);
  se = wave_sum(se);
  const float lse = m + logf(se);
  if (l == 0) loss_parts[r] = lse - logits[at(tgt)];
  if (dlogits) {
    for (int j = l; j < C; j += 64) {
      float g = 0.f;
      if (j != mcol) g = (expf(logits[at(j)] - lse) - (j == tgt ? 1.f : 0.f)) * gscale;
      const size_t o = atd(j);
      dlogits[o] = accumulate ? dlogits[o] + g : g;
    }
  }
}

// Cosine-consistency term of UniModalDINOLightning (_cosine_consistency_loss, dino.py:1575-1594):
// one block per sample b over its V view rows e_v = emb[v*B + b] (view-major [V*B, D]):
//   n_v = e_v / max(|e_v|, eps),  loss_b = sum_{i<j} (1 - n_i.n_j)^2 / (count * B)
//   demb_i = alpha * (dn_i - n_i (n_i.dn_i)) / max(|e_i|, eps),
//   dn_i = sum_{j != i} -2 (1 - n_i.n_j) n_j / (count * B)
// demb is ACCUMULATED (added to the projection head's input gradient); either output may be
// NULL (forward: loss only; backward: gradient only).
constexpr int COS_MAXV = 32;
__global__ __launch_bounds__(256) void cosine_consistency_kernel(
    const float* __restrict__ emb, int V, int B, int D, float alpha, float* __restrict__ loss_parts,
    float* __restrict__ demb) {
  __shared__ float inv[COS_MAXV];
  __shared__ float sim[COS_MAXV][COS_MAXV];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  auto row = [&](int v) { return emb + ((size_t)v * B + b) * D; };
  // norms: wave w handles views w, w+4, ...
  for (int v = w; v < V; v += 4) {
    float ss = 0.f;
    for (int k = l; k < D; k += 64) { const float x = row(v)[k]; ss += x * x; }
    ss = wave_sum(ss);
    if (l == 0) inv[v] = 1.f / fmaxf(sqrtf(ss), NORM_EPS);
  }
  __syncthreads();
  // pairwise cosine similarities (i < j), one wave per pair
  const int npair = V * (V - 1) / 2;
  for (int q = w; q < npair; q += 4) {
    int i = 0, rem = q;
    while (rem >= V - 1 - i) { rem -= V - 1 - i; ++i; }
    const int j = i + 1 + rem;
    float d = 0.f;
    for (int k = l; k < D; k += 64) d += row(i)[k] * row(j)[k];
    d = wave_sum(d) * inv[i] * inv[j];
    if (l == 0) { sim[i][j] = d; sim[j][i] = d; }
  }
  __syncthreads();
  const float scale = 1.f / ((float)npair * (float)B);
  if (tid == 0 && loss_parts) {
    float s = 0.f;
    for (int i = 0; i < V; ++i)
      for (int j = i + 1; j < V; ++j) s += (1.f - sim[i][j]) * (1.f - sim[i][j]);
    loss_parts[b] = s * scale * alpha;
  }
  if (!demb) return;
  // gradient: wave w handles views w, w+4, ...
  for (int i = w; i < V; i += 4) {
    float dot = 0.f;   // n_i . dn_i
    for (int k = l; k < D; k += 64) {
      float dn = 0.f;
      for (int j = 0; j < V; ++j)
        if (j != i) dn += -2.f * (1.f - sim[i][j]) * scale * row(j)[k] * inv[j];
      dot += dn * row(i)[k] * inv[i];
    }
    dot = wave_sum(dot);
    for (int k = l; k < D; k += 64) {
      float dn = 0.f;
      for (int j = 0; j < V; ++j)
        if (j != i) dn += -2.f * (1.f - sim[i][j]) * scale * row(j)[k] * inv[j];
      const float g = alpha * (dn - row(i)[k] * inv[i] * dot) * inv[i];
      demb[((size_t)i * B + b) * D + k] += g;
    }
  }
}

// correct[r] = 1 if argmax_j logits[r, j] (first maximum, torch.max semantics) == targets[r]
__global__ __launch_bounds__(256) void argmax_correct_kernel(const float* __restrict__ logits,
                                                             long long ld, int R, int C,
                                                             const int64_t* __restrict__ targets,
                                                             float* __restrict__ correct) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (r >= R) return;
  float best = -INFINITY;
  int bi = C;
  for (int j = l; j < C; j += 64) {
    const float v = logits[(size_t)r * ld + j];
    if (v > best) { best = v; bi = j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (l == 0) correct[r] = bi == (int)targets[r] ? 1.f : 0.f;
}

}  // namespace

extern "C" {

int avd_dino_loss(const float* s, const float* t_raw, const float* center, int V, int T, int B,
                  int P, float tau_s, float tau_t, float center_m, int center_teacher,
                  float* loss_parts, float* ds, float* center_new, float* work, void* stream) {
  if (!s || !t_raw || !center || !loss_parts || !ds || !center_new || !work) return AVD_ERR_ARG;
  if (V <= 0 || T <= 0 || B <= 0 || P <= 0 || P > 64 * MAXV) return AVD_ERR_SHAPE;
  hipStream_t st = avd_stream(stream);
  float* ptsum = work;                    // [B, P]
  float* tn = work + (size_t)B * P;       // [T*B, P]
  teacher_norm_kernel<<<avd_cdiv((long long)T * B, 4), 256, 0, st>>>(t_raw, center, tn, T * B, P);
  if (center_teacher) {
    dim3 g(avd_cdiv(P, 256), T);
    teacher_center_kernel<<<g, 256, 0, st>>>(tn, T, B, P);
  }
  teacher_probs_kernel<<<avd_cdiv(B, 4), 256, 0, st>>>(tn, ptsum, T, B, P, 1.f / tau_t);
  student_kernel<<<avd_cdiv((long long)V * B, 4), 256, 0, st>>>(s, ptsum, loss_parts, ds, V, T, B,
                                                                 P, 1.f / tau_s);
  center_kernel<<<avd_cdiv(P, 16), 1024, 0, st>>>(t_raw, center, center_new, T * B, P, center_m);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_mse_loss(const float* a, const float* b, int B, int P, float* loss_parts, float* da,
                 float* db, void* stream) {
  if (!a || !b || !loss_parts || !da || !db) return AVD_ERR_ARG;
  if (B <= 0 || P <= 0 || P > 64 * MAXV) return AVD_ERR_SHAPE;
  mse_kernel<<<avd_cdiv(B, 4), 256, 0, avd_stream(stream)>>>(a, b, loss_parts, da, db, B, P);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_l2norm_fwd(const float* x, float* y, float* norms, int rows, int P, void* stream) {
  if (!x || !y || !norms) return AVD_ERR_ARG;
  if (rows <= 0 || P <= 0 || P > 64 * MAXV) return AVD_ERR_SHAPE;
  l2norm_fwd_kernel<<<avd_cdiv(rows, 4), 256, 0, avd_stream(stream)>>>(x, y, norms, rows, P);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_l2norm_bwd(const float* y, const float* norms, const float* dy, float* dx, int rows, int P,
                   void* stream) {
  if (!y || !norms || !dy || !dx) return AVD_ERR_ARG;
  if (rows <= 0 || P <= 0 || P > 64 * MAXV) return AVD_ERR_SHAPE;
  l2norm_bwd_kernel<<<avd_cdiv(rows, 4), 256, 0, avd_stream(stream)>>>(y, norms, dy, dx, rows, P);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_softmax_xent(const float* logits, long long ld, int R, int C, const int64_t* targets,
                     int target_mode, int tgt_off, int col_major, int mask_off, float gscale,
                     float* loss_parts, float* dlogits, long long ldd, int accumulate,
                     void* stream) {
  if (!logits || !loss_parts || (target_mode == 0 && !targets)) return AVD_ERR_ARG;
  if (target_mode < 0 || target_mode > 2) return AVD_ERR_ARG;
  if (R <= 0 || C <= 0) return AVD_ERR_SHAPE;
  if (target_mode == 1 && (tgt_off < 0 || R - 1 + tgt_off >= C)) return AVD_ERR_SHAPE;
  softmax_xent_kernel<<<avd_cdiv(R, 4), 256, 0, avd_stream(stream)>>>(
      logits, ld, R, C, targets, target_mode, tgt_off, col_major, mask_off, gscale, loss_parts,
      dlogits, ldd, accumulate);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_argmax_correct(const float* logits, long long ld, int R, int C, const int64_t* targets,
                       float* correct, void* stream) {
  if (!logits || !targets || !correct) return AVD_ERR_ARG;
  if (R <= 0 || C <= 0 || ld < C) return AVD_ERR_SHAPE;
  argmax_correct_kernel<<<avd_cdiv(R, 4), 256, 0, avd_stream(stream)>>>(logits, ld, R, C, targets,
                                                                         correct);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_cosine_consistency(const float* emb, int V, int B, int D, float alpha, float* loss_parts,
                           float* demb, void* stream) {
  if (!emb || (!loss_parts && !demb)) return AVD_ERR_ARG;
  if (V < 2 || V > COS_MAXV || B <= 0 || D <= 0) return AVD_ERR_SHAPE;
  cosine_consistency_kernel<<<B, 256, 0, avd_stream(stream)>>>(emb, V, B, D, alpha, loss_parts,
                                                               demb);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

}  // extern "C"
