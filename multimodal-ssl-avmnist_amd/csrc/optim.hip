// Flat-arena parameter updates: teacher EMA (MultiModalDINO.update_teacher, dino.py:635-646)
// and Adam with L2 weight decay (configure_optimizers, dino.py:953-962).  Both stream the
// arenas once with 16-byte vector accesses (HBM-bound: EMA 12 B/param, Adam 28 B/param).
#include <string.h>

#include "common.h"

using namespace avd;

static thread_local char g_err[128] = "ok";
void avd_set_error(hipError_t e) {
  strncpy(g_err, hipGetErrorString(e), sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

namespace {

__global__ __launch_bounds__(256) void ema_kernel(float* __restrict__ t, const float* __restrict__ s,
                                                  long long n, float m) {
  const float om = 1.f - m;
  const long long n4 = n / 4;
  float4* t4 = reinterpret_cast<float4*>(t);
  const float4* s4 = reinterpret_cast<const float4*>(s);
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 a = t4[i];
    const float4 b = s4[i];
    a.x = m * a.x + om * b.x;
    a.y = m * a.y + om * b.y;
    a.z = m * a.z + om * b.z;
    a.w = m * a.w + om * b.w;
    t4[i] = a;
  }
  for (long long i = n4 * 4 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    t[i] = m * t[i] + om * s[i];
}

// DECOUPLED = false: torch.optim.Adam (wd added to the gradient);
// DECOUPLED = true:  torch.optim.AdamW (p *= 1 - lr*wd before the moment update; the linear
//                    probe's optimiser, dino.py:898)
template <bool DECOUPLED>
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float lr, float b1,
                                      float b2, float eps, float wd, float inv_bc1,
                                      float inv_sqrt_bc2) {
  if (DECOUPLED) p *= 1.f - lr * wd;
  else g = fmaf(wd, p, g);
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
  p -= lr * inv_bc1 * m / denom;
}

template <bool DECOUPLED>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   long long n, float lr, float b1, float b2,
                                                   float eps, float wd, float inv_bc1,
                                                   float inv_sqrt_bc2,
                                                   const float* __restrict__ hyp) {
  if (hyp) {   // per-step scalars from the device step state (graph-replayable steps)
    lr = hyp[0];
    inv_bc1 = 1.f / hyp[1];
    inv_sqrt_bc2 = 1.f / sqrtf(hyp[2]);
  }
  const long long n4 = n / 4;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam1<DECOUPLED>(pp.x, gg.x, mm.x, vv.x, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2);
    adam1<DECOUPLED>(pp.y, gg.y, mm.y, vv.y, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2);
    adam1<DECOUPLED>(pp.z, gg.z, mm.z, vv.z, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2);
    adam1<DECOUPLED>(pp.w, gg.w, mm.w, vv.w, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (long long i = n4 * 4 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    adam1<DECOUPLED>(p[i], g[i], m[i], v[i], lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2);
}

__global__ __launch_bounds__(256) void axpy_kernel(float* __restrict__ y, const float* __restrict__ x,
                                                   long long n, float a) {
  const long long n4 = n / 4;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 yy = reinterpret_cast<float4*>(y)[i];
    const float4 xx = reinterpret_cast<const float4*>(x)[i];
    yy.x = fmaf(a, xx.x, yy.x);
    yy.y = fmaf(a, xx.y, yy.y);
    yy.z = fmaf(a, xx.z, yy.z);
    yy.w = fmaf(a, xx.w, yy.w);
    reinterpret_cast<float4*>(y)[i] = yy;
  }
  for (long long i = n4 * 4 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = fmaf(a, x[i], y[i]);
}

inline int stream_grid(long long n) {
  long long b = (n / 4 + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// One thread: the device step state of a graph-replayable training step (see avdino.h).
__global__ void step_begin_kernel(long long* __restrict__ t, float* __restrict__ hyp,
                                  unsigned long long* __restrict__ seed_off, double b1, double b2,
                                  unsigned long long stride) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long done = t[0];
  if (seed_off) seed_off[0] = (unsigned long long)done * stride;
  const long long k = done + 1;
  t[0] = k;
  hyp[1] = (float)(1.0 - pow(b1, (double)k));
  hyp[2] = (float)(1.0 - pow(b2, (double)k));
}

// BatchNorm num_batches_tracked increments of one forward, all layers at once:
// arena[idx[i]] += val[i] (distinct indices; one thread each)
__global__ void counters_add_kernel(long long* __restrict__ arena, const long long* __restrict__ idx,
                                    const long long* __restrict__ val, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) arena[idx[i]] += val[i];
}

}  // namespace

namespace avd {
avd_options g_opts{};
}  // namespace avd

extern "C" {

int avd_counters_add(long long* arena, const long long* idx, const long long* val, int n,
                     void* stream) {
  if (!arena || !idx || !val) return AVD_ERR_ARG;
  if (n < 0) return AVD_ERR_SHAPE;
  if (n == 0) return AVD_OK;
  counters_add_kernel<<<avd_cdiv(n, 64), 64, 0, avd_stream(stream)>>>(arena, idx, val, n);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_version(void) { return (0 << 16) | 2; }

int avd_set_options(const avd_options* opts) {
  if (opts && (opts->grid_cap < 0 || (opts->generic_conv & ~1) || (opts->generic_m2 & ~1)))
    return AVD_ERR_ARG;
  avd::g_opts = opts ? *opts : avd_options{};
  return AVD_OK;
}

int avd_get_options(avd_options* opts) {
  if (!opts) return AVD_ERR_ARG;
  *opts = avd::g_opts;
  return AVD_OK;
}

const char* avd_last_error(void) { return g_err; }

int avd_ema(float* teacher, const float* student, long long n, float m, void* stream) {
  if (!teacher || !student) return AVD_ERR_ARG;
  if (n < 0 || !aligned16(teacher) || !aligned16(student)) return AVD_ERR_SHAPE;
  if (n == 0) return AVD_OK;
  ema_kernel<<<stream_grid(n), 256, 0, avd_stream(stream)>>>(teacher, student, n, m);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float b1,
             float b2, float eps, float wd, float bc1, float bc2, void* stream) {
  if (!p || !g || !m || !v) return AVD_ERR_ARG;
  if (n < 0 || !aligned16(p) || !aligned16(g) || !aligned16(m) || !aligned16(v)) return AVD_ERR_SHAPE;
  if (n == 0) return AVD_OK;
  adam_kernel<false><<<stream_grid(n), 256, 0, avd_stream(stream)>>>(p, g, m, v, n, lr, b1, b2, eps,
                                                                     wd, 1.f / bc1, 1.f / sqrtf(bc2), nullptr);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_axpy(float* y, const float* x, long long n, float a, void* stream) {
  if (!y || !x) return AVD_ERR_ARG;
  if (n < 0 || !aligned16(y) || !aligned16(x)) return AVD_ERR_SHAPE;
  if (n == 0) return AVD_OK;
  axpy_kernel<<<stream_grid(n), 256, 0, avd_stream(stream)>>>(y, x, n, a);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_adamw(float* p, const float* g, float* m, float* v, long long n, float lr, float b1,
              float b2, float eps, float wd, float bc1, float bc2, void* stream) {
  if (!p || !g || !m || !v) return AVD_ERR_ARG;
  if (n < 0 || !aligned16(p) || !aligned16(g) || !aligned16(m) || !aligned16(v)) return AVD_ERR_SHAPE;
  if (n == 0) return AVD_OK;
  adam_kernel<true><<<stream_grid(n), 256, 0, avd_stream(stream)>>>(p, g, m, v, n, lr, b1, b2, eps,
                                                                    wd, 1.f / bc1, 1.f / sqrtf(bc2), nullptr);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_step_begin(long long* t, float* hyp, unsigned long long* seed_off, double b1, double b2,
                   unsigned long long seed_stride, void* stream) {
  if (!t || !hyp) return AVD_ERR_ARG;
  step_begin_kernel<<<1, 64, 0, avd_stream(stream)>>>(t, hyp, seed_off, b1, b2, seed_stride);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

static int adam_dev(bool decoupled, float* p, const float* g, float* m, float* v, long long n,
                    const float* hyp, float b1, float b2, float eps, float wd, void* stream) {
  if (!p || !g || !m || !v || !hyp) return AVD_ERR_ARG;
  if (n < 0 || !aligned16(p) || !aligned16(g) || !aligned16(m) || !aligned16(v)) return AVD_ERR_SHAPE;
  if (n == 0) return AVD_OK;
  if (decoupled)
    adam_kernel<true><<<stream_grid(n), 256, 0, avd_stream(stream)>>>(p, g, m, v, n, 0.f, b1, b2, eps,
                                                                      wd, 1.f, 1.f, hyp);
  else
    adam_kernel<false><<<stream_grid(n), 256, 0, avd_stream(stream)>>>(p, g, m, v, n, 0.f, b1, b2, eps,
                                                                       wd, 1.f, 1.f, hyp);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

int avd_adam_dev(float* p, const float* g, float* m, float* v, long long n, const float* hyp,
                 float b1, float b2, float eps, float wd, void* stream) {
  return adam_dev(false, p, g, m, v, n, hyp, b1, b2, eps, wd, stream);
}

int avd_adamw_dev(float* p, const float* g, float* m, float* v, long long n, const float* hyp,
                  float b1, float b2, float eps, float wd, void* stream) {
  return adam_dev(true, p, g, m, v, n, hyp, b1, b2, eps, wd, stream);
}

}  // extern "C"
