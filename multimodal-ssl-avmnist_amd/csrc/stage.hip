// Input staging: the reference feeds the encoder one view at a time
// (MultiModalDINO.forward, dino.py:680-704: global_images[:, v] ...) from collated batches
// [B, V, 1, H, W].  Here all views of a step go through each conv layer in one launch, so the
// batch is re-laid view-major: out[n = v*B + b] = views[b, v] for the global views, then the
// local views, then (optionally) the un-augmented originals [B, 1, H, W] used by the
// MSE / InfoNCE / supervised heads (dino.py:1168-1169).  Optional cast to bf16.
#include "common.h"

using namespace avd;

namespace {

template <typename TO>
__global__ __launch_bounds__(256) void stage_kernel(const float* __restrict__ g, int G,
                                                    const float* __restrict__ l, int L,
                                                    const float* __restrict__ orig, int B,
                                                    int HW4, TO* __restrict__ out, long long total4) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const int p = (int)(i % HW4);
    const long long n = i / HW4;
    const int v = (int)(n / B), b = (int)(n % B);
    const float4* src;
    if (v < G) src = reinterpret_cast<const float4*>(g) + ((size_t)b * G + v) * HW4;
    else if (v < G + L) src = reinterpret_cast<const float4*>(l) + ((size_t)b * L + (v - G)) * HW4;
    else src = reinterpret_cast<const float4*>(orig) + (size_t)b * HW4;
    const float4 x = src[p];
    io<TO>::st(out, 4 * i + 0, x.x);
    io<TO>::st(out, 4 * i + 1, x.y);
    io<TO>::st(out, 4 * i + 2, x.z);
    io<TO>::st(out, 4 * i + 3, x.w);
  }
}

}  // namespace

extern "C" int avd_stage_views(const float* g, int G, const float* l, int L, const float* orig,
                               int B, int HW, void* out, int odt, void* stream) {
  if (!g || !out || (L > 0 && !l)) return AVD_ERR_ARG;
  if (B <= 0 || G <= 0 || L < 0 || HW <= 0 || HW % 4) return AVD_ERR_SHAPE;
  const int nv = G + L + (orig ? 1 : 0);
  const long long total4 = (long long)nv * B * (HW / 4);
  long long blocks = (total4 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipStream_t st = avd_stream(stream);
  if (odt == AVD_F32)
    stage_kernel<float><<<(int)blocks, 256, 0, st>>>(g, G, l, L, orig, B, HW / 4, (float*)out, total4);
  else if (odt == AVD_BF16)
    stage_kernel<bf16><<<(int)blocks, 256, 0, st>>>(g, G, l, L, orig, B, HW / 4, (bf16*)out, total4);
  else
    return AVD_ERR_DTYPE;
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// ---------------------------------------------------------------------------- timeline marks
// One lane stores the GPU's constant-rate real-time counter (s_memrealtime, 100 MHz) into
// marks[idx] when the stream reaches this launch: phase boundaries of a captured step, timed
// without a profiler (whose per-dispatch tracing stretches a replayed graph's timeline).
namespace {
__global__ void mark_kernel(unsigned long long* __restrict__ marks, int idx) {
  if (threadIdx.x == 0) marks[idx] = wall_clock64();
}

// Launch spans: spans[3 slot] = the counter at the begin mark, spans[3 slot + 1] += end - begin,
// spans[3 slot + 2] += 1 -- the in-graph duration of one launch site summed over replays.
__global__ void mark_span_kernel(unsigned long long* __restrict__ spans, int slot, int end) {
  if (threadIdx.x != 0) return;
  const unsigned long long t = wall_clock64();
  unsigned long long* s = spans + 3 * (size_t)slot;
  if (!end) {
    s[0] = t;
  } else {
    s[1] += t - s[0];
    s[2] += 1;
  }
}
}  // namespace

extern "C" int avd_mark_span(unsigned long long* spans, int slot, int end, void* stream) {
  if (!spans || slot < 0) return AVD_ERR_ARG;
  mark_span_kernel<<<1, 64, 0, avd_stream(stream)>>>(spans, slot, end);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

extern "C" int avd_mark(unsigned long long* marks, int idx, void* stream) {
  if (!marks || idx < 0) return AVD_ERR_ARG;
  mark_kernel<<<1, 64, 0, avd_stream(stream)>>>(marks, idx);
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}

// Test hook: every block fills its 64 KB of LDS with NaN bit patterns and exits; 8 blocks per CU
// slot cover every CU's LDS several times over.  A later kernel that reads LDS it never wrote
// then reads NaN (tools/lds_poison.py finds such reads by comparing results with and without).
__global__ __launch_bounds__(1024) void lds_poison_kernel() {
  extern __shared__ __attribute__((aligned(16))) unsigned lds_all[];
  constexpr int WORDS = 64 * 1024 / 4;
  for (int i = threadIdx.x; i < WORDS; i += blockDim.x) lds_all[i] = 0x7fc07fc0u;
  __syncthreads();
  // keep the stores: a value read back decides nothing, but the compiler cannot drop the loop
  if (lds_all[(threadIdx.x * 37) % WORDS] == 1u) lds_all[0] = 0u;
}

extern "C" int avd_lds_poison(void* stream) {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  lds_poison_kernel<<<cus * 8, 1024, 64 * 1024, avd_stream(stream)>>>();
  AVD_CHECK_LAUNCH();
  return AVD_OK;
}
