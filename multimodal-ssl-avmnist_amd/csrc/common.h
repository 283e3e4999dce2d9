// Shared device helpers for libavdino (gfx950 / CDNA4: wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/avdino.h"

namespace avd {

// The library's launch options (avd_set_options, include/avdino.h): test hooks set explicitly
// through the C ABI; no environment variable is read anywhere in the library.
extern avd_options g_opts;

// avd_options.grid_cap: caps the persistent kernels' grids (conv_ws, wgrad_ws, conv_ws8, the
// conv1 passes) at n blocks, so at test sizes every block walks several tiles -- the cross-tile
// loop, the LDS reuse barrier and the next-tile prefetch run exactly as at bench size.  0 (the
// default) changes nothing.
inline int grid_cap(int grid) {
  const int c = g_opts.grid_cap;
  return (c > 0 && c < grid) ? c : grid;
}

typedef uint16_t bf16;

__device__ __forceinline__ float bf2f(bf16 v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN kept NaN): the hardware v_cvt_pk_bf16_f32 (CDNA4),
// which a plain cast emits -- one VALU op for two values instead of ~6 integer ops each.
__device__ __forceinline__ bf16 f2bf(float f) { return __builtin_bit_cast(bf16, (__bf16)f); }
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_hw;
// two values -> one dword (a in the low half): a single v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16x2_hw v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// 16-byte load through the global address space.  A pointer selected between a tensor and a
// __device__ zero vector is otherwise a generic pointer, i.e. a flat_load, which also counts in
// lgkmcnt: every later LDS wait would then wait for the (prefetch) loads to land as well.
typedef __attribute__((ext_vector_type(4))) unsigned u4v;
__device__ __forceinline__ u4v ldg16(const void* p) {
  return *(const __attribute__((address_space(1))) u4v*)p;
}

template <typename T> struct io;
template <> struct io<float> {
  static __device__ __forceinline__ float ld(const float* p, size_t i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, size_t i, float v) { p[i] = v; }
  static __device__ __forceinline__ float rnd(float v) { return v; }
};
template <> struct io<bf16> {
  static __device__ __forceinline__ float ld(const bf16* p, size_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void st(bf16* p, size_t i, float v) { p[i] = f2bf(v); }
  static __device__ __forceinline__ float rnd(float v) { return bf2f(f2bf(v)); }
};

constexpr int WAVE = 64;

// Division by a block-uniform divisor through an f32 reciprocal: exact for 0 <= p < 2^22
// ((p + 0.5)/d sits >= 0.5/d from an integer; the two roundings err by <= (p+0.5)/d * 2^-23).
// Replaces ~30-instruction integer divisions in index decoding of the conv kernels.
struct FastDiv {
  float r;
  int d;
  __device__ __forceinline__ explicit FastDiv(int dd) : r(1.0f / (float)dd), d(dd) {}
  __device__ __forceinline__ int div(int p) const { return (int)(((float)p + 0.5f) * r); }
  __device__ __forceinline__ int mod(int p) const { return p - div(p) * d; }
};

// Exact unsigned 32-bit division by a run-time constant d (1 <= d < 2^31), set up on the host
// (Granlund-Montgomery): q = (t + ((n - t) >> 1)) >> s with t = umulhi(m, n).  Replaces the
// 64-bit division chains of flat-index decompositions (~4 VALU instead of ~40).
struct U32Div {
  unsigned m;
  int s;      // -1: d == 1
  __host__ __device__ static U32Div make(unsigned d) {
    U32Div r{0u, -1};
    if (d <= 1) return r;
    int l = 0;
    while ((1ull << l) < d) ++l;
    r.m = (unsigned)((((1ull << l) - d) << 32) / d + 1);
    r.s = l - 1;
    return r;
  }
  __device__ __forceinline__ unsigned div(unsigned n) const {
    if (s < 0) return n;
    const unsigned t = __umulhi(m, n);
    return (t + ((n - t) >> 1)) >> s;
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64).  `sh` needs NT/64 floats.
// Result valid in every thread.  Deterministic (fixed tree).
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += sh[i];
  return r;
}

// Counter-based hash (murmur3 finaliser on a mixed 64-bit counter): dropout masks that
// forward and backward regenerate identically from (seed, element index).
__device__ __forceinline__ uint32_t hash_u32(unsigned long long seed, unsigned long long idx) {
  unsigned long long x = seed * 0x9E3779B97F4A7C15ull ^ (idx + 0xD1B54A32D192ED03ull);
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}
// Keep-scale for inverted dropout: 0 or 1/(1-p).
__device__ __forceinline__ float dropout_scale(unsigned long long seed, unsigned long long idx, float p) {
  if (p <= 0.f) return 1.f;
  float u = (hash_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// sum over each 16-lane row (the MFMA C columns) with DPP adds: quad swaps, half-row and
// row mirrors; no LDS traffic (a __shfl_xor is a ds_bpermute)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);    // row_half_mirror
  v += dpp_f<0x140>(v);    // row_mirror
  return v;
}


}  // namespace avd

#define AVD_CHECK_LAUNCH()                                  \
  do {                                                      \
    hipError_t e_ = hipGetLastError();                      \
    if (e_ != hipSuccess) { avd_set_error(e_); return AVD_ERR_HIP; } \
  } while (0)

void avd_set_error(hipError_t e);

static inline hipStream_t avd_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int avd_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
