// BatchNorm-backward APPLY of one 2x2 pooling window, for kernels that stage the conv-output
// gradient dy into LDS themselves instead of reading a dy tensor written by
// bwd_apply_cl_kernel (bn_cl.hip): the input-gradient and weight-gradient kernels of the
// mid-layer convs (conv_ws.hip, wgrad_ws.hip).  Per channel, bit-identical to that kernel:
//   z_k = max(y_k * scale + shift, 0) (k = the window's 4 pixels), a = first argmax, mx = z_a
//   dz  = mx > 0 ? gout : 0
//   dy_k = bf16(k1 * (k == a ? dz : 0) + (kx * y_k + k0))
// where (k1, kx, k0) are avd_bn_bwd_finalize's per-(group, channel) coefficients.  The
// reference's chain is nn.BatchNorm2d -> ReLU -> MaxPool2d(2) (unimodal.py:185-221) with the
// gradient routed through the pool's argmax (PyTorch's first-max tie rule).
//
// Fusing this into both consumers means dy never reaches HBM: per layer the step reads y and
// the pooled gradient twice (1.25 + 1.25 units of the y size) instead of writing dy and reading
// it twice (2.25 + 1 + 1).
#pragma once
#include "common.h"

namespace avd {

// gout layout: 0 = pooled map NHWC bf16 (the next conv's input gradient); 2 = f32 [N][C*Hp*Wp]
// in the reference's (c, h, w) flatten order (the gradient of the encoder's Linear input)
struct ApplyArgs {
  const void* gout;
  const float* scale;
  const float* shift;
  const float* coef;   // [G*C][3] = (k1, kx, k0)
  int B;               // samples per BN group
  int G;               // groups (<= APPLY_GMAX)
  void* dy = nullptr;  // input-gradient kernel only: also store the dY it forms (tile interiors)
};
constexpr int APPLY_GMAX = 8;

// ctab[g][5][C] = (scale, shift, k1, kx, k0) for every group, once per block
template <int C>
__device__ __forceinline__ void apply_load_ctab(float* ctab, const ApplyArgs& a, int tid, int nthr) {
  for (int i = tid; i < a.G * 5 * C; i += nthr) {
    const int g = i / (5 * C), r = i - g * 5 * C, k = r / C, c = r - k * C;
    const int gc = g * C + c;
    ctab[i] = k == 0 ? a.scale[gc] : k == 1 ? a.shift[gc] : a.coef[gc * 3 + (k - 2)];
  }
}

typedef __attribute__((ext_vector_type(4))) unsigned u4a;

// the prefetched inputs of one window task: 4 pixels x 8 channels of y, 8 pooled gradients
struct WinIn {
  u4a y[4];
  u4a g0, g1;   // gmode 0: g0 = 8 bf16; gmode 2: g0, g1 = 8 f32
};

__device__ __forceinline__ void apply_unpack8(u4a v, float (&f)[8]) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// dy of the window's 4 pixels (order: (0,0), (0,1), (1,0), (1,1)) as packed bf16 vectors.
// ct = ctab + g * 5 * C + c0 (stride C between the 5 coefficient rows).
template <int GMODE, int C>
__device__ __forceinline__ void apply_window(const WinIn& in, const float* ct, u4a (&out)[4]) {
  float yv[4][8], gg[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) apply_unpack8(in.y[k], yv[k]);
  if constexpr (GMODE == 0) {
    apply_unpack8(in.g0, gg);
  } else {
    gg[0] = __uint_as_float(in.g0.x); gg[1] = __uint_as_float(in.g0.y);
    gg[2] = __uint_as_float(in.g0.z); gg[3] = __uint_as_float(in.g0.w);
    gg[4] = __uint_as_float(in.g1.x); gg[5] = __uint_as_float(in.g1.y);
    gg[6] = __uint_as_float(in.g1.z); gg[7] = __uint_as_float(in.g1.w);
  }
  float sc[8], sf[8], k1[8], kx[8], k0[8];
#pragma unroll
  for (int e = 0; e < 8; e += 4) {
    const float4 a = *reinterpret_cast<const float4*>(ct + e);
    const float4 b = *reinterpret_cast<const float4*>(ct + C + e);
    const float4 c = *reinterpret_cast<const float4*>(ct + 2 * C + e);
    const float4 d = *reinterpret_cast<const float4*>(ct + 3 * C + e);
    const float4 f = *reinterpret_cast<const float4*>(ct + 4 * C + e);
    sc[e] = a.x; sc[e + 1] = a.y; sc[e + 2] = a.z; sc[e + 3] = a.w;
    sf[e] = b.x; sf[e + 1] = b.y; sf[e + 2] = b.z; sf[e + 3] = b.w;
    k1[e] = c.x; k1[e + 1] = c.y; k1[e + 2] = c.z; k1[e + 3] = c.w;
    kx[e] = d.x; kx[e + 1] = d.y; kx[e + 2] = d.z; kx[e + 3] = d.w;
    k0[e] = f.x; k0[e + 1] = f.y; k0[e + 2] = f.z; k0[e + 3] = f.w;
  }
  unsigned ow[4][4];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    float d[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = e + h;
      float best = fmaxf(fmaf(yv[0][c], sc[c], sf[c]), 0.f);
      int am = 0;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float r = fmaxf(fmaf(yv[k][c], sc[c], sf[c]), 0.f);
        if (r > best) { best = r; am = k; }
      }
      const float dz = best > 0.f ? gg[c] : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k][h] = fmaf(k1[c], am == k ? dz : 0.f, fmaf(kx[c], yv[k][c], k0[c]));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) ow[k][e >> 1] = pack_bf16x2(d[k][0], d[k][1]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = u4a{ow[k][0], ow[k][1], ow[k][2], ow[k][3]};
}

}  // namespace avd
