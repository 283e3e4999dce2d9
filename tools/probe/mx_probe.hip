#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef __attribute__((ext_vector_type(8))) int i8v;
typedef __attribute__((ext_vector_type(4))) float f4;

// A: [16][128] fp8 bytes, B: [128][16] bytes (stored k-major: B[k][n]); lane l: row/col l&15, k = 32*(l>>4)+j
template <int SEL>
__global__ void probe_sel(const unsigned char* A, const unsigned char* B, float* D, int sa, int sb) {
  const int l = threadIdx.x;
  i8v a, b;
  unsigned char* pa = (unsigned char*)&a;
  unsigned char* pb = (unsigned char*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, SEL, sa, SEL, sb);
  for (int i = 0; i < 4; ++i) D[((l >> 4) * 4 + i) * 16 + (l & 15)] = c[i];
}
// scale registers given per lane (arrays)
__global__ void probe_lane(const unsigned char* A, const unsigned char* B, float* D, const int* sa, const int* sb) {
  const int l = threadIdx.x;
  i8v a, b;
  unsigned char* pa = (unsigned char*)&a;
  unsigned char* pb = (unsigned char*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 4; ++i) D[((l >> 4) * 4 + i) * 16 + (l & 15)] = c[i];
}
__global__ void probe(const unsigned char* A, const unsigned char* B, float* D, int sa, int sb) {
  const int l = threadIdx.x;
  i8v a, b;
  unsigned char* pa = (unsigned char*)&a;
  unsigned char* pb = (unsigned char*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  for (int i = 0; i < 4; ++i) D[((l >> 4) * 4 + i) * 16 + (l & 15)] = c[i];
}

__global__ void rate(float* out, int iters, int sa) {
  i8v a, b;
  for (int j = 0; j < 8; ++j) { a[j] = 0x38383838 ^ (threadIdx.x + j); b[j] = 0x30303030 + j; }
  f4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c0, 0, 0, 0, sa, 0, sa);
    c1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c1, 0, 0, 0, sa, 0, sa);
    c2 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, c2, 0, 0, 0, sa, 0, sa);
    c3 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, b, c3, 0, 0, 0, sa, 0, sa);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
__global__ void rate_bf16(float* out, int iters) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(threadIdx.x * 0.001f + j); b[j] = (__bf16)(0.5f * j); }
  f4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

// e4m3fn encode of small integers (exact for |v| <= 16)
unsigned char enc(int v) {
  if (v == 0) return 0;
  unsigned s = v < 0 ? 0x80 : 0; int a = abs(v);
  int e = 0; while ((1 << (e + 1)) <= a) ++e;        // a in [2^e, 2^(e+1))
  int m = (a - (1 << e)) * 8 >> e;                    // 3 mantissa bits (exact for a<=16)
  return s | ((e + 7) << 3) | m;
}

int main() {
  unsigned char hA[16 * 128], hB[128 * 16];
  int iA[16 * 128], iB[128 * 16];
  srand(3);
  for (int i = 0; i < 16 * 128; ++i) { iA[i] = rand() % 9 - 4; hA[i] = enc(iA[i]); }
  for (int i = 0; i < 128 * 16; ++i) { iB[i] = rand() % 7 - 3; hB[i] = enc(iB[i]); }
  unsigned char *dA, *dB; float* dD;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  int scales[][2] = {{127, 127}, {128, 127}, {127, 125}, {130, 120}};
  for (auto& sc : scales) {
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, dA, dB, dD, sc[0], sc[1]);
    float hD[256]; hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    double f = ldexp(1.0, sc[0] - 127 + sc[1] - 127);
    int bad = 0;
    for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) {
      long s = 0; for (int k = 0; k < 128; ++k) s += iA[m * 128 + k] * iB[k * 16 + n];
      if (fabs(hD[m * 16 + n] - s * f) > 1e-6) { if (bad < 4) printf("  m%d n%d got %g want %g\n", m, n, hD[m*16+n], s * f); ++bad; }
    }
    printf("scales %d %d: %d mismatches\n", sc[0], sc[1], bad);
  }
  for (int sel = 0; sel < 4; ++sel) {
    // the wanted scales in byte `sel`, other bytes junk (0x7c = 2^-3, 0x85 = 2^6)
    int want_a = 128, want_b = 126;
    unsigned ra = 0x857c857cu, rb = 0x7c857c85u;
    ra = (ra & ~(0xffu << (8 * sel))) | ((unsigned)want_a << (8 * sel));
    rb = (rb & ~(0xffu << (8 * sel))) | ((unsigned)want_b << (8 * sel));
    switch (sel) {
      case 0: hipLaunchKernelGGL(probe_sel<0>, 1, 64, 0, 0, dA, dB, dD, (int)ra, (int)rb); break;
      case 1: hipLaunchKernelGGL(probe_sel<1>, 1, 64, 0, 0, dA, dB, dD, (int)ra, (int)rb); break;
      case 2: hipLaunchKernelGGL(probe_sel<2>, 1, 64, 0, 0, dA, dB, dD, (int)ra, (int)rb); break;
      default: hipLaunchKernelGGL(probe_sel<3>, 1, 64, 0, 0, dA, dB, dD, (int)ra, (int)rb); break;
    }
    float hD[256]; hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    long s00 = 0; for (int k = 0; k < 128; ++k) s00 += iA[k] * iB[k * 16];
    int bad = 0;
    for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) {
      long s = 0; for (int k = 0; k < 128; ++k) s += iA[m * 128 + k] * iB[k * 16 + n];
      if (fabs(hD[m * 16 + n] - s * 0.5) > 1e-6) ++bad;
    }
    printf("opsel %d: %d mismatches (D00 %g, exact %ld -> ratio %g)\n", sel, bad, hD[0], s00, s00 ? hD[0] / s00 : 0.0);
  }
  {
    int *dsa, *dsb; hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
    for (int which = 0; which < 2; ++which) {
      for (int L = 0; L < 64; ++L) {
        int hsa[64], hsb[64];
        for (int i = 0; i < 64; ++i) { hsa[i] = 127; hsb[i] = 127; }
        (which ? hsb : hsa)[L] = 128;
        hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe_lane, 1, 64, 0, 0, dA, dB, dD, dsa, dsb);
        float hD[256]; hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
        // which (row-or-col, kblock) changed: D - exact = partial sum over one kblock
        int found = 0;
        for (int rc = 0; rc < 16 && !found; ++rc) for (int kb = 0; kb < 4 && !found; ++kb) {
          bool ok = true;
          for (int m = 0; m < 16 && ok; ++m) for (int n = 0; n < 16 && ok; ++n) {
            long s = 0, p = 0;
            for (int k = 0; k < 128; ++k) { long t = iA[m * 128 + k] * iB[k * 16 + n]; s += t; if (k / 32 == kb) p += t; }
            bool hit = which ? (n == rc) : (m == rc);
            double want = s + (hit ? p : 0);
            if (fabs(hD[m * 16 + n] - want) > 1e-6) ok = false;
          }
          if (ok) { printf("%s lane %2d -> %s %2d kblock %d\n", which ? "B" : "A", L, which ? "col" : "row", rc, kb); found = 1; }
        }
        if (!found) {
          // which outputs changed, and as which subset of kblock partials (rows of A / cols of B)
          printf("%s lane %2d:", which ? "B" : "A", L);
          int shown = 0;
          for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) {
            long s = 0, p[16];
            for (int i = 0; i < 16; ++i) p[i] = 0;
            for (int k = 0; k < 128; ++k) { long t = iA[m * 128 + k] * iB[k * 16 + n]; s += t; p[k / 8] += t; }
            double d = hD[m * 16 + n] - s;
            if (fabs(d) < 1e-6) continue;
            int mask = -1;
            for (int c = 0; c < 65536; ++c) {
              double w = 0; for (int kb = 0; kb < 16; ++kb) if (c >> kb & 1) w += p[kb];
              if (fabs(w - d) < 1e-6) { mask = c; break; }
            }
            if (shown < 3) printf(" (%d,%d 8B-pieces %04x)", m, n, mask);
            ++shown;
          }
          printf(" total %d\n", shown);
        }
      }
    }
  }
  float* o; hipMalloc(&o, 1024 * 256 * 4 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    int iters = 4096, blocks = 256 * 8;
    hipEventRecord(e0); hipLaunchKernelGGL(rate, blocks, 256, 0, 0, o, iters, 127); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 16 * 16 * 128 * 4.0 * iters * blocks * 4;
    printf("mx fp8: %.1f TF/s\n", fl / ms / 1e9);
    hipEventRecord(e0); hipLaunchKernelGGL(rate_bf16, blocks, 256, 0, 0, o, iters); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    fl = 2.0 * 16 * 16 * 32 * 4.0 * iters * blocks * 4;
    printf("bf16: %.1f TF/s\n", fl / ms / 1e9);
  }
  return 0;
}
