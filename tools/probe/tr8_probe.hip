#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(2))) int i2;
__global__ void k(int* out, int mode) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  for (int a = threadIdx.x; a < 1024; a += 64) s[a] = mode ? (a % 8) : (a / 8);
  __syncthreads();
  const int l = threadIdx.x;
  i2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i2*)(reinterpret_cast<uintptr_t>(s + 8 * l)));
  out[2 * l] = v.x; out[2 * l + 1] = v.y;
}
int main() {
  int* d; hipMalloc(&d, 512);
  int h[2][128];
  for (int m = 0; m < 2; ++m) {
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d, m);
    hipMemcpy(h[m], d, 512, hipMemcpyDeviceToHost);
  }
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) {
      const unsigned char* b0 = (const unsigned char*)&h[0][2 * l];
      const unsigned char* b1 = (const unsigned char*)&h[1][2 * l];
      printf(" (L%d,b%d)", b0[j], b1[j]);
    }
    printf("\n");
  }
  return 0;
}
