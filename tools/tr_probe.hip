#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[16*64];   // 16 rows x 64 cols
  for (int i = threadIdx.x; i < 16*64; i += 64) lds[i] = (short)((i / 64) * 100 + (i % 64)); // row*100+col
  __syncthreads();
  int l = threadIdx.x; int gi = l & 15; int q = gi >> 2, pp = gi & 3; int g = l >> 4;
  // lane 4q+pp -> row (4g + q), cols 4pp..4pp+3
  int row = 4 * g + q;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds + row * 64 + pp * 4));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64*4*2); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) { printf("lane %2d:", l); for (int e = 0; e < 4; ++e) printf(" %4d", h[l*4+e]); printf("\n"); }
  return 0;
}
