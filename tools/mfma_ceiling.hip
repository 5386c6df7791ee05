// Practical bf16 MFMA ceiling of the chip: back-to-back
// v_mfma_f32_16x16x32_bf16 with operands in registers, random data, every CU,
// NW waves per SIMD (DVFS: the clock the chip holds under this load sets the
// ceiling a real kernel can approach; MI355X_MICROARCH.md 'DVFS give-back').
// usage: ./mfma_ceiling   (prints TFLOP/s for 1 and 2 waves per SIMD)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_loop(const bf16x8 *in, float *out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const bf16x8 a = in[t & 4095], b = in[(t * 7 + 3) & 4095];
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
  for (int it = 0; it < iters; ++it) {
    // fixed accumulator registers (the compiler otherwise rotates them with
    // accvgpr moves inside the loop)
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %8, %9, %0\n"
        "v_mfma_f32_16x16x32_bf16 %1, %8, %9, %1\n"
        "v_mfma_f32_16x16x32_bf16 %2, %8, %9, %2\n"
        "v_mfma_f32_16x16x32_bf16 %3, %8, %9, %3\n"
        "v_mfma_f32_16x16x32_bf16 %4, %8, %9, %4\n"
        "v_mfma_f32_16x16x32_bf16 %5, %8, %9, %5\n"
        "v_mfma_f32_16x16x32_bf16 %6, %8, %9, %6\n"
        "v_mfma_f32_16x16x32_bf16 %7, %8, %9, %7\n"
        : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), "+a"(c4), "+a"(c5), "+a"(c6), "+a"(c7)
        : "v"(a), "v"(b));
  }
  const f32x4 s = ((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7));
  out[t] = s[0] + s[1] + s[2] + s[3];
}

int main(int argc, char **argv) {
  const bool zeros = argc > 1;   // ./mfma_ceiling 0 : all-zero operands (clock reference)
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<unsigned short> h(4096 * 8);
  unsigned s = 12345;
  for (auto &v : h) { s = s * 1664525u + 1013904223u; v = 0x3c00 + ((s >> 16) & 0x3ff) - 0x200 + ((s >> 31) << 15); }
  bf16x8 *in; float *out;
  hipMalloc(&in, h.size() * 2);
  if (zeros) for (auto &v : h) v = 0;
  hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)ncu * 8 * 256 * 4);
  const int iters = 20000;
  for (int wps = 1; wps <= 2; ++wps) {
    const int blocks = ncu * wps;              // 256 threads = 4 waves = 1 per SIMD
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, in, out, iters / 10);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = 5.0 * blocks * 4.0 * iters * 8 * 16384.0;
    printf("{\"zeros\": %d, \"waves_per_simd\": %d, \"cus\": %d, \"tflops\": %.1f, \"ms\": %.3f}\n", (int)zeros, wps, ncu, fl / (ms * 1e-3) / 1e12, ms);
  }
  return 0;
}
