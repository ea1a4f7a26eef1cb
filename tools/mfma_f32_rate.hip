// Dev tool: sustained v_mfma_f32_32x32x2_f32 rate (4 independent accumulators per wave, one
// wave per SIMD, every CU), random operands.  hipcc --offload-arch=gfx950 -O3 tools/mfma_f32_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void k(float* out, int iters, float a0, float b0) {
  f32x16 acc[4] = {};
  float a = a0 + threadIdx.x * 1e-3f, b = b0 - threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[u], 0, 0, 0);
  }
  float s = 0;
  for (int u = 0; u < 4; ++u) for (int r = 0; r < 16; ++r) s += acc[u][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  float* o; hipMalloc(&o, 1024 * 256 * 4);
  const int iters = 20000;
  hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, o, 100, 1.0f, 2.0f);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, o, iters, 1.0f, 2.0f);
  hipEventRecord(e1); hipDeviceSynchronize();
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double fl = 256.0 * 4 * iters * 4 * 32 * 32 * 2 * 2;
  printf("f32 32x32x2: %.3f ms  %.1f TFLOP/s  (%.1f cycles/MFMA at 2.4 GHz)\n", ms, fl / ms / 1e9,
         ms * 1e-3 * 2.4e9 / (iters * 4.0));
  return 0;
}
