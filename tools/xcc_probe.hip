// Probe (dev tool): which XCD (XCC_ID) runs workgroup b of a 256 / 512-workgroup grid, and which
// CU.  The Gram / EF / gemmx tile orders assume b % 8 = XCD ("for speed only").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(int* out) {
  if (threadIdx.x == 0) {
    unsigned x, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = x & 0xf;
    out[2 * blockIdx.x + 1] = hw;
    __builtin_amdgcn_s_sleep(100);
  }
}
int main() {
  for (int grid : {256, 512, 1024}) {
    int* d;
    hipMalloc(&d, grid * 8);
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, d);
    std::vector<int> h(2 * grid);
    hipMemcpy(h.data(), d, grid * 8, hipMemcpyDeviceToHost);
    int match = 0;
    for (int b = 0; b < grid; ++b) match += (h[2 * b] == b % 8);
    printf("grid %d: %d of %d workgroups on XCD b %% 8; first 24 XCDs:", grid, match, grid);
    for (int b = 0; b < 24; ++b) printf(" %d", h[2 * b]);
    printf("\n");
    hipFree(d);
  }
  return 0;
}
