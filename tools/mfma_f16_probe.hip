// Numerics probe (dev tool): what does v_mfma_f32_32x32x16_f16 compute per output element?
// One wave per tile; D = C + A(32x16) B(16x32).  Inputs/outputs are raw files analysed by
// tools/mfma_f16_probe.py.  Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_f16_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef short s8v __attribute__((ext_vector_type(8)));

__global__ void probe(const _Float16* A, const _Float16* B, const float* C, float* D, int bf) {
  const int t = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
  const _Float16* a = A + (size_t)t * 512;
  const _Float16* b = B + (size_t)t * 512;
  h8 av, bv;
  for (int j = 0; j < 8; ++j) {
    av[j] = a[r * 16 + 8 * h + j];
    bv[j] = b[(8 * h + j) * 32 + r];
  }
  f16v acc;
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
    acc[q] = C[(size_t)t * 1024 + row * 32 + r];
  }
  if (bf) {
    s8v ab, bb;
    __builtin_memcpy(&ab, &av, 16);
    __builtin_memcpy(&bb, &bv, 16);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(__bf16 __attribute__((ext_vector_type(8))), ab),
                                                  __builtin_bit_cast(__bf16 __attribute__((ext_vector_type(8))), bb), acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc, 0, 0, 0);
  }
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
    D[(size_t)t * 1024 + row * 32 + r] = acc[q];
  }
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  char p[512];
  snprintf(p, sizeof p, "%s/probe_in.bin", dir);
  FILE* f = fopen(p, "rb");
  if (!f) { printf("no input\n"); return 1; }
  int tiles = 0;
  fread(&tiles, 4, 1, f);
  std::vector<_Float16> A((size_t)tiles * 512), B((size_t)tiles * 512);
  std::vector<float> C((size_t)tiles * 1024), D((size_t)tiles * 1024);
  fread(A.data(), 2, A.size(), f);
  fread(B.data(), 2, B.size(), f);
  fread(C.data(), 4, C.size(), f);
  fclose(f);
  _Float16 *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
  const int bf = argc > 2 && argv[2][0] == 'b';
  hipLaunchKernelGGL(probe, dim3(tiles), dim3(64), 0, 0, dA, dB, dC, dD, bf);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  snprintf(p, sizeof p, "%s/probe_out.bin", dir);
  f = fopen(p, "wb");
  fwrite(D.data(), 4, D.size(), f);
  fclose(f);
  printf("probe done %d tiles\n", tiles);
  return 0;
}
