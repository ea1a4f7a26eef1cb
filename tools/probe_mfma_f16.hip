// Probe (dev tool): what exactly does v_mfma_f32_32x32x16_f16 / _bf16 compute on gfx950?
// Writes A, B, C-in and D for one 32x32x16 tile (and an 8-instruction K=128 chain) to binary
// files; tools/analyze_mfma_f16.py tests candidate accumulation semantics exactly.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mfma_f16.hip -o tools/probe_mfma_f16.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <cmath>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A: 32 x K row-major fp16, B: K x 32 row-major, C: 32x32 fp32 in, D out. K multiple of 16.
__global__ void mfma_f16(const _Float16* A, const _Float16* B, const float* C, float* D, int K, int ld) {
  int l = threadIdx.x;
  f16v acc;
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    acc[r] = C[row * 32 + (l & 31)];
  }
  for (int k0 = 0; k0 < K; k0 += 16) {
    h8 a, b;
    for (int j = 0; j < 8; ++j) {
      int k = k0 + 8 * (l >> 5) + j;
      a[j] = A[(l & 31) * ld + k];
      b[j] = B[k * 32 + (l & 31)];
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    D[row * 32 + (l & 31)] = acc[r];
  }
}

__global__ void mfma_bf16(const uint16_t* A, const uint16_t* B, const float* C, float* D, int K, int ld) {
  int l = threadIdx.x;
  f16v acc;
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    acc[r] = C[row * 32 + (l & 31)];
  }
  for (int k0 = 0; k0 < K; k0 += 16) {
    s8 a, b;
    for (int j = 0; j < 8; ++j) {
      int k = k0 + 8 * (l >> 5) + j;
      a[j] = (short)A[(l & 31) * ld + k];
      b[j] = (short)B[k * 32 + (l & 31)];
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    D[row * 32 + (l & 31)] = acc[r];
  }
}

static uint64_t st = 99;
static uint64_t nxt() { uint64_t z = (st += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }

int main() {
  const int K = 128;
  std::vector<_Float16> A(32 * K), B(K * 32);
  std::vector<uint16_t> Ab(32 * K), Bb(K * 32);
  std::vector<float> C(1024), D(1024), Db(1024);
  for (int i = 0; i < 32 * K; ++i) {
    // wide exponent spread + cancellations
    uint64_t z = nxt();
    float v = ((z & 1) ? -1.f : 1.f) * std::ldexp(1.0f + (float)((z >> 8) & 1023) / 1024.0f, (int)((z >> 20) % 12) - 6);
    A[i] = (_Float16)v;
    uint32_t u; float vb = v; memcpy(&u, &vb, 4); Ab[i] = (uint16_t)(u >> 16);
  }
  for (int i = 0; i < K * 32; ++i) {
    uint64_t z = nxt();
    float v = ((z & 1) ? -1.f : 1.f) * std::ldexp(1.0f + (float)((z >> 8) & 1023) / 1024.0f, (int)((z >> 20) % 12) - 6);
    B[i] = (_Float16)v;
    uint32_t u; float vb = v; memcpy(&u, &vb, 4); Bb[i] = (uint16_t)(u >> 16);
  }
  for (int i = 0; i < 1024; ++i) { uint64_t z = nxt(); C[i] = ((z & 1) ? -1.f : 1.f) * std::ldexp(1.0f + (float)((z >> 8) & 0xFFFFF) / 1048576.0f, (int)((z >> 40) % 10) - 3); }
  _Float16 *dA, *dB; uint16_t *dAb, *dBb; float *dC, *dD, *dDb;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2); hipMalloc(&dAb, Ab.size() * 2); hipMalloc(&dBb, Bb.size() * 2);
  hipMalloc(&dC, 4096); hipMalloc(&dD, 4096); hipMalloc(&dDb, 4096);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dAb, Ab.data(), Ab.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dBb, Bb.data(), Bb.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
  FILE* f = fopen("gpurun_out/mfma_f16_probe.bin", "wb");
  for (int kk : {16, 128}) {
    mfma_f16<<<1, 64>>>(dA, dB, dC, dD, kk, K);
    mfma_bf16<<<1, 64>>>(dAb, dBb, dC, dDb, kk, K);
    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(Db.data(), dDb, 4096, hipMemcpyDeviceToHost);
    fwrite(D.data(), 4, 1024, f);
    fwrite(Db.data(), 4, 1024, f);
  }
  fclose(f);
  f = fopen("gpurun_out/mfma_f16_inputs.bin", "wb");
  fwrite(A.data(), 2, A.size(), f); fwrite(B.data(), 2, B.size(), f);
  fwrite(Ab.data(), 2, Ab.size(), f); fwrite(Bb.data(), 2, Bb.size(), f); fwrite(C.data(), 4, 1024, f);
  fclose(f);
  printf("probe written\n");
  return 0;
}
