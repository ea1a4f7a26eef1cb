// Numerics probe for gfx950 (dev tool, not product code).
// Checks the assumptions the PT2Q arithmetic contract relies on:
//   1. v_mfma_f32_32x32x2_f32 / 16x16x4 accumulate as a k-ordered fmaf chain.
//   2. f32 division and sqrtf are correctly rounded under our build flags.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probe_numerics.hip -o /tmp/probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 2; } } while (0)

// C[32x32] = sum_k A[i][k] B[k][j], K even, A row-major 32xK, B row-major Kx32
__global__ void mfma32(const float* A, const float* B, float* C, int K) {
  int l = threadIdx.x;
  f32x16 acc = {0};
  for (int k0 = 0; k0 < K; k0 += 2) {
    float a = A[(l & 31) * K + k0 + (l >> 5)];
    float b = B[(k0 + (l >> 5)) * 32 + (l & 31)];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    C[row * 32 + (l & 31)] = acc[r];
  }
}

__global__ void mfma16(const float* A, const float* B, float* C, int K) {
  int l = threadIdx.x;
  f32x4 acc = {0};
  for (int k0 = 0; k0 < K; k0 += 4) {
    float a = A[(l & 15) * K + k0 + (l >> 4)];
    float b = B[(k0 + (l >> 4)) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) * 4 + r;
    C[row * 16 + (l & 15)] = acc[r];
  }
}

__global__ void divsqrt(const float* x, const float* y, float* q, float* s, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { q[i] = x[i] / y[i]; s[i] = sqrtf(fabsf(x[i])); }
}

static uint64_t sm(uint64_t& s) { uint64_t z = (s += 0x9E3779B97F4A7C15ull); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }
static float rnd(uint64_t& s) { // wide dynamic range, both signs
  uint64_t z = sm(s); float m = (float)((z >> 40) & 0xFFFFFF) / 16777216.0f; int e = (int)((z >> 8) & 15) - 8;
  return ((z & 1) ? -1.f : 1.f) * std::ldexp(0.5f + m, e);
}
static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main() {
  uint64_t seed = 12345;
  int fails = 0;
  for (int K : {2, 4, 64, 1024}) {
    std::vector<float> A(32 * K), B(K * 32), C(32 * 32);
    for (auto& v : A) v = rnd(seed);
    for (auto& v : B) v = rnd(seed);
    float *dA, *dB, *dC;
    CK(hipMalloc(&dA, A.size() * 4)); CK(hipMalloc(&dB, B.size() * 4)); CK(hipMalloc(&dC, C.size() * 4));
    CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    mfma32<<<1, 64>>>(dA, dB, dC, K);
    CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
    int bad_chain = 0, bad_pair = 0;
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc = std::fmaf(A[i * K + k], B[k * 32 + j], acc);
      if (bits(acc) != bits(C[i * 32 + j])) ++bad_chain;
      // alternative hypothesis: exact pair products summed then one rounding per pair
      double accd = 0.0; float accp = 0.f;
      for (int k = 0; k < K; k += 2) { accd = (double)accp + (double)A[i*K+k]*B[k*32+j] + (double)A[i*K+k+1]*B[(k+1)*32+j]; accp = (float)accd; }
      if (bits(accp) != bits(C[i * 32 + j])) ++bad_pair;
    }
    printf("mfma32x32x2 K=%d: mismatches vs fmaf-chain %d, vs pair-rounded %d (of 1024)\n", K, bad_chain, bad_pair);
    fails += bad_chain;
    hipFree(dA); hipFree(dB); hipFree(dC);
  }
  for (int K : {4, 64, 1024}) {
    std::vector<float> A(16 * K), B(K * 16), C(16 * 16);
    for (auto& v : A) v = rnd(seed);
    for (auto& v : B) v = rnd(seed);
    float *dA, *dB, *dC;
    CK(hipMalloc(&dA, A.size() * 4)); CK(hipMalloc(&dB, B.size() * 4)); CK(hipMalloc(&dC, C.size() * 4));
    CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    mfma16<<<1, 64>>>(dA, dB, dC, K);
    CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc = std::fmaf(A[i * K + k], B[k * 16 + j], acc);
      if (bits(acc) != bits(C[i * 16 + j])) ++bad;
    }
    printf("mfma16x16x4 K=%d: mismatches vs fmaf-chain %d (of 256)\n", K, bad);
    hipFree(dA); hipFree(dB); hipFree(dC);
  }
  {
    const int n = 1 << 22;
    std::vector<float> x(n), y(n), q(n), s(n);
    for (int i = 0; i < n; ++i) { x[i] = rnd(seed); y[i] = rnd(seed); }
    float *dx, *dy, *dq, *ds;
    CK(hipMalloc(&dx, n * 4)); CK(hipMalloc(&dy, n * 4)); CK(hipMalloc(&dq, n * 4)); CK(hipMalloc(&ds, n * 4));
    CK(hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice));
    divsqrt<<<(n + 255) / 256, 256>>>(dx, dy, dq, ds, n);
    CK(hipMemcpy(q.data(), dq, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost));
    int bq = 0, bs = 0;
    for (int i = 0; i < n; ++i) {
      volatile float qq = x[i] / y[i]; volatile float ss = std::sqrt(std::fabs(x[i]));
      if (bits(qq) != bits(q[i])) ++bq;
      if (bits(ss) != bits(s[i])) ++bs;
    }
    printf("div mismatches %d, sqrt mismatches %d (of %d)\n", bq, bs, n);
    fails += bq + bs;
  }
  printf(fails ? "PROBE: FAIL\n" : "PROBE: OK\n");
  return fails ? 1 : 0;
}
