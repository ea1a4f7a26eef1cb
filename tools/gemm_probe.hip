// Dev tool: time the f32 GEMM shapes of the layer loop in isolation.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//   -I snlp---tenary-post-train-quantization_amd/csrc tools/gemm_probe.hip -o tools/gemm_probe.bin
#include "../snlp---tenary-post-train-quantization_amd/csrc/gemm.hip"

#include <cstdio>
#include <cstdlib>

static float time_gemm(const GemmDesc& g, int reps = 20) {
  pt2q_launch_gemm(g, 0);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) pt2q_launch_gemm(g, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  const int m = 4096, n = 4096;
  float *U, *C, *W;
  int* rows;
  hipMalloc(&U, (size_t)m * m * 4);
  hipMalloc(&C, (size_t)m * m * 4);
  hipMalloc(&W, (size_t)m * n * 4);
  hipMalloc(&rows, m * 4);
  hipMemset(U, 0, (size_t)m * m * 4);
  hipMemset(C, 0, (size_t)m * m * 4);
  hipMemset(W, 0, (size_t)m * n * 4);
  int* hr = (int*)malloc(m * 4);
  for (int i = 0; i < m; ++i) hr[i] = (i * 7919) % m;
  hipMemcpy(rows, hr, m * 4, hipMemcpyHostToDevice);
  for (int rest : {4032, 2048, 1024}) {
    GemmDesc g{};
    g.M = rest; g.N = rest; g.K = 64;
    g.A = U; g.lda = m; g.a_layout = LAY_KMAJOR;
    g.B = U; g.ldb = m; g.b_layout = LAY_KMAJOR;
    g.in_dtype = PT2Q_F32; g.C = C + 64 * m + 64; g.ldc = m;
    g.mode = GEMM_CHAIN_NEG; g.upper = 1;
    float us = time_gemm(g);
    double bytes = (double)rest * rest * 8 / 2;
    printf("trailing upper %d^2 K=64: %.1f us  (C RMW %.1f GB/s)\n", rest, us, bytes / us / 1e3);
  }
  for (int nr : {3968, 2048, 512}) {
    GemmDesc g{};
    g.M = nr; g.N = n; g.K = 128;
    g.A = U; g.lda = m; g.a_layout = LAY_KMAJOR;
    g.B = U; g.ldb = m; g.b_layout = LAY_KMAJOR;
    g.in_dtype = PT2Q_F32; g.C = W; g.ldc = n; g.crow = rows;
    g.mode = GEMM_SUB;
    float us = time_gemm(g);
    double bytes = (double)nr * n * 8;
    printf("EF SUB %d x %d K=128: %.1f us  (C RMW %.1f GB/s)\n", nr, n, us, bytes / us / 1e3);
  }
  {
    GemmDesc g{};
    g.M = m; g.N = m; g.K = m;
    g.A = U; g.lda = m; g.a_layout = LAY_ROWMAJOR;
    g.B = U; g.ldb = m; g.b_layout = LAY_ROWMAJOR;
    g.in_dtype = PT2Q_F32; g.C = C; g.ldc = m;
    g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1; g.kstart_diag = 2;
    float us = time_gemm(g, 5);
    printf("lauum %d: %.1f us (%.1f TF)\n", m, us, (double)m * m * m / 3 * 2 / us / 1e6);
  }
  return 0;
}
