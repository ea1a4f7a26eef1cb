// Dev tool: where the 16-bit stream-K Gram spends its cycles (per-workgroup s_memtime sums).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DPT2Q_GRAM_PROFILE \
//   -I include -I snlp---tenary-post-train-quantization_amd/csrc tools/gram_probe.hip -o tools/gram_probe.bin
#include "../snlp---tenary-post-train-quantization_amd/csrc/gemm.hip"

#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  const long N = argc > 1 ? atol(argv[1]) : 262144;
  const int m = argc > 2 ? atoi(argv[2]) : 4096;
  std::vector<_Float16> hx((size_t)N * m);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (_Float16)((float)((i * 2654435761u) % 2001) / 1000.0f - 1.0f);
  void *X, *G, *F;
  hipMalloc(&X, hx.size() * 2);
  hipMalloc(&G, (size_t)m * m * 4);
  hipMalloc(&F, pt2q_gram_flags_ints(m) * 4);
  hipMemcpy(X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  GemmDesc g{};
  g.M = m; g.N = m; g.K = (int)N;
  g.A = X; g.lda = m; g.a_layout = LAY_KMAJOR;
  g.B = X; g.ldb = m; g.b_layout = LAY_KMAJOR;
  g.in_dtype = PT2Q_F16; g.C = (float*)G; g.ldc = m; g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1;
  pt2q_launch_gram(g, (int*)F, 0);
  hipDeviceSynchronize();
  unsigned long long z[4] = {0, 0, 0, 0};
  hipMemcpyToSymbol(HIP_SYMBOL(g16_prof), z, sizeof(z));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  pt2q_launch_gram(g, (int*)F, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long p[4];
  hipMemcpyFromSymbol(p, HIP_SYMBOL(g16_prof), sizeof(p));
  double wgs = (double)p[3];
  printf("gram %ld x %d: %.2f ms; per WG (s_memtime units): wait+reload %.0f  mma %.0f  total %.0f  -> mma %.1f%%, wait %.1f%%, other %.1f%% (wgs %.0f)\n",
         N, m, ms, p[0] / wgs, p[1] / wgs, p[2] / wgs, 100.0 * p[1] / p[2], 100.0 * p[0] / p[2],
         100.0 * (p[2] - p[0] - p[1]) / p[2], wgs);
  return 0;
}
