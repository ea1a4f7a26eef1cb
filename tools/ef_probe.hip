// Dev tool: time the error-feedback kernel (ef.hip) alone, with build-time knock-outs
// (-DEF_PROBE_NO_MFMA / -DEF_PROBE_NO_C / -DEF_PROBE_NO_DMA) to split its time.
// usage: tools/ef_probe*.bin [n] [nr] [bs] [reps]
#include "../snlp---tenary-post-train-quantization_amd/csrc/ef.hip"

#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int nr = argc > 2 ? atoi(argv[2]) : 2048;
  const int bs = argc > 3 ? atoi(argv[3]) : 128;
  const int reps = argc > 4 ? atoi(argv[4]) : 20;
  const int m = 4096;
  float *Ck, *Et, *Wt;
  int* crow;
  (void)hipMalloc(&Ck, (size_t)128 * m * 4);
  (void)hipMalloc(&Et, (size_t)128 * n * 4);
  (void)hipMalloc(&Wt, (size_t)m * n * 4);
  (void)hipMalloc(&crow, (size_t)m * 4);
  (void)hipMemset(Ck, 0, (size_t)128 * m * 4);
  (void)hipMemset(Et, 0, (size_t)128 * n * 4);
  (void)hipMemset(Wt, 0, (size_t)m * n * 4);
  std::vector<int> h(m);
  for (int e = 0; e < m; ++e) h[e] = (e * 7 + 3) % m;  // a permutation (7 odd, m power of 2)
  (void)hipMemcpy(crow, h.data(), m * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  pt2q_launch_ef(Ck, m, Et, Wt, n, m, crow, nr, bs, 0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) pt2q_launch_ef(Ck, m, Et, Wt, n, m, crow, nr, bs, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / reps;
  const double fl = 2.0 * n * nr * bs;
  printf("ef n=%d nr=%d bs=%d: %.2f us  %.1f TFLOP/s  Wt RMW %.1f GB/s\n", n, nr, bs, us, fl / us / 1e6,
         2.0 * n * nr * 4 / us / 1e3);
  return 0;
}
