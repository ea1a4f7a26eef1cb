// Dev tool: time the error-feedback kernel (ef.hip) alone on random data, with build-time
// knock-outs from csrc/probe.hpp (-DPT2Q_PROBE=8: Wt loads / stores dropped, 16: no MFMAs,
// 32: operand DMAs all from one chunk) to split its time.  tools/build_ef_probe.sh builds them.
// usage: tools/_probe/ef_probe_<mask> [n] [nr] [bs] [reps] [part]
#include "../snlp---tenary-post-train-quantization_amd/csrc/ef.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384;
  const int nr = argc > 2 ? atoi(argv[2]) : 4096;
  const int bs = argc > 3 ? atoi(argv[3]) : 128;
  const int reps = argc > 4 ? atoi(argv[4]) : 20;
  const bool part = argc > 5 ? atoi(argv[5]) != 0 : true;
  const int m = nr + bs;
  float *Ck, *Et, *Wt, *P;
  int* crow;
  (void)hipMalloc(&Ck, (size_t)bs * m * 4);
  (void)hipMalloc(&Et, (size_t)bs * n * 4);
  (void)hipMalloc(&Wt, (size_t)m * n * 4);
  (void)hipMalloc(&P, (size_t)((nr + 127) / 128) * n * 4);
  (void)hipMalloc(&crow, (size_t)m * 4);
  std::vector<float> h((size_t)m * n);
  unsigned s = 12345u;
  for (auto& v : h) {
    s = s * 1664525u + 1013904223u;
    v = ((int)(s >> 9) - (1 << 22)) * (1.0f / (1 << 22));
  }
  (void)hipMemcpy(Wt, h.data(), (size_t)m * n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(Ck, h.data(), (size_t)bs * m * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(Et, h.data() + 7, (size_t)bs * n * 4, hipMemcpyHostToDevice);
  std::vector<int> r(m);
  for (int e = 0; e < m; ++e) r[e] = (int)(((long)e * 7919 + 3) % m);  // a permutation (gcd(7919, m) = 1)
  (void)hipMemcpy(crow, r.data(), m * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float* pp = part ? P : nullptr;
  int rc = pt2q_launch_ef(Ck, m, Et, Wt, n, m, crow, nr, bs, 0, nullptr, pp, n);
  (void)hipDeviceSynchronize();
  if (rc) {
    printf("launch error %d\n", rc);
    return 1;
  }
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) pt2q_launch_ef(Ck, m, Et, Wt, n, m, crow, nr, bs, 0, nullptr, pp, n);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / reps;
  const double fl = 2.0 * n * nr * bs;
  const long tiles = (long)((nr + 127) / 128) * ((n + 127) / 128);
  printf("ef probe %d/%d n=%d nr=%d bs=%d part=%d: %.1f us  %.1f TFLOP/s  Wt RMW %.0f GB/s  %.2f us/tile/CU\n",
         PT2Q_PROBE, PT2Q_EF2_KPROBE, n, nr, bs, (int)part, us, fl / us / 1e6, 2.0 * n * nr * 4 / us / 1e3, us * 256 / tiles);
#if (PT2Q_PROBE & 64) != 0
  // ef2_gemm_kernel's clock over the last launch: sum over workgroups of the s_memtime cycles
  // divided by the s_memrealtime ticks (100 MHz)
  static long long ck[1024][4];
  (void)hipMemcpyFromSymbol(ck, HIP_SYMBOL(ef2_clk), sizeof(ck));
  double cyc = 0, rt = 0;
  int wgs = 0;
  for (int w = 0; w < 1024; ++w)
    if (ck[w][1] && ck[w][3] > ck[w][1]) {
      cyc += (double)(ck[w][2] - ck[w][0]);
      rt += (double)(ck[w][3] - ck[w][1]);
      ++wgs;
    }
  printf("  kprobe %d: clock %.2f GHz, workgroup %.1f us (%d workgroups)\n", PT2Q_EF2_KPROBE,
         rt > 0 ? cyc / rt * 0.1 : 0.0, wgs ? rt / wgs / 100.0 : 0.0, wgs);
#endif
  return 0;
}
