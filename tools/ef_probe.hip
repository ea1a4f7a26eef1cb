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
  printf("ef probe %d n=%d nr=%d bs=%d part=%d: %.1f us  %.1f TFLOP/s  Wt RMW %.0f GB/s  %.2f us/tile/CU\n",
         PT2Q_PROBE, n, nr, bs, (int)part, us, fl / us / 1e6, 2.0 * n * nr * 4 / us / 1e3, us * 256 / tiles);
#if (PT2Q_PROBE & 64) != 0
  // phase durations (s_memrealtime ticks, 100 MHz -> us) of tiles 1..6 of the first 64 workgroups
  // (the stamps of the last launch): 0 top, 1 stage 0 landed, 2 barrier, 3 half 0 done,
  // 4 stage 1 landed, 5 barrier, 6 half 1 done, 7 old values landed
  static long long st[64][8][12];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(ef_stamps), sizeof(st));
  const char* nm[8] = {"wait stage0", "barrier0", "half0", "wait stage1", "barrier1", "half1", "wait old Wt", "epilogue+loop"};
  {  // the mid-tile gap (3 -> 4) in pieces: lgkmcnt + barrier, next stage-0 DMA issue, w-bar store, vmcnt
    double g[4] = {0};
    int c2 = 0;
    for (int w = 0; w < 64; ++w)
      for (int t = 1; t < 7; ++t) {
        if (!st[w][t][3] || !st[w][t][8]) continue;
        g[0] += (double)(st[w][t][8] - st[w][t][3]);
        g[1] += (double)(st[w][t][9] - st[w][t][8]);
        g[2] += (double)(st[w][t][10] - st[w][t][9]);
        g[3] += (double)(st[w][t][4] - st[w][t][10]);
        ++c2;
      }
    if (c2)
      printf("  mid-tile: barrier %.2f us, stage-0 DMA issue %.2f us, w-bar store %.2f us, stage-1 wait %.2f us\n",
             g[0] / c2 / 100.0, g[1] / c2 / 100.0, g[2] / c2 / 100.0, g[3] / c2 / 100.0);
  }
  double sum[8] = {0};
  int cnt = 0;
  for (int w = 0; w < 64; ++w)
    for (int t = 1; t < 7; ++t) {
      if (!st[w][t][0] || !st[w][t + 1][0]) continue;
      for (int i = 0; i < 7; ++i) sum[i] += (double)(st[w][t][i + 1] - st[w][t][i]);
      sum[7] += (double)(st[w][t + 1][0] - st[w][t][7]);
      ++cnt;
    }
  double tot = 0;
  for (int i = 0; i < 8; ++i) tot += sum[i];
  for (int i = 0; i < 8; ++i)
    printf("  %-14s %7.2f us  %5.1f %%\n", nm[i], cnt ? sum[i] / cnt / 100.0 : 0.0, tot > 0 ? 100.0 * sum[i] / tot : 0.0);
  printf("  tile           %7.2f us  (%d samples)\n", cnt ? tot / cnt / 100.0 : 0.0, cnt);
  static long long ck[64][8][2];
  (void)hipMemcpyFromSymbol(ck, HIP_SYMBOL(ef_clk), sizeof(ck));
  double cyc = 0, rt = 0;
  for (int w = 0; w < 64; ++w)
    for (int t = 1; t < 7; ++t)
      if (st[w][t][0] && st[w][t][7]) {
        cyc += (double)(ck[w][t][1] - ck[w][t][0]);
        rt += (double)(st[w][t][7] - st[w][t][0]);
      }
  printf("  clock          %7.2f GHz (s_memtime / s_memrealtime over the tiles)\n", rt > 0 ? cyc / rt * 0.1 : 0.0);
#endif
  return 0;
}
