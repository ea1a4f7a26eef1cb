// Dev tool: phase timestamps of the SSR top-k launch (ssr.hip built with -DPT2Q_PROBE=4, csrc/probe.hpp).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DPT2Q_PROBE=4 -I include \
//   -I snlp---tenary-post-train-quantization_amd/csrc tools/topk_probe.hip -o tools/topk_probe.bin
#include "../snlp---tenary-post-train-quantization_amd/csrc/ssr.hip"

#include <cstdio>
#include <vector>

// the library's tuning (api.hip) at its defaults
const Pt2qTuning& pt2q_tuning() {
  static Pt2qTuning t;
  return t;
}

int main() {
  const int r = 3968, b = 128, m = 4096;
  std::vector<float> hs(r);
  std::vector<int> hr(r);
  for (int e = 0; e < r; ++e) {
    hs[e] = 0.01f + 1e-3f * (float)((e * 2654435761u) % 1000) / 1000.0f;
    hr[e] = e;
  }
  float *sim, *G, *S1, *d;
  int *rem, *blk, *nrem, *sync;
  (void)hipMalloc(&sim, r * 4);
  (void)hipMalloc(&rem, r * 4);
  (void)hipMalloc(&blk, b * 4);
  (void)hipMalloc(&nrem, r * 4);
  (void)hipMalloc(&G, (size_t)m * m * 4);
  (void)hipMalloc(&S1, b * 4);
  (void)hipMalloc(&d, 4);
  (void)hipMalloc(&sync, 8);
  (void)hipMemset(G, 0, (size_t)m * m * 4);
  (void)hipMemcpy(sim, hs.data(), r * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(rem, hr.data(), r * 4, hipMemcpyHostToDevice);
  for (int it = 0; it < 3; ++it) {
    (void)hipMemset(sync, 0, 8);
    pt2q_launch_ssr_topk(sim, rem, r, b, blk, nrem, nullptr, 0, G, m, S1, d, sync);
    (void)hipDeviceSynchronize();
  }
  long long st[64][16];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(topk_stamps), sizeof(st));
  const long long t0 = st[0][0];
  printf("wg0 phases (cycles from start):");
  for (int i = 1; i <= 7; ++i) printf(" %d:%lld", i, st[0][i] - t0);
  printf("\nhelpers 8 (flag seen), 9 (S1 done):");
  for (int w = 1; w <= 16; w += 5) printf(" [%d] %lld %lld", w, st[w][8] - t0, st[w][9] - t0);
  printf("\n");
  return 0;
}
