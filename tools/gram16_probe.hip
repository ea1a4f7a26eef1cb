// Dev tool: time the 16-bit Gram kernel (gram16.hip) on real X and on an L2-resident X (every
// k-row aliased to row 0: ld = 0), to separate the compute/LDS ceiling from the fetch path.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//   -I snlp---tenary-post-train-quantization_amd/csrc tools/gram16_probe.hip -o tools/gram16_probe.bin
// usage: tools/gram16_probe.bin [N] [m] [reps]
#include "../snlp---tenary-post-train-quantization_amd/csrc/gram16.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

// the library's tuning (api.hip), reduced to the Gram knobs this probe varies
const Pt2qTuning& pt2q_tuning() {
  static Pt2qTuning t = [] {
    Pt2qTuning u;
    auto gi = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
    u.gram_wide = gi("PT2Q_GRAM_WIDE", 1);
    u.gram_super = gi("PT2Q_GRAM_SUPER", 0);
    return u;
  }();
  return t;
}

static float time_launch(GemmDesc g, int* F, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  pt2q_launch_gram16(g, F, 0, nullptr);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) pt2q_launch_gram16(g, F, 0, nullptr);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char** argv) {
  const long N = argc > 1 ? atol(argv[1]) : 262144;
  const int m = argc > 2 ? atoi(argv[2]) : 4096;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  std::vector<_Float16> hx((size_t)N * m);
  for (size_t i = 0; i < hx.size(); ++i)
    hx[i] = (_Float16)((float)((i * 2654435761u) % 2001) / 1000.0f - 1.0f);
  void *X, *G, *F;
  (void)hipMalloc(&X, hx.size() * 2);
  (void)hipMalloc(&G, (size_t)m * m * 4);
  (void)hipMalloc(&F, pt2q_gram16_flags_ints(m) * 4);
  (void)hipMemcpy(X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  GemmDesc g{};
  g.M = m; g.N = m; g.K = (int)N;
  g.A = X; g.lda = m; g.a_layout = LAY_KMAJOR;
  g.B = X; g.ldb = m; g.b_layout = LAY_KMAJOR;
  g.in_dtype = PT2Q_F16; g.C = (float*)G; g.ldc = m; g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1;
  const double fl = (double)N * m * (m + 1);
  float ms = time_launch(g, (int*)F, reps);
  printf("real X     N=%ld m=%d: %.3f ms  %.1f TFLOP/s\n", N, m, ms, fl / ms / 1e9);
  g.lda = 0; g.ldb = 0;
  ms = time_launch(g, (int*)F, reps);
  printf("resident X N=%ld m=%d: %.3f ms  %.1f TFLOP/s\n", N, m, ms, fl / ms / 1e9);
  int info = 0;
  (void)hipMemcpy(&info, (int*)F + gx_ntile(m), 4, hipMemcpyDeviceToHost);
  printf("status word %d\n", info);
  return 0;
}
