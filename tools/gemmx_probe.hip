// Dev tool: gemmx (K-major f32 chain GEMM, gemmx.hip) vs the generic GEMM (gemm.hip):
// bit-exactness on random data and timing.  Build:
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//   -I snlp---tenary-post-train-quantization_amd/csrc tools/gemmx_probe.hip -o tools/_probe/gemmx_probe
#include "../snlp---tenary-post-train-quantization_amd/csrc/gemm.hip"
#include "../snlp---tenary-post-train-quantization_amd/csrc/gemmx.hip"

#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

const Pt2qTuning& pt2q_tuning() {
  static Pt2qTuning t;
  return t;
}
int pt2q_launch_gram16(const GemmDesc&, int*, hipStream_t, int*) { return PT2Q_E_UNSUPPORTED; }
size_t pt2q_gram16_flags_ints(int) { return 0; }

static float time_us(const std::function<void()>& f, int reps = 10) {
  f();
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  const long m = 11008;
  const size_t bytes = (size_t)m * m * 4;
  float *A, *C1, *C2;
  hipMalloc(&A, bytes);
  hipMalloc(&C1, bytes);
  hipMalloc(&C2, bytes);
  std::vector<float> h((size_t)m * m);
  uint64_t s = 12345;
  for (auto& x : h) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    x = (float)((int)(s >> 40) - (1 << 23)) / (float)(1 << 23);
  }
  hipMemcpy(A, h.data(), bytes, hipMemcpyHostToDevice);
  struct Case { const char* name; int M, N, K; int mode, upper, mirror, kd; long aoff, boff; };
  std::vector<Case> cases = {
      {"store rect 1000x772 K=333", 1000, 772, 333, GEMM_STORE, 0, 0, 0, 0, 4},
      {"chain_neg upper 900 K=128", 900, 900, 128, GEMM_CHAIN_NEG, 1, 0, 0, 64, 64},
      {"chain_pos rect 640x1284 K=64", 640, 1284, 64, GEMM_CHAIN_POS, 0, 0, 0, 8, 128},
      {"lauum-like 1100 kd2 mirror", 1100, 1100, 1100, GEMM_STORE, 1, 1, 2, 0, 0},
      {"chain_neg upper 10000 K=512", 10000, 10000, 512, GEMM_CHAIN_NEG, 1, 0, 0, 64, 64},
      {"chain_neg upper 6000 K=512", 6000, 6000, 512, GEMM_CHAIN_NEG, 1, 0, 0, 64, 64},
      {"chain_neg upper 2000 K=512", 2000, 2000, 512, GEMM_CHAIN_NEG, 1, 0, 0, 64, 64},
      {"chain_neg upper 10000 K=128", 10000, 10000, 128, GEMM_CHAIN_NEG, 1, 0, 0, 64, 64},
      {"chain_pos rect 5000x6000 K=512", 5000, 6000, 512, GEMM_CHAIN_POS, 0, 0, 0, 8, 128},
      {"store 8192x8192 K=4096", 8192, 8192, 4096, GEMM_STORE, 0, 0, 0, 0, 8192},
      {"lauum 11008", 11008, 11008, 11008, GEMM_STORE, 1, 1, 2, 0, 0},
  };
  for (auto& c : cases) {
    GemmDesc g{};
    g.M = c.M; g.N = c.N; g.K = c.K;
    g.A = A + c.aoff; g.lda = m; g.a_layout = LAY_KMAJOR;
    g.B = A + c.boff; g.ldb = m; g.b_layout = LAY_KMAJOR;
    g.in_dtype = PT2Q_F32; g.ldc = m; g.mode = c.mode; g.upper = c.upper; g.mirror = c.mirror;
    g.kstart_diag = c.kd;
    hipMemcpy(C1, A, bytes, hipMemcpyDeviceToDevice);
    hipMemcpy(C2, A, bytes, hipMemcpyDeviceToDevice);
    g.C = C1;
    int r1 = pt2q_launch_gemm(g, 0);
    g.C = C2;
    int r2 = pt2q_launch_gemmx(g, 0);
    hipDeviceSynchronize();
    std::vector<float> o1((size_t)c.M * m), o2((size_t)c.M * m);
    hipMemcpy(o1.data(), C1, o1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o2.data(), C2, o2.size() * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (long i = 0; i < c.M; ++i)
      for (long j = (c.upper && !c.mirror ? (i / 128) * 128 : 0); j < c.N; ++j) {
        float a = o1[i * m + j], b = o2[i * m + j];
        if (memcmp(&a, &b, 4) != 0 && !(a == 0.0f && b == 0.0f)) ++bad;
      }
    double flops = (double)c.M * c.N * c.K * 2 * (c.upper ? 0.5 : 1.0);
    if (c.kd == 2) flops = (double)c.M * c.M * c.M / 3.0;
    float t1 = time_us([&] { g.C = C1; pt2q_launch_gemm(g, 0); }, 3);
    float t2 = time_us([&] { g.C = C2; pt2q_launch_gemmx(g, 0); }, 3);
    printf("%-34s rc %d/%d mismatches %8ld | generic %9.1f us %6.1f TF | gemmx %9.1f us %6.1f TF\n", c.name, r1,
           r2, bad, t1, flops / t1 / 1e6, t2, flops / t2 / 1e6);
    fflush(stdout);
  }
  return 0;
}
