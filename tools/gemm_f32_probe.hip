// Dev tool: f32 chain-GEMM shapes of the Cholesky inverse in isolation (TF/s on algorithmic flops).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//   -I snlp---tenary-post-train-quantization_amd/csrc tools/gemm_f32_probe.hip -o tools/_probe/gemm_f32_probe
#include "../snlp---tenary-post-train-quantization_amd/csrc/gemm.hip"

#include <cstdio>
#include <functional>

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
  const int m = 11008;
  float *U, *C, *D;
  hipMalloc(&U, (size_t)m * m * 4);
  hipMalloc(&C, (size_t)m * m * 4);
  hipMalloc(&D, (size_t)m * m * 4);
  hipMemset(U, 0, (size_t)m * m * 4);
  hipMemset(C, 0, (size_t)m * m * 4);
  hipMemset(D, 0, (size_t)m * m * 4);
  auto rep = [](const char* what, float us, double flops, double bytes) {
    printf("%-48s %9.1f us  %6.1f TF/s  %6.2f TB/s(C)\n", what, us, flops / us / 1e6, bytes / us / 1e6);
  };
  {  // plain square GEMM, K = 4096
    GemmDesc g{};
    g.M = 8192; g.N = 8192; g.K = 4096;
    g.A = U; g.lda = m; g.a_layout = LAY_KMAJOR;
    g.B = U + 8192; g.ldb = m; g.b_layout = LAY_KMAJOR;
    g.in_dtype = PT2Q_F32; g.C = C; g.ldc = m; g.mode = GEMM_STORE;
    float us = time_us([&] { pt2q_launch_gemm(g, 0); });
    rep("store 8192x8192 K=4096", us, 2.0 * 8192 * 8192 * 4096, 8192.0 * 8192 * 4);
  }
  for (int K : {128, 256, 512}) {
    for (int r : {10000, 6000, 2000}) {
      GemmDesc g{};
      g.M = r; g.N = r; g.K = K;
      g.A = U + 64; g.lda = m; g.a_layout = LAY_KMAJOR;
      g.B = U + 64; g.ldb = m; g.b_layout = LAY_KMAJOR;
      g.in_dtype = PT2Q_F32; g.C = C + (long)K * m + K; g.ldc = m;
      g.mode = GEMM_CHAIN_NEG; g.upper = 1;
      char s[96];
      snprintf(s, sizeof s, "trailing upper r=%d K=%d generic", r, K);
      float us = time_us([&] { pt2q_launch_gemm(g, 0); });
      rep(s, us, (double)r * r * K, (double)r * r * 4);
      if (K <= 128) {
        GemmDesc e{};
        snprintf(s, sizeof s, "trailing upper r=%d K=%d rank_update2", r, K);
        float us2 = time_us([&] { pt2q_launch_gemm2(g, e, 0); });
        rep(s, us2, (double)r * r * K, (double)r * r * 4);
      }
    }
  }
  for (int K : {64, 512}) {  // triangular-inverse update: Ui[0..c, c..] += Ui[:, J] U[J, c..]
    const int c = 5000, rest = 6000;
    GemmDesc g{};
    g.M = c; g.N = rest; g.K = K;
    g.A = D; g.lda = m; g.a_layout = LAY_ROWMAJOR;
    g.B = U; g.ldb = m; g.b_layout = LAY_KMAJOR;
    g.in_dtype = PT2Q_F32; g.C = D + c; g.ldc = m; g.mode = GEMM_CHAIN_POS;
    char s[96];
    snprintf(s, sizeof s, "trtri %dx%d K=%d generic", c, rest, K);
    float us = time_us([&] { pt2q_launch_gemm(g, 0); });
    rep(s, us, 2.0 * c * rest * K, 8.0 * c * rest);
    if (K <= 128) {
      GemmDesc e{};
      snprintf(s, sizeof s, "trtri %dx%d K=%d rank_update2", c, rest, K);
      float us2 = time_us([&] { pt2q_launch_gemm2(g, e, 0); });
      rep(s, us2, 2.0 * c * rest * K, 8.0 * c * rest);
    }
  }
  {  // lauum
    GemmDesc g{};
    g.M = m; g.N = m; g.K = m;
    g.A = D; g.lda = m; g.a_layout = LAY_ROWMAJOR;
    g.B = D; g.ldb = m; g.b_layout = LAY_ROWMAJOR;
    g.in_dtype = PT2Q_F32; g.C = C; g.ldc = m;
    g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1; g.kstart_diag = 2;
    float us = time_us([&] { pt2q_launch_gemm(g, 0); }, 3);
    rep("lauum 11008", us, (double)m * m * m / 3 * 2, (double)m * m * 4);
  }
  return 0;
}
