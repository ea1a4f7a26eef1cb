// Dev tool: time the 64 x 64 diagonal-block factor (chol_diag.hpp) alone.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//   -I snlp---tenary-post-train-quantization_amd/csrc tools/diag_probe.hip -o tools/diag_probe.bin
#include "../snlp---tenary-post-train-quantization_amd/csrc/chol_diag.hpp"

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void diag_probe_kernel(const float* D, float* A, int* info, int reps) {
  __shared__ __attribute__((aligned(16))) float urow[3][pt2q_chol::DG][pt2q_chol::NB];
  for (int i = 0; i < reps; ++i) {
    pt2q_chol::diag_factor([&](int r, int c) { return D[r * 64 + c]; }, A, 64, 0, 64, info, urow);
    __syncthreads();
  }
}

int main() {
  std::vector<float> h(64 * 64);
  for (int r = 0; r < 64; ++r)
    for (int c = 0; c < 64; ++c) h[r * 64 + c] = (r == c ? 70.0f : 0.0f) + 1.0f / (1 + r + c);
  float *D, *A;
  int* info;
  (void)hipMalloc(&D, 64 * 64 * 4);
  (void)hipMalloc(&A, 64 * 64 * 4);
  (void)hipMalloc(&info, 4);
  (void)hipMemcpy(D, h.data(), 64 * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemset(info, 0, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int reps : {1, 11}) {
    diag_probe_kernel<<<1, 256>>>(D, A, info, reps);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < 20; ++i) diag_probe_kernel<<<1, 256>>>(D, A, info, reps);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("reps %d: %.2f us per launch\n", reps, 1000.0f * ms / 20);
  }
  return 0;
}
