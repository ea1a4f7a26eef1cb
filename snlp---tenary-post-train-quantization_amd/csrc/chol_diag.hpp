// The 64 x 64 diagonal-block Cholesky factor (chol.hip's chol_diag_kernel, and fused into the
// trailing-update launch that produces the block: gemm.hip rank_update2_kernel).
#pragma once
#include "common.hpp"

namespace pt2q_chol {

constexpr int NB = 64;
constexpr int DG = 4;  // rows per barrier

// The diagonal-block factorisation with four waves: wave q keeps rows [16q, 16q+16) of every
// column in registers (lane c = column c, col[s] = D[16q+s][c]).  Rows are finalised in groups
// of four (one barrier per group instead of per row): the wave owning the group forms its rows
// one after another -- U[k][k] = sqrt(D[k][k]) via readlane, U[k][c] = D[k][c]/U[k][k] -- and,
// before the next row of the group, applies row k's update to the group's later rows itself
// (U[k][r] by readlane); it publishes the four rows in LDS (entries c <= k as 0).  After the
// barrier every wave applies D[r][c] = fmaf(-U[k][r], U[k][c], D[r][c]) for the four rows in
// order to its other rows (an fmaf with a zero factor is an exact no-op, so rows <= k and
// columns <= k are untouched).  Each element thus gets exactly the row updates of the
// one-row-at-a-time order, k ascending.  Entries below the diagonal are scratch, never written
// back.  Padding (nb < NB) is an identity block.  load(r, c) gives D[r][c] for r, c < nb;
// urow: 2 * DG * NB floats of LDS.  Writes U (r <= c < nb) to A at (p0, p0).
template <class Load>
PT2Q_DEV void diag_factor(Load load, float* A, long lda, int p0, int nb, int* info,
                          float (*urow)[DG][NB]) {
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  float col[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int r = 16 * q + s;
    const bool in = r < nb && c < nb;
    col[s] = load(in ? r : 0, in ? c : 0);  // branch-free loads
    col[s] = in ? col[s] : ((r == c) ? 1.0f : 0.0f);
  }
  for (int kq = 0; kq < 4; ++kq) {
#pragma unroll
    for (int kg = 0; kg < 16 / DG; ++kg) {
      const int ks0 = DG * kg, k0 = 16 * kq + ks0;
      float(*ur)[NB] = urow[kg & 1];
      const bool own = q == kq;
      if (own) {
#pragma unroll
        for (int t = 0; t < DG; ++t) {
          const int ks = ks0 + t, k = k0 + t;
          const float dkk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(col[ks]), k));
          if (c == 0 && k < nb && !(dkk > 0.0f)) atomicCAS(info, 0, p0 + k + 1);
          const float ukk = sqrtf(dkk);
          col[ks] = (c == k) ? ukk : ((c > k) ? col[ks] / ukk : col[ks]);
          const float ukc = (c > k) ? col[ks] : 0.0f;
          ur[t][c] = ukc;
#pragma unroll
          for (int t2 = t + 1; t2 < DG; ++t2) {  // row k's term for the group's later rows
            const float ukr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ukc), k0 + t2));
            col[ks0 + t2] = fmaf(-ukr, ukc, col[ks0 + t2]);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < DG; ++t) {
        const float ukc = ur[t][c];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const bool grp = own && s >= ks0 && s < ks0 + DG;  // done by the owner above
          const float x = fmaf(-ur[t][16 * q + s], ukc, col[s]);
          col[s] = grp ? col[s] : x;
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int r = 16 * q + s;
    if (r <= c && c < nb) A[(long)(p0 + r) * lda + p0 + c] = col[s];
  }
}

}  // namespace pt2q_chol
