// The 64 x 64 diagonal-block Cholesky factor (chol.hip's chol_diag_kernel, and fused into the
// trailing-update launch that produces the block: gemm.hip rank_update2_kernel).
#pragma once
#include "common.hpp"

namespace pt2q_chol {

constexpr int NB = 64;
constexpr int DG = 4;            // rows per barrier (a group; 4, 8 or 16)
constexpr int NG = NB / DG;      // groups
constexpr int SL = NB / 4;       // rows (slots) per wave
static_assert(SL % DG == 0, "a wave holds whole groups");

// The diagonal-block factorisation with four waves.  Rows are finalised in NG groups of DG
// (one barrier per group); group g (rows DG·g .. DG·g+DG-1) belongs to wave g % 4, which keeps
// them in registers (lane c = column c; slot s of wave q holds row rowof(q, s) =
// DG(4(s/DG) + q) + s%DG).
// The owner forms its group's rows one after another -- U[k][k] = sqrt(D[k][k]) via readlane,
// U[k][c] = D[k][c]/U[k][k] -- applying each row's term to the group's later rows itself
// (U[k][r] by readlane), and publishes the four rows in LDS (entries c <= k as 0).  After the
// barrier every wave applies D[r][c] = fmaf(-U[k][r], U[k][c], D[r][c]) for the four rows in
// order to its rows (an fmaf with a zero factor is an exact no-op, so rows <= k and columns
// <= k are untouched) -- except that the owner of the next group first updates only that group
// and defers the rest to after the next barrier, so that the chain from one group to the next
// is one barrier, DG·DG fmas and the group itself.  Each element still gets exactly the row
// updates of the one-row-at-a-time order, k ascending.  Entries below the diagonal are scratch,
// never written back.  Padding (nb < NB) is an identity block.  load(r, c) gives D[r][c] for
// r, c < nb; urow: 3 * DG * NB floats of LDS (a group's rows stay readable for two barriers).
// Writes U (r <= c < nb) to A at (p0, p0).
PT2Q_DEV int diag_rowof(int q, int s) { return DG * (4 * (s / DG) + q) + (s % DG); }

// this wave's slots s in [s_lo, s_hi) (excluding [x_lo, x_hi)) get group ur's four row updates
PT2Q_DEV void diag_apply(float (&col)[SL], const float (*ur)[NB], int q, int c, int s_lo, int s_hi,
                         int x_lo, int x_hi) {
#pragma unroll
  for (int t = 0; t < DG; ++t) {
    const float ukc = ur[t][c];
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      const bool in = s >= s_lo && s < s_hi && !(s >= x_lo && s < x_hi);
      const float x = fmaf(-ur[t][diag_rowof(q, s)], ukc, col[s]);
      col[s] = in ? x : col[s];
    }
  }
}

template <class Load>
PT2Q_DEV void diag_factor(Load load, float* A, long lda, int p0, int nb, int* info,
                          float (*urow)[DG][NB]) {
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  float col[SL];
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int r = diag_rowof(q, s);
    const bool in = r < nb && c < nb;
    col[s] = load(in ? r : 0, in ? c : 0);  // branch-free loads
    col[s] = in ? col[s] : ((r == c) ? 1.0f : 0.0f);
  }
  int pend = -1;  // a group whose updates this wave has so far applied to its next group only
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int s0 = DG * (g >> 2), k0 = DG * g;  // the owner's slots of group g, its first row
    float(*ur)[NB] = urow[g % 3];
    if (q == (g & 3)) {
#pragma unroll
      for (int t = 0; t < DG; ++t) {
        const int ks = s0 + t, k = k0 + t;
        const float dkk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(col[ks]), k));
        if (c == 0 && k < nb && !(dkk > 0.0f)) atomicCAS(info, 0, p0 + k + 1);
        const float ukk = sqrtf(dkk);
        col[ks] = (c == k) ? ukk : ((c > k) ? col[ks] / ukk : col[ks]);
        const float ukc = (c > k) ? col[ks] : 0.0f;
        ur[t][c] = ukc;
#pragma unroll
        for (int t2 = t + 1; t2 < DG; ++t2) {  // row k's term for the group's later rows
          const float ukr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ukc), k0 + t2));
          col[s0 + t2] = fmaf(-ukr, ukc, col[s0 + t2]);
        }
      }
    }
    __syncthreads();
    if (pend >= 0) {  // the deferred rest of group pend (= g - 1), before group g's updates
      diag_apply(col, urow[pend % 3], q, c, 0, SL, s0, s0 + DG);
      pend = -1;
    }
    const int gn = g + 1, sn = DG * (gn >> 2);
    if (gn < NG && q == (gn & 3)) {  // the next owner: its next group now, the rest later
      diag_apply(col, ur, q, c, sn, sn + DG, 0, 0);
      pend = g;
    } else {
      diag_apply(col, ur, q, c, 0, SL, q == (g & 3) ? s0 : 0, q == (g & 3) ? s0 + DG : 0);
    }
  }
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int r = diag_rowof(q, s);
    if (r <= c && c < nb) A[(long)(p0 + r) * lda + p0 + c] = col[s];
  }
}

}  // namespace pt2q_chol
