// f32 MFMA GEMM for the PT2Q hot path: C (op)= A·B with every output a k-ascending fmaf chain.
//
// Used for the Gram XᵀX (main.py:128, gptq.py:75), the Cholesky trailing update and the
// triangular-inverse / lauum products behind cholesky_inverse (main.py:138-139), and the
// error-feedback update W[:,rem] -= E @ C (main.py:214).
//
// v_mfma_f32_32x32x2_f32 accumulates as D = fma(a1,b1, fma(a0,b0,C)) (bit-exact, verified on
// gfx950 by tools/probe_numerics.hip), so issuing the k-steps in ascending order reproduces the
// oracle's sequential fmaf chains bit-for-bit.  Zero-padding K is an exact no-op (the chain
// never holds -0 when it starts from +0).
//
// Tile: BM x BN x 16, 256 threads = 4 waves in a 2x2 grid, each wave (BM/2)x(BN/2) as
// 32x32 MFMA sub-tiles; LDS double-buffered with register prefetch of the next K-tile.
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int BK = 16;

template <typename T>
PT2Q_DEV float to_f32(T v);
template <>
PT2Q_DEV float to_f32<float>(float v) { return v; }
template <>
PT2Q_DEV float to_f32<_Float16>(_Float16 v) { return (float)v; }
template <>
PT2Q_DEV float to_f32<uint16_t>(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Loads a BK x BDIM tile of a matrix into registers (as f32) and writes it to LDS as
// lds[k][d] (k-major).  KMAJOR: element (d,k) at base[k*ld + d]; ROWMAJOR: base[d*ld + k].
template <typename TIn, int BDIM>
struct TileLoader {
  static constexpr int ELEMS = BK * BDIM / 256;  // per thread
  float v[ELEMS];
  PT2Q_DEV void load(const TIn* base, long ld, int layout, int d0, int k0, int DMAX, int KMAX) {
    const int tid = threadIdx.x;
    if (layout == LAY_KMAJOR) {
      // thread -> (k, d): consecutive threads along d
#pragma unroll
      for (int e = 0; e < ELEMS; ++e) {
        int q = tid + e * 256;
        int k = q / BDIM, d = q % BDIM;
        int gk = k0 + k, gd = d0 + d;
        v[e] = (gk < KMAX && gd < DMAX) ? to_f32<TIn>(base[(long)gk * ld + gd]) : 0.0f;
      }
    } else {
      // thread -> (d, k): consecutive threads along k
#pragma unroll
      for (int e = 0; e < ELEMS; ++e) {
        int q = tid + e * 256;
        int d = q / BK, k = q % BK;
        int gk = k0 + k, gd = d0 + d;
        v[e] = (gk < KMAX && gd < DMAX) ? to_f32<TIn>(base[(long)gd * ld + gk]) : 0.0f;
      }
    }
  }
  PT2Q_DEV void store(float (*lds)[BDIM + 4], int layout) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int e = 0; e < ELEMS; ++e) {
      int q = tid + e * 256;
      if (layout == LAY_KMAJOR)
        lds[q / BDIM][q % BDIM] = v[e];
      else
        lds[q % BK][q / BK] = v[e];
    }
  }
};

template <int BM, int BN, typename TIn>
__global__ __launch_bounds__(256) void gemm_kernel(GemmDesc g, int tiles_m, int tiles_n) {
  __shared__ float As[2][BK][BM + 4];
  __shared__ float Bs[2][BK][BN + 4];
  constexpr int RM = BM / 64, RN = BN / 64;

  int ti, tj;
  {
    int bid = blockIdx.x;
    if (g.upper) {
      ti = 0;
      while (bid >= tiles_n - ti) {
        bid -= tiles_n - ti;
        ++ti;
      }
      tj = ti + bid;
    } else {
      ti = bid / tiles_n;
      tj = bid % tiles_n;
    }
  }
  const int i0 = ti * BM, j0 = tj * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int li = lane & 31, lk = lane >> 5;

  f32x16 acc[RM][RN];
#pragma unroll
  for (int rm = 0; rm < RM; ++rm)
#pragma unroll
    for (int rn = 0; rn < RN; ++rn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float c0 = 0.0f;
        if (g.mode == GEMM_CHAIN_NEG) {
          int row = i0 + wr * (BM / 2) + rm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
          int col = j0 + wc * (BN / 2) + rn * 32 + li;
          if (row < g.M && col < g.N) {
            long crow = g.crow ? g.crow[row] : row;
            c0 = g.C[crow * g.ldc + col];
          }
        }
        acc[rm][rn][r] = c0;
      }

  int kbeg = 0;
  if (g.kstart_diag == 1) kbeg = i0 - (i0 % BK);
  if (g.kstart_diag == 2) kbeg = j0 - (j0 % BK);
  const TIn* Ab = (const TIn*)g.A;
  const TIn* Bb = (const TIn*)g.B;
  const float sgn = (g.mode == GEMM_CHAIN_NEG) ? -1.0f : 1.0f;

  TileLoader<TIn, BM> la;
  TileLoader<TIn, BN> lb;
  if (kbeg < g.K) {
    la.load(Ab, g.lda, g.a_layout, i0, kbeg, g.M, g.K);
    lb.load(Bb, g.ldb, g.b_layout, j0, kbeg, g.N, g.K);
    la.store(As[0], g.a_layout);
    lb.store(Bs[0], g.b_layout);
  }
  __syncthreads();
  int cur = 0;
  for (int k0 = kbeg; k0 < g.K; k0 += BK) {
    const bool more = (k0 + BK < g.K);
    if (more) {
      la.load(Ab, g.lda, g.a_layout, i0, k0 + BK, g.M, g.K);
      lb.load(Bb, g.ldb, g.b_layout, j0, k0 + BK, g.N, g.K);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[RM], b[RN];
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) a[rm] = sgn * As[cur][kk + lk][wr * (BM / 2) + rm * 32 + li];
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) b[rn] = Bs[cur][kk + lk][wc * (BN / 2) + rn * 32 + li];
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
          acc[rm][rn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rm], b[rn], acc[rm][rn], 0, 0, 0);
    }
    if (more) {
      la.store(As[cur ^ 1], g.a_layout);
      lb.store(Bs[cur ^ 1], g.b_layout);
    }
    __syncthreads();
    cur ^= 1;
  }

  const bool mirror = g.upper && g.mirror && (ti != tj);
#pragma unroll
  for (int rm = 0; rm < RM; ++rm)
#pragma unroll
    for (int rn = 0; rn < RN; ++rn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int row = i0 + wr * (BM / 2) + rm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        int col = j0 + wc * (BN / 2) + rn * 32 + li;
        if (row >= g.M || col >= g.N) continue;
        long crow = g.crow ? g.crow[row] : row;
        float* p = g.C + crow * g.ldc + col;
        float v = acc[rm][rn][r];
        if (g.mode == GEMM_ADD) v = *p + v;
        else if (g.mode == GEMM_SUB) v = *p - v;
        *p = v;
        if (mirror) g.C[(long)col * g.ldc + row] = v;
      }
}

template <int BM, int BN, typename TIn>
int launch_t(const GemmDesc& g, hipStream_t st) {
  int tm = ceil_div(g.M, BM), tn = ceil_div(g.N, BN);
  long ntiles;
  if (g.upper) {
    if (tm != tn || BM != BN) return PT2Q_E_ARG;
    ntiles = (long)tm * (tm + 1) / 2;
  } else {
    ntiles = (long)tm * tn;
  }
  if (ntiles <= 0) return PT2Q_OK;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, TIn>), dim3((unsigned)ntiles), dim3(256), 0, st, g, tm,
                     tn);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

template <typename TIn>
int launch_dt(const GemmDesc& g, hipStream_t st) {
  // small problems: 64x64 tiles for more workgroups
  long big = (long)ceil_div(g.M, 128) * ceil_div(g.N, 128);
  if (big >= 256) return launch_t<128, 128, TIn>(g, st);
  return launch_t<64, 64, TIn>(g, st);
}

}  // namespace

int pt2q_launch_gemm(const GemmDesc& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return PT2Q_OK;
  if (g.K < 0 || !g.A || !g.B || !g.C) return PT2Q_E_ARG;
  switch (g.in_dtype) {
    case PT2Q_F32:
      return launch_dt<float>(g, st);
    case PT2Q_F16:
      return launch_dt<_Float16>(g, st);
    case PT2Q_BF16:
      return launch_dt<uint16_t>(g, st);
  }
  return PT2Q_E_ARG;
}
