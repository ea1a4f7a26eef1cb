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
// Tile: BM x BN x 32, 256 threads = 4 waves in a 2x2 grid, each wave (BM/2)x(BN/2) as 32x32
// MFMA sub-tiles.  Operands stream global -> registers (16-byte vector loads, fp16/bf16
// converted to fp32 on the way) -> LDS [k][d] (double-buffered); the next K-tile's loads are
// issued before the current tile's MFMAs so their latency hides under the MFMA work.
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BK = 32;
constexpr int PAD = 4;

template <typename T>
PT2Q_DEV float to_f32(T v);
template <>
PT2Q_DEV float to_f32<float>(float v) { return v; }
template <>
PT2Q_DEV float to_f32<_Float16>(_Float16 v) { return (float)v; }
template <>
PT2Q_DEV float to_f32<uint16_t>(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Raw 16-byte vector of TIn kept in registers between the load and the LDS store, so the
// load's latency overlaps the MFMA work of the current K-tile (no wait at the load site).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename TIn>
PT2Q_DEV void unpack16(u32x4 raw, float* out) {
  if constexpr (sizeof(TIn) == 4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = __uint_as_float(raw[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      uint16_t u = (uint16_t)(raw[e >> 1] >> (16 * (e & 1)));
      TIn t;
      __builtin_memcpy(&t, &u, 2);
      out[e] = to_f32<TIn>(t);
    }
  }
}

// Loads a BK x BDIM tile (element (d, k)) into registers, then stores it to lds[k][d].
//   KMAJOR: element (d,k) at base[k*ld + d]   (vectors run along d)
//   ROWMAJOR: element (d,k) at base[d*ld + k] (vectors run along k)
// VEC requires 16-byte aligned rows and the vector dimension to be a multiple of the vector
// width (checked at launch), so a vector is either wholly inside or wholly outside the matrix;
// outside vectors load from the (valid) base address and are zeroed at store time.
template <typename TIn, int BDIM, bool VEC>
struct TileLoader {
  static constexpr int VW = VEC ? 16 / (int)sizeof(TIn) : 1;
  static constexpr int NV = BK * BDIM / VW / 256;  // vectors per thread
  static_assert(NV >= 1, "tile too small");
  u32x4 raw[VEC ? NV : 1];
  bool ok[NV];
  float v[VEC ? 1 : NV];

  PT2Q_DEV void coords(int q, int layout, int& d, int& k) const {
    if (layout == LAY_KMAJOR) {
      k = q / (BDIM / VW);
      d = (q % (BDIM / VW)) * VW;
    } else {
      d = q / (BK / VW);
      k = (q % (BK / VW)) * VW;
    }
  }

  PT2Q_DEV void load(const TIn* base, long ld, int layout, int d0, int k0, int DMAX, int KMAX) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      int d, k;
      coords(tid + e * 256, layout, d, k);
      const int gd = d0 + d, gk = k0 + k;
      ok[e] = gk < KMAX && gd < DMAX;
      const long off = (layout == LAY_KMAJOR) ? (long)gk * ld + gd : (long)gd * ld + gk;
      const TIn* p = base + (ok[e] ? off : 0);
      if constexpr (VEC) {
        raw[e] = *(const u32x4*)p;
      } else {
        float x = to_f32<TIn>(*p);
        v[e] = ok[e] ? x : 0.0f;
      }
    }
  }

  PT2Q_DEV void store(float (*lds)[BDIM + PAD], int layout) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      int d, k;
      coords(tid + e * 256, layout, d, k);
      if constexpr (VEC) {
        float f[VW];
        unpack16<TIn>(raw[e], f);
#pragma unroll
        for (int w = 0; w < VW; ++w) f[w] = ok[e] ? f[w] : 0.0f;
        if (layout == LAY_KMAJOR) {
#pragma unroll
          for (int w = 0; w < VW; w += 4) {
            f32x4 x = {f[w], f[w + 1], f[w + 2], f[w + 3]};
            *(f32x4*)&lds[k][d + w] = x;
          }
        } else {
#pragma unroll
          for (int w = 0; w < VW; ++w) lds[k + w][d] = f[w];
        }
      } else {
        lds[k][d] = v[e];
      }
    }
  }
};

template <int BM, int BN, typename TIn, bool VEC>
__global__ __launch_bounds__(256) void gemm_kernel(GemmDesc g, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
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
      for (int r = 0; r < 16; ++r) acc[rm][rn][r] = 0.0f;
  if (g.mode == GEMM_CHAIN_NEG || g.mode == GEMM_CHAIN_POS) {
    // chains continue from C (no output-row gather in this mode); all loads issued before use
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int row = i0 + wr * (BM / 2) + rm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
          int col = j0 + wc * (BN / 2) + rn * 32 + li;
          bool in = row < g.M && col < g.N;
          acc[rm][rn][r] = g.C[in ? (long)row * g.ldc + col : 0];
        }
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int row = i0 + wr * (BM / 2) + rm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
          int col = j0 + wc * (BN / 2) + rn * 32 + li;
          if (!(row < g.M && col < g.N)) acc[rm][rn][r] = 0.0f;
        }
  }

  int kbeg = 0;
  if (g.kstart_diag == 1) kbeg = i0 - (i0 % BK);
  if (g.kstart_diag == 2) kbeg = j0 - (j0 % BK);
  const TIn* Ab = (const TIn*)g.A;
  const TIn* Bb = (const TIn*)g.B;
  const float sgn = (g.mode == GEMM_CHAIN_NEG) ? -1.0f : 1.0f;

  TileLoader<TIn, BM, VEC> la;
  TileLoader<TIn, BN, VEC> lb;
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
  const int vw = 16 / (int)sizeof(TIn);
  auto ok_vec = [&](const void* p, long ld, int layout, int dim) {
    int vdim = (layout == LAY_KMAJOR) ? dim : g.K;
    return ((uintptr_t)p % 16 == 0) && (ld % vw == 0) && (vdim % vw == 0);
  };
  const bool vec = ok_vec(g.A, g.lda, g.a_layout, g.M) && ok_vec(g.B, g.ldb, g.b_layout, g.N);
  if (vec)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, TIn, true>), dim3((unsigned)ntiles), dim3(256), 0, st, g,
                       tm, tn);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, TIn, false>), dim3((unsigned)ntiles), dim3(256), 0, st,
                       g, tm, tn);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

// Pick the tile so that the grid balances over the 256 CUs: every workgroup carries the same
// work, so the makespan is ceil(tiles / slots); prefer 128x128 (higher operand reuse) unless
// 64x64 packs the chip clearly better.
template <typename TIn>
int launch_dt(const GemmDesc& g, hipStream_t st) {
  auto count = [&](int t) -> long {
    long tm = ceil_div(g.M, t), tn = ceil_div(g.N, t);
    return g.upper ? tm * (tm + 1) / 2 : tm * tn;
  };
  const double slots = 256.0;
  long c128 = count(128), c64 = count(64);
  static const char* force = std::getenv("PT2Q_GEMM_TILE");
  if (force && force[0] == '1') return launch_t<128, 128, TIn>(g, st);
  if (force && force[0] == '6') return launch_t<64, 64, TIn>(g, st);
  // efficiency = useful tiles / (rounds * slots); 64x64 tiles cost 1/4 of a 128x128 tile
  double r128 = std::ceil(c128 / slots), r64 = std::ceil(c64 / slots);
  double t128 = r128 * 4.0, t64 = r64 * 1.0 * 1.15;  // 64x64: ~15% lower per-tile efficiency
  if (c128 >= 64 && t128 <= t64) return launch_t<128, 128, TIn>(g, st);
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
