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
#include "chol_diag.hpp"

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

// Upper-triangle tile order: 8x8-tile supertiles, row-major over the super-triangle, row-major
// (i <= j) inside a supertile.  L is a logical tile index in [0, T(T+1)/2).
PT2Q_DEV void upper_tile(int L, int T, int& ti, int& tj) {
  constexpr int S = 8;
  const int Ts = (T + S - 1) / S;
  int I = 0, J = 0;
  for (;;) {
    const int h = min(S, T - I * S), w = min(S, T - J * S);
    const int cnt = (I == J) ? h * (h + 1) / 2 : h * w;
    if (L < cnt) {
      if (I == J) {
        int rr = 0;
        while (L >= h - rr) {
          L -= h - rr;
          ++rr;
        }
        ti = I * S + rr;
        tj = I * S + rr + L;
      } else {
        ti = I * S + L / w;
        tj = J * S + L % w;
      }
      return;
    }
    L -= cnt;
    if (++J == Ts) {
      ++I;
      J = I;
    }
  }
}

// Bijective XCD-aware remap: blocks b, b+8, ... (one XCD under round-robin dispatch) get a
// contiguous range of logical ids.  Speed only; any placement is correct.
PT2Q_DEV int xcd_remap(int b, int nwg) {
  const int xcd = b % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// Accumulator tile.  SW = false: MFMA rows are C rows (lane <-> C column).  SW = true: the
// MFMA computes the transposed tile (operands swapped; fmaf(a,b,c) == fmaf(b,a,c), so the chains
// are unchanged), so lane <-> C row and each group of 4 registers <-> 4 consecutive C columns,
// which lets the epilogue move C with 16-byte accesses.
template <int BM, int BN, bool SW = false>
struct Frag {
  static constexpr int RM = BM / 64, RN = BN / 64;
  f32x16 acc[RM][RN];
  PT2Q_DEV static int row_of(int i0, int rm, int r) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = wave >> 1, li = lane & 31, lk = lane >> 5;
    return SW ? i0 + wr * (BM / 2) + rm * 32 + li
              : i0 + wr * (BM / 2) + rm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
  }
  PT2Q_DEV static int col_of(int j0, int rn, int r) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wc = wave & 1, li = lane & 31, lk = lane >> 5;
    return SW ? j0 + wc * (BN / 2) + rn * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk
              : j0 + wc * (BN / 2) + rn * 32 + li;
  }
  template <typename F>
  PT2Q_DEV void for_each(int i0, int j0, F&& f) {
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[rm][rn][r];
          f(v, row_of(i0, rm, r), col_of(j0, rn, r));
          acc[rm][rn][r] = v;
        }
  }
};

// Extend the chains of one output tile over K-range [kbeg, kend) (k ascending).
template <int BM, int BN, typename TIn, bool VEC, bool SW = false>
PT2Q_DEV void tile_mma(Frag<BM, BN, SW>& F, const GemmDesc& g, int i0, int j0, int kbeg, int kend,
                       float (*As)[BK][BM + PAD], float (*Bs)[BK][BN + PAD]) {
  constexpr int RM = BM / 64, RN = BN / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1, li = lane & 31, lk = lane >> 5;
  const TIn* Ab = (const TIn*)g.A;
  const TIn* Bb = (const TIn*)g.B;
  const float sgn = (g.mode == GEMM_CHAIN_NEG) ? -1.0f : 1.0f;
  // Two register stages (loop unrolled by 2, so no dynamic register indexing): while the MFMAs
  // of K-tile t run from LDS, the loads of tiles t+1 and t+2 are in flight.
  TileLoader<TIn, BM, VEC> la0, la1;
  TileLoader<TIn, BN, VEC> lb0, lb1;
  auto compute = [&](int buf) {
    float a[BK / 2][RM], b[BK / 2][RN];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) a[s][rm] = As[buf][2 * s + lk][wr * (BM / 2) + rm * 32 + li];
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) b[s][rn] = Bs[buf][2 * s + lk][wc * (BN / 2) + rn * 32 + li];
    }
#pragma unroll
    for (int s = 0; s < BK / 2; ++s)
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
          F.acc[rm][rn] =
              SW ? __builtin_amdgcn_mfma_f32_32x32x2f32(b[s][rn], sgn * a[s][rm], F.acc[rm][rn], 0, 0, 0)
                 : __builtin_amdgcn_mfma_f32_32x32x2f32(sgn * a[s][rm], b[s][rn], F.acc[rm][rn], 0, 0, 0);
  };
  // elements with k >= kend are zero-filled: an exact no-op for the chains
  if (kbeg < kend) {
    la0.load(Ab, g.lda, g.a_layout, i0, kbeg, g.M, kend);
    lb0.load(Bb, g.ldb, g.b_layout, j0, kbeg, g.N, kend);
    la0.store(As[0], g.a_layout);
    lb0.store(Bs[0], g.b_layout);
    if (kbeg + BK < kend) {
      la1.load(Ab, g.lda, g.a_layout, i0, kbeg + BK, g.M, kend);
      lb1.load(Bb, g.ldb, g.b_layout, j0, kbeg + BK, g.N, kend);
    }
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += 2 * BK) {
    if (k0 + 2 * BK < kend) {
      la0.load(Ab, g.lda, g.a_layout, i0, k0 + 2 * BK, g.M, kend);
      lb0.load(Bb, g.ldb, g.b_layout, j0, k0 + 2 * BK, g.N, kend);
    }
    compute(0);
    if (k0 + BK >= kend) break;
    la1.store(As[1], g.a_layout);
    lb1.store(Bs[1], g.b_layout);
    __syncthreads();
    if (k0 + 3 * BK < kend) {
      la1.load(Ab, g.lda, g.a_layout, i0, k0 + 3 * BK, g.M, kend);
      lb1.load(Bb, g.ldb, g.b_layout, j0, k0 + 3 * BK, g.N, kend);
    }
    compute(1);
    if (k0 + 2 * BK >= kend) break;
    la0.store(As[0], g.a_layout);
    lb0.store(Bs[0], g.b_layout);
    __syncthreads();
  }
  __syncthreads();  // LDS is reused by the next tile / epilogue
}

// One output tile of g: bid-th of nblocks workgroups of this GEMM (grouped launches pass
// their own offsets).
template <int BM, int BN, typename TIn, bool VEC>
PT2Q_DEV void gemm_tile(const GemmDesc& g, int tiles_m, int tiles_n, int bid, int nblocks,
                        float (*As)[BK][BM + PAD], float (*Bs)[BK][BN + PAD]) {
  int ti, tj;
  (void)tiles_m;
  if (g.upper && g.kstart_diag == 2) {
    // K starts at the tile's column (lauum): work falls with tj, so dispatch tiles column by
    // column (tj ascending = longest first) for a greedy longest-processing-time balance
    const int L = bid;
    tj = (int)((sqrtf(8.0f * (float)L + 1.0f) - 1.0f) * 0.5f);
    while ((tj + 1) * (tj + 2) / 2 <= L) ++tj;
    while (tj * (tj + 1) / 2 > L) --tj;
    ti = L - tj * (tj + 1) / 2;
  } else if (g.upper) {
    upper_tile(xcd_remap(bid, nblocks), tiles_n, ti, tj);
  } else {
    ti = bid / tiles_n;
    tj = bid % tiles_n;
  }
  const int i0 = ti * BM, j0 = tj * BN;
  Frag<BM, BN, true> F;
  // C moves in 16-byte groups of 4 consecutive columns when rows are 16-byte aligned
  const bool cvec = (g.ldc % 4 == 0) && ((uintptr_t)g.C % 16 == 0);
  constexpr int RM = BM / 64, RN = BN / 64;
  F.for_each(i0, j0, [&](float& a, int, int) { a = 0.0f; });
  if (g.mode == GEMM_CHAIN_NEG || g.mode == GEMM_CHAIN_POS) {
    // chains continue from C (no output-row gather in this mode); all loads issued before use
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = F.row_of(i0, rm, 4 * q), col = F.col_of(j0, rn, 4 * q);
          const bool rin = row < g.M;
          const float* p = g.C + (rin ? (long)row * g.ldc : 0);
          if (cvec && rin && col + 3 < g.N) {
            const f32x4 v = *(const f32x4*)(p + col);
#pragma unroll
            for (int e = 0; e < 4; ++e) F.acc[rm][rn][4 * q + e] = v[e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bool in = rin && col + e < g.N;
              const float v = p[in ? col + e : 0];
              F.acc[rm][rn][4 * q + e] = in ? v : 0.0f;
            }
          }
        }
  }
  int kbeg = 0;
  if (g.kstart_diag == 1) kbeg = i0 - (i0 % BK);
  if (g.kstart_diag == 2) kbeg = j0 - (j0 % BK);
  tile_mma<BM, BN, TIn, VEC, true>(F, g, i0, j0, kbeg, g.K, As, Bs);
  // ADD / SUB read the old C: all of its loads are issued together before the first store,
  // instead of one dependent load per 16-byte group between stores that may alias them
  const bool pre_c = cvec && (g.mode == GEMM_ADD || g.mode == GEMM_SUB);
  f32x4 cold[RM][RN][4];
  if (pre_c) {
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = F.row_of(i0, rm, 4 * q), col = F.col_of(j0, rn, 4 * q);
          const bool in = row < g.M && col + 3 < g.N;
          const long crow = in ? (g.crow ? g.crow[row] : row) : 0;
          cold[rm][rn][q] = *(const f32x4*)(g.C + crow * g.ldc + (in ? col : 0));
        }
  }
  const bool mirror = g.upper && g.mirror && (ti != tj);
#pragma unroll
  for (int rm = 0; rm < RM; ++rm)
#pragma unroll
    for (int rn = 0; rn < RN; ++rn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = F.row_of(i0, rm, 4 * q), col = F.col_of(j0, rn, 4 * q);
        if (row >= g.M) continue;
        const long crow = g.crow ? g.crow[row] : row;
        float* p = g.C + crow * g.ldc + col;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = F.acc[rm][rn][4 * q + e];
        if (cvec && col + 3 < g.N) {
          if (pre_c) {
            const f32x4 c = cold[rm][rn][q];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (g.mode == GEMM_ADD) ? c[e] + v[e] : c[e] - v[e];
          }
          *(f32x4*)p = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (col + e >= g.N) continue;
            float x = v[e];
            if (g.mode == GEMM_ADD) x = p[e] + x;
            else if (g.mode == GEMM_SUB) x = p[e] - x;
            p[e] = x;
            v[e] = x;
          }
        }
        if (mirror) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < g.N) g.C[(long)(col + e) * g.ldc + row] = v[e];
        }
      }
}

template <int BM, int BN, typename TIn, bool VEC>
__global__ __launch_bounds__(256) void gemm_kernel(GemmDesc g, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
  if (gridDim.y > 1) {  // batch item blockIdx.y (f32, no row index)
    const long o = (long)blockIdx.y * g.bstride;
    g.A = (const TIn*)g.A + o;
    g.B = (const TIn*)g.B + o;
    g.C += o;
  }
  gemm_tile<BM, BN, TIn, VEC>(g, tiles_m, tiles_n, blockIdx.x, gridDim.x, As, Bs);
}

// A batch of symmetric f32 Grams G[z] = X[z]ᵀX[z] with their own X pointers (pt2q_gram_batched on
// f32 activations): item blockIdx.y reads X[z], writes G + z * bstride.  Every element is the same
// k-ascending chain as pt2q_gram on the item alone (the tile size never changes a chain), so the
// bits are equal; the batch fills the chip where one small Gram's tiles cannot (GPT-2: 21 or 300
// tiles per Gram).
constexpr int GF_MAX = 128;
struct GramF32Ptrs {
  const float* X[GF_MAX];
};
template <int BM, int BN, bool VEC>
__global__ __launch_bounds__(256) void gram_f32_batched_kernel(GemmDesc g, GramF32Ptrs P, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
  g.A = g.B = P.X[blockIdx.y];
  g.C += (long)blockIdx.y * g.bstride;
  gemm_tile<BM, BN, float, VEC>(g, tiles_m, tiles_n, blockIdx.x, gridDim.x, As, Bs);
}

// Two independent GEMMs in one launch (workgroups [0, n0) -> g0, the rest -> g1): saves a
// kernel boundary on a serial chain (Cholesky trailing update + triangular-inverse update).
template <int BM, int BN, typename TIn, bool VEC>
__global__ __launch_bounds__(256) void gemm2_kernel(GemmDesc g0, int tm0, int tn0, int n0, GemmDesc g1,
                                                    int tm1, int tn1) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
  const int b = blockIdx.x;
  if (b < n0)
    gemm_tile<BM, BN, TIn, VEC>(g0, tm0, tn0, b, n0, As, Bs);
  else
    gemm_tile<BM, BN, TIn, VEC>(g1, tm1, tn1, b - n0, (int)gridDim.x - n0, As, Bs);
}

// Persistent, balanced ("stream-K with exact chain continuation") symmetric Gram, STORE mode:
// the K range is cut into nseg segments and unit u = seg * T + tile.  Workgroups take units in
// increasing u from a global counter.  A unit with seg > 0 waits for the tile's previous segment
// (flag), continues the chains from the partial tile stored in C (plain fp32, so the fmaf chain
// is exactly the unsplit one), and stores the partial back; the last segment writes the final
// tile and its mirror.  A unit only waits on a smaller unit, which was taken earlier by a
// workgroup that is already running, so progress never depends on how many workgroups are
// resident.  Units taken together share a K range, so the X panels they read are shared in L2.
template <typename TIn, bool VEC>
__global__ __launch_bounds__(256) void gram_streamk_kernel(GemmDesc g, int T, int nseg, int seglen,
                                                           int* flags, int* counter, int* status,
                                                           long cap) {
  constexpr int BM = 128, BN = 128;
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
  __shared__ long s_unit;
  const int ntile = T * (T + 1) / 2;
  const long units = (long)ntile * nseg;
  for (;;) {
    if (threadIdx.x == 0) s_unit = atomicAdd(counter, 1);
    __syncthreads();
    const long u = s_unit;
    __syncthreads();
    if (u >= units) break;
    const int seg = (int)(u / ntile), tl = (int)(u % ntile);
    int ti, tj;
    upper_tile(tl, T, ti, tj);
    const int i0 = ti * BM, j0 = tj * BN;
    Frag<BM, BN> F;
    if (seg == 0 && g.mode != GEMM_CHAIN_POS) {
      F.for_each(i0, j0, [&](float& a, int, int) { a = 0.0f; });
    } else if (seg == 0) {
      // continue mode: segment 0 extends the chains already held in C
      F.for_each(i0, j0, [&](float& a, int row, int col) {
        bool in = row < g.M && col < g.N;
        a = g.C[in ? (long)row * g.ldc + col : 0];
      });
      F.for_each(i0, j0, [&](float& a, int row, int col) {
        if (!(row < g.M && col < g.N)) a = 0.0f;
      });
    } else {
      if (threadIdx.x == 0) {
        wait_flag_ge<2>(&flags[tl], seg, cap, status, STALL_GRAM);  // gives up loudly
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      F.for_each(i0, j0, [&](float& a, int row, int col) {
        bool in = row < g.M && col < g.N;
        a = g.C[in ? (long)row * g.ldc + col : 0];
      });
    }
    const int kbeg = seg * seglen, kend = min(g.K, kbeg + seglen);
    tile_mma<BM, BN, TIn, VEC>(F, g, i0, j0, kbeg, kend, As, Bs);
    const bool last = (seg == nseg - 1);
    const bool mirror = last && (ti != tj);
    F.for_each(i0, j0, [&](float& a, int row, int col) {
      if (row >= g.M || col >= g.N) return;
      g.C[(long)row * g.ldc + col] = a;
      if (mirror) g.C[(long)col * g.ldc + row] = a;
    });
    if (!last) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&flags[tl], seg + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int BM, int BN, typename TIn>
bool vec_ok(const GemmDesc& g) {
  const int vw = 16 / (int)sizeof(TIn);
  auto ok_vec = [&](const void* p, long ld, int layout, int dim) {
    int vdim = (layout == LAY_KMAJOR) ? dim : g.K;
    return ((uintptr_t)p % 16 == 0) && (ld % vw == 0) && (vdim % vw == 0);
  };
  return ok_vec(g.A, g.lda, g.a_layout, g.M) && ok_vec(g.B, g.ldb, g.b_layout, g.N) &&
         (g.batch <= 1 || g.bstride % vw == 0);  // every batch item aligned like item 0
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
  const unsigned nb = g.batch > 1 ? (unsigned)g.batch : 1u;  // grid.y = batch item
  if (vec_ok<BM, BN, TIn>(g))
    hipLaunchKernelGGL((gemm_kernel<BM, BN, TIn, true>), dim3((unsigned)ntiles, nb), dim3(256), 0, st, g,
                       tm, tn);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, TIn, false>), dim3((unsigned)ntiles, nb), dim3(256), 0, st,
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
    return (g.upper ? tm * (tm + 1) / 2 : tm * tn) * (g.batch > 1 ? g.batch : 1);
  };
  const double slots = 256.0;
  long c128 = count(128), c64 = count(64);
  const int force = pt2q_tuning().gemm_tile;
  if (force == 1) return launch_t<128, 128, TIn>(g, st);
  if (force == 6) return launch_t<64, 64, TIn>(g, st);
  // efficiency = useful tiles / (rounds * slots); 64x64 tiles cost 1/4 of a 128x128 tile
  double r128 = std::ceil(c128 / slots), r64 = std::ceil(c64 / slots);
  double t128 = r128 * 4.0, t64 = r64 * 1.0 * 1.15;  // 64x64: ~15% lower per-tile efficiency
  if (c128 >= 64 && t128 <= t64) return launch_t<128, 128, TIn>(g, st);
  return launch_t<64, 64, TIn>(g, st);
}

template <typename TIn>
int launch_streamk(const GemmDesc& g, int* flags, int nflags, hipStream_t st, int* status) {
  const Pt2qTuning& tu = pt2q_tuning();
  const int T = ceil_div(g.M, 128);
  const int ntile = T * (T + 1) / 2;
  if (ntile > nflags) return PT2Q_E_WORKSPACE;
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  auto kern = vec_ok<128, 128, TIn>(g) ? gram_streamk_kernel<TIn, true> : gram_streamk_kernel<TIn, false>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int P = cus * per_cu;  // one resident wave of workgroups (correctness does not need it)
  // segment length (>= 2048 rows, multiple of 2*BK): minimise the makespan estimate
  // rounds(units / P) * (seglen + per-unit overhead of ~256 rows: partial reload/store, wait)
  int nseg = 1, seglen = ceil_div(g.K, 2 * BK) * 2 * BK;
  double best = 1e300;
  for (int s = 1; s <= 256; ++s) {
    int len = ceil_div(ceil_div(g.K, s), 2 * BK) * 2 * BK;
    if (s > 1 && len < 2048) break;
    const int ns = ceil_div(g.K, len);
    const double cost = std::ceil((double)ntile * ns / P) * (len + 256.0);
    if (cost < best * 0.999) {
      best = cost;
      nseg = ns;
      seglen = len;
    }
  }
  // flags: ntile tile flags, status, unit counter
  if (tu.gram_seglen >= 64) {
    seglen = tu.gram_seglen / (2 * BK) * (2 * BK);
    nseg = ceil_div(g.K, seglen);
  }
  if (hipMemsetAsync(flags, 0, sizeof(int) * (ntile + 2), st) != hipSuccess) return PT2Q_E_HIP;
  if (!status) status = flags + ntile;
  int* counter = flags + ntile + 1;
  hipLaunchKernelGGL(kern, dim3(P), dim3(256), 0, st, g, T, nseg, seglen, flags, counter, status,
                     tu.spin_cap_long);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

// ---------------------------------------------------------------- rank-<=64 chain updates
// C[i][j] = chain continued over k < K <= 64 of sgn * A(i,k) * B(k,j), k ascending (the
// Cholesky trailing update, GEMM_CHAIN_NEG, and the triangular-inverse update, GEMM_CHAIN_POS).
// Such a GEMM is a pass over C: one 64 x 64 tile per workgroup with every load in flight at once
// -- both K x 64 operand panels straight into LDS and the C tile into registers -- then K/2
// f32 MFMAs per wave and one store.  Bit-identical to the generic kernel (same chain order).
constexpr int RU_T = 64, RU_K = 128;

// Operand panel (64 columns d, the first KQ >= K rows k) into lds[k][d] (zero outside the matrix
// / past K); KQ = 64 or 128.
template <int KQ>
PT2Q_DEV void ru_panel(const float* base, long ld, int layout, int d0, int DMAX, int K,
                       float (*lds)[RU_T + 4], bool neg = false) {
  constexpr int NV = KQ * RU_T / 4 / 256;  // float4 per thread
  constexpr int KV = KQ / 4;               // float4 per d row (ROWMAJOR)
  const int tid = threadIdx.x;
  float4 v[NV];
  bool ok[NV];
#pragma unroll
  for (int e = 0; e < NV; ++e) {
    const int q = tid + 256 * e;
    int d, k;
    if (layout == LAY_KMAJOR) {
      k = q >> 4;
      d = (q & 15) * 4;
    } else {
      d = q / KV;
      k = (q % KV) * 4;
    }
    const long off = layout == LAY_KMAJOR ? (long)k * ld + d0 + d : (long)(d0 + d) * ld + k;
    // vectors are whole inside or outside (checked at launch: DMAX % 4 == 0 / K % 4 == 0)
    ok[e] = k < K && d0 + d < DMAX;
    v[e] = *(const float4*)(base + (ok[e] ? off : 0));
  }
#pragma unroll
  for (int e = 0; e < NV; ++e) {
    const int q = tid + 256 * e;
    float4 x = ok[e] ? v[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (neg) x = make_float4(-x.x, -x.y, -x.z, -x.w);  // exact: (-a)·b is the chain's term
    if (layout == LAY_KMAJOR) {
      *(float4*)&lds[q >> 4][(q & 15) * 4] = x;
    } else {
      const int d = q / KV, k = (q % KV) * 4;
      lds[k][d] = x.x;
      lds[k + 1][d] = x.y;
      lds[k + 2][d] = x.z;
      lds[k + 3][d] = x.w;
    }
  }
}

template <int OFF>
PT2Q_DEV float ru_ld(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// k-pair S of the chain: operands in set S % 4, the pair two ahead is read into set (S+2) % 4,
// which no MFMA still waiting to issue reads.  LDS reads are asm (hipcc would wait for each one
// right before its MFMA); the order reads -> MFMA -> wait is pinned.
template <int S, int NS>
PT2Q_DEV void ru_chain(f32x16& acc, uint32_t bA, uint32_t bB, float (&a)[4], float (&b)[4]) {
  constexpr int ROW = 2 * (RU_T + 4) * 4;  // bytes per k-pair
  if constexpr (S == 0) {
    a[0] = ru_ld<0>(bA);
    b[0] = ru_ld<0>(bB);
    a[1] = ru_ld<ROW>(bA);
    b[1] = ru_ld<ROW>(bB);
    asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a[0]), "+v"(b[0]));
  }
  if constexpr (S < NS) {
    constexpr int c = S % 4, n2 = (S + 2) % 4;
    if constexpr (S + 2 < NS) {
      a[n2] = ru_ld<(S + 2) * ROW>(bA);
      b[n2] = ru_ld<(S + 2) * ROW>(bB);
    }
    if constexpr (S > 0) {  // pair S-1's operands stay allocated until these reads are out
      constexpr int p = (S + 3) % 4;
      asm volatile("" ::"v"(a[p]), "v"(b[p]));
    }
    __builtin_amdgcn_sched_barrier(0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(b[c], a[c], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (S + 1 < NS) {  // pair S+1 landed (pair S+2 may stay in flight)
      constexpr int c1 = (S + 1) % 4;
      if constexpr (S + 2 < NS)
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a[c1]), "+v"(b[c1]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[c1]), "+v"(b[c1]));
    }
    ru_chain<S + 1, NS>(acc, bA, bB, a, b);
  }
}

// diag.A != nullptr: tile 0 of this GEMM is the next diagonal block; the workgroup that updates
// it factors it right away from its registers (chol_diag.hpp) instead of storing it.
struct RuDiag {
  float* A;
  long lda;
  int p0, nb;
  int* info;
};

PT2Q_DEV void ru_tile(const GemmDesc& g, int tn, int bid, float (*As)[RU_T + 4], float (*Bs)[RU_T + 4],
                      const RuDiag& diag = RuDiag{nullptr, 0, 0, 0, nullptr}) {
  const long zo = (long)blockIdx.y * g.bstride;  // batch item (grid.y)
  const float* const Az = (const float*)g.A + zo;
  const float* const Bz = (const float*)g.B + zo;
  float* const Cz = g.C + zo;
  int ti, tj;
  if (g.upper) {
    upper_tile(bid, tn, ti, tj);
  } else {
    ti = bid / tn;
    tj = bid % tn;
  }
  const int i0 = ti * RU_T, j0 = tj * RU_T;
  Frag<RU_T, RU_T, true> F;
  // C tile (16-byte groups of 4 columns: launch checks ldc % 4 == 0, N % 4 == 0, alignment)
  const float* Cr = Cz;
  {
    const int row = F.row_of(i0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = F.col_of(j0, 0, 4 * q);
      const bool in = row < g.M && col < g.N;
      const f32x4 v = *(const f32x4*)(Cr + (in ? (long)row * g.ldc + col : 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) F.acc[0][0][4 * q + e] = in ? v[e] : 0.0f;
    }
  }
  const bool k128 = g.K > 64, neg = g.mode == GEMM_CHAIN_NEG;
  if (k128) {
    ru_panel<128>(Az, g.lda, g.a_layout, i0, g.M, g.K, As, neg);
    ru_panel<128>(Bz, g.ldb, g.b_layout, j0, g.N, g.K, Bs);
  } else {
    ru_panel<64>(Az, g.lda, g.a_layout, i0, g.M, g.K, As, neg);
    ru_panel<64>(Bz, g.ldb, g.b_layout, j0, g.N, g.K, Bs);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1, li = lane & 31, lk = lane >> 5;
  const uint32_t bA = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)&As[lk][wr * 32 + li];
  const uint32_t bB = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)&Bs[lk][wc * 32 + li];
  // 32 or 64 k-pairs (the panels are zero past K: a zero term is an exact no-op on a chain)
  float a[4], b[4];
  if (k128)
    ru_chain<0, RU_K / 2>(F.acc[0][0], bA, bB, a, b);
  else
    ru_chain<0, 32>(F.acc[0][0], bA, bB, a, b);
  const int row = F.row_of(i0, 0, 0);
  if (diag.A && bid == 0) {  // the updated diagonal block, through LDS, into the factor
    __syncthreads();         // every wave is done with the panels: As becomes the D tile
    float (*D)[RU_T + 1] = (float (*)[RU_T + 1])&As[0][0];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = F.col_of(j0, 0, 4 * q) - j0;
#pragma unroll
      for (int e = 0; e < 4; ++e) D[row - i0][col + e] = F.acc[0][0][4 * q + e];
    }
    __syncthreads();
    pt2q_chol::diag_factor([&](int r, int c) { return D[r][c]; }, diag.A + zo, diag.lda, diag.p0, diag.nb,
                           diag.info + blockIdx.y, (float (*)[pt2q_chol::DG][pt2q_chol::NB])&Bs[0][0]);
    return;
  }
  if (row < g.M) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = F.col_of(j0, 0, 4 * q);
      if (col >= g.N) continue;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = F.acc[0][0][4 * q + e];
      *(f32x4*)(Cz + (long)row * g.ldc + col) = v;
    }
  }
}

// KQ: operand rows the LDS panels hold (64: every K <= 64 -- the Cholesky's rank-64 strip updates --
// at 34 KiB per workgroup, four per CU instead of two; 128 otherwise)
template <int KQ>
__global__ __launch_bounds__(256) void rank_update2_kernel(GemmDesc g0, int tn0, int n0, GemmDesc g1, int tn1,
                                                           RuDiag diag) {
  __shared__ __attribute__((aligned(16))) float As[KQ][RU_T + 4];
  __shared__ __attribute__((aligned(16))) float Bs[KQ][RU_T + 4];
  static_assert(KQ * (RU_T + 4) >= RU_T * (RU_T + 1), "the fused diagonal factor's D tile lives in As");
  const int b = blockIdx.x;
  if (b < n0)
    ru_tile(g0, tn0, b, As, Bs, diag);
  else
    ru_tile(g1, tn1, b - n0, As, Bs);
}

bool ru_ok(const GemmDesc& g) {
  if (g.M <= 0 || g.N <= 0) return true;
  auto al = [](const void* p) { return (uintptr_t)p % 16 == 0; };
  auto vdim = [&](int layout, int dim) { return layout == LAY_KMAJOR ? dim : g.K; };
  return g.in_dtype == PT2Q_F32 && g.K <= RU_K && !g.crow && !g.mirror &&
         (g.mode == GEMM_CHAIN_NEG || g.mode == GEMM_CHAIN_POS) && al(g.A) && al(g.B) && al(g.C) &&
         g.lda % 4 == 0 && g.ldb % 4 == 0 && g.ldc % 4 == 0 && g.N % 4 == 0 &&
         vdim(g.a_layout, g.M) % 4 == 0 && vdim(g.b_layout, g.N) % 4 == 0;
}

template <int BM, int BN>
long tiles_of(const GemmDesc& g, int& tm, int& tn) {
  tm = ceil_div(g.M, BM);
  tn = ceil_div(g.N, BN);
  if (g.M <= 0 || g.N <= 0) return 0;
  return g.upper ? (long)tm * (tm + 1) / 2 : (long)tm * tn;
}

template <int BM, int BN>
int launch2_t(const GemmDesc& g0, const GemmDesc& g1, hipStream_t st) {
  int tm0, tn0, tm1, tn1;
  const long n0 = tiles_of<BM, BN>(g0, tm0, tn0), n1 = tiles_of<BM, BN>(g1, tm1, tn1);
  if ((g0.upper && tm0 != tn0) || (g1.upper && tm1 != tn1)) return PT2Q_E_ARG;
  if (n0 + n1 <= 0) return PT2Q_OK;
  const bool vec = (n0 == 0 || vec_ok<BM, BN, float>(g0)) && (n1 == 0 || vec_ok<BM, BN, float>(g1));
  void (*k)(GemmDesc, int, int, int, GemmDesc, int, int) =
      vec ? gemm2_kernel<BM, BN, float, true> : gemm2_kernel<BM, BN, float, false>;
  hipLaunchKernelGGL(k, dim3((unsigned)(n0 + n1)), dim3(256), 0, st, g0, tm0, tn0, (int)n0, g1, tm1, tn1);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

}  // namespace

int pt2q_launch_gemm2(const GemmDesc& g0, const GemmDesc& g1, hipStream_t st, float* dA, long dld,
                      int dp0, int dnb, int* info, bool* fused) {
  if (fused) *fused = false;
  if (g0.in_dtype != PT2Q_F32 || g1.in_dtype != PT2Q_F32) return PT2Q_E_ARG;
  const int nb = g0.batch > 1 ? g0.batch : 1;
  if (nb != (g1.batch > 1 ? g1.batch : 1) || (nb > 1 && g0.bstride != g1.bstride)) return PT2Q_E_ARG;
  if (ru_ok(g0) && ru_ok(g1) && pt2q_tuning().rank_update) {
    int tm0, tn0, tm1, tn1;
    const long n0 = tiles_of<RU_T, RU_T>(g0, tm0, tn0), n1 = tiles_of<RU_T, RU_T>(g1, tm1, tn1);
    if (n0 + n1 <= 0) return PT2Q_OK;
    // the fused factor needs g0's tile 0 to be exactly the next diagonal block at (dp0, dp0)
    const bool fuse = dA && n0 > 0 && g0.C == dA + (long)dp0 * dld + dp0 && g0.ldc == dld &&
                      dnb > 0 && dnb <= RU_T && g0.M >= dnb && g0.N >= dnb;
    RuDiag d{fuse ? dA : nullptr, dld, dp0, dnb, info};
    const bool k64 = (n0 == 0 || g0.K <= 64) && (n1 == 0 || g1.K <= 64);
    hipLaunchKernelGGL(k64 ? rank_update2_kernel<64> : rank_update2_kernel<RU_K>, dim3((unsigned)(n0 + n1), (unsigned)nb),
                       dim3(256), 0, st, g0, tn0, (int)n0, g1, tn1, d);
    PT2Q_LAUNCH_CHECK();
    if (fused) *fused = fuse;
    return PT2Q_OK;
  }
  if (nb > 1) {  // the generic kernels run one item per launch
    for (int z = 0; z < nb; ++z) {
      GemmDesc h0 = g0, h1 = g1;
      const long o = (long)z * g0.bstride;
      h0.A = (const float*)g0.A + o; h0.B = (const float*)g0.B + o; h0.C = g0.C + o; h0.batch = 1;
      h1.A = (const float*)g1.A + o; h1.B = (const float*)g1.B + o; h1.C = g1.C + o; h1.batch = 1;
      const int rc = pt2q_launch_gemm2(h0, h1, st);
      if (rc != PT2Q_OK) return rc;
    }
    return PT2Q_OK;
  }
  int a, b;
  const long c128 = tiles_of<128, 128>(g0, a, b) + tiles_of<128, 128>(g1, a, b);
  const long c64 = tiles_of<64, 64>(g0, a, b) + tiles_of<64, 64>(g1, a, b);
  // the launch_dt balance rule on the combined grid
  const double t128 = std::ceil(c128 / 256.0) * 4.0, t64 = std::ceil(c64 / 256.0) * 1.15;
  if (c128 >= 64 && t128 <= t64) return launch2_t<128, 128>(g0, g1, st);
  return launch2_t<64, 64>(g0, g1, st);
}

int pt2q_launch_gemm(const GemmDesc& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return PT2Q_OK;
  if (g.K < 0 || !g.A || !g.B || !g.C) return PT2Q_E_ARG;
  if (g.batch > 1) {  // every item in one launch (grid.y); f32 chains without a row index
    if (g.in_dtype != PT2Q_F32 || g.crow) return PT2Q_E_ARG;
    return launch_dt<float>(g, st);
  }
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

int pt2q_launch_gram_f32_batched(const float* const* X, long N, int m, long ldx, float* G, long gstride, int batch,
                                 hipStream_t st) {
  if (batch <= 0 || batch > GF_MAX || m <= 0 || N < 0 || N > INT_MAX || ldx < m || !G) return PT2Q_E_ARG;
  // the LDS-DMA kernel where the operands allow it (aligned rows)
  if (pt2q_tuning().gemmx_gram) {
    const int rc = pt2q_launch_gemmx_gram(X, N, m, ldx, G, gstride, batch, st);
    if (rc != PT2Q_E_UNSUPPORTED) return rc;
  }
  GemmDesc g{};
  g.M = m; g.N = m; g.K = (int)N;
  g.lda = ldx; g.a_layout = LAY_KMAJOR;
  g.ldb = ldx; g.b_layout = LAY_KMAJOR;
  g.in_dtype = PT2Q_F32;
  g.C = G; g.ldc = m;
  g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1;
  g.batch = batch; g.bstride = gstride;
  GramF32Ptrs P{};
  bool vec = true;
  for (int z = 0; z < batch; ++z) {
    if (!X[z] && N > 0) return PT2Q_E_ARG;
    P.X[z] = X[z];
    g.A = g.B = X[z];
    vec = vec && vec_ok<128, 128, float>(g);  // every item vector-aligned, or none uses it
  }
  // the launch_dt balance rule on the whole batch
  const long t1 = ceil_div(m, 128), t6 = ceil_div(m, 64);
  const long c128 = t1 * (t1 + 1) / 2 * batch, c64 = t6 * (t6 + 1) / 2 * batch;
  const double r128 = std::ceil(c128 / 256.0) * 4.0, r64 = std::ceil(c64 / 256.0) * 1.15;
  const bool big = c128 >= 64 && r128 <= r64;
  const int tm = (int)(big ? t1 : t6);
  const dim3 grid((unsigned)(tm * (tm + 1) / 2), (unsigned)batch);
  auto kern = big ? (vec ? gram_f32_batched_kernel<128, 128, true> : gram_f32_batched_kernel<128, 128, false>)
                  : (vec ? gram_f32_batched_kernel<64, 64, true> : gram_f32_batched_kernel<64, 64, false>);
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, g, P, tm, tm);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

size_t pt2q_gram_flags_ints(int m) {
  long T = ceil_div(m, 128);
  // tile flags, status, unit counter, zero chunk; or the 16-bit kernel's
  return std::max((size_t)(T * (T + 1) / 2 + 2 + 8), pt2q_gram16_flags_ints(m));
}

// Symmetric Gram C = XᵀX (STORE): balanced persistent kernel when it pays (big K, enough
// tiles), else the one-tile-per-workgroup GEMM.  flags: pt2q_gram_flags_ints(m) ints or NULL.
int pt2q_launch_gram(const GemmDesc& g, int* flags, hipStream_t st, int* status) {
  if (g.in_dtype == PT2Q_F16 || g.in_dtype == PT2Q_BF16) return pt2q_launch_gram16(g, flags, st, status);
  const int T = ceil_div(g.M, 128);
  const long ntile = (long)T * (T + 1) / 2;
  const bool allow = pt2q_tuning().gram_split;
  if (flags && allow && (g.mode == GEMM_STORE || g.mode == GEMM_CHAIN_POS) && g.upper && g.mirror && g.M == g.N &&
      ntile >= 128 && g.K >= 16384) {
    if (g.in_dtype == PT2Q_F32) return launch_streamk<float>(g, flags, (int)ntile, st, status);
  }
  return pt2q_launch_gemm(g, st);
}
