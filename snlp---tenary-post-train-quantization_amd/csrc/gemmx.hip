// f32 chain GEMM with K-major operands on the f32 MFMA, LDS-DMA staged (the large GEMMs of the
// Cholesky inverse: bulk trailing updates, triangular-inverse updates, lauum; main.py:136-139).
//
//   C(i, j) (op)= chain over k in [kbeg, kend) ascending of A(i, k) * B(k, j)
//   A(i, k) = A[k * lda + i], B(k, j) = B[k * ldb + j]  (both K-major: rows of the factor)
//
// Every output is the k-ascending fmaf chain of the PT2Q contract (v_mfma_f32_32x32x2_f32 is
// fma(a1,b1, fma(a0,b0,C))), so results are bit-identical to the generic GEMM (gemm.hip) and to
// the oracle.  GEMM_CHAIN_NEG runs the positive chain on -C: fmaf(-a,b,c) == -fmaf(a,b,-c) under
// round-to-nearest-even, so no operand is negated in the loop.
//
// Tile 128 x 128 per workgroup (4 waves 2 x 2, each 64 x 64 = 2 x 2 MFMA tiles of 32 x 32).
// Operand panels go global -> LDS by LDS-DMA (16 B per lane, no register staging) into a ring of
// XNS stages of 32 k-rows; the 16-byte chunks of a row are XOR-swizzled by (row & 1) << 3 so that
// the two half-waves of an MFMA operand read (k = 2s and 2s+1, 32 consecutive i each) fall in
// disjoint bank halves.  LDS reads are inline asm (the compiler cannot tell them from the DMA
// writes in flight and would wait vmcnt(0) before each); their order is pinned by hand-counted
// lgkmcnt waits.  One barrier per stage.
#include "common.hpp"
#include "internal.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int XT = 128;              // tile side
constexpr int XROW = XT * 4;         // 512 B per k row of a panel

// ring geometry: KR k rows per stage, NS stages (LDS = NS * 2 * KR * 512 B)
template <int KR>
struct XGeo {
  static constexpr int PANEL = KR * XROW;       // one operand's rows of a stage
  static constexpr int STG = 2 * PANEL;         // A + B panels
  static constexpr int DMA = PANEL / 1024 / 4;  // DMA wave-instructions per wave per panel
};

__device__ uint4 gxz_zero16[4];      // the source of out-of-range chunks (zero-initialised)

// Upper-triangle tile order (8x8 super-tiles, as gemm.hip's upper_tile).
PT2Q_DEV void x_upper_tile(int L, int T, int& ti, int& tj) {
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

PT2Q_DEV int x_xcd_remap(int b, int nwg) {
  const int xcd = b % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// One panel of one stage: rows [k0, k0 + KR) (valid below kend) x columns [d0, d0 + 128) (valid
// below DMAX) of a K-major operand, into panel memory `pan` (swizzled).  Lane l of the wave's
// q-th instruction fills LDS chunk L = (wave * DMA + q) * 64 + l: row L / 32, position L % 32,
// which holds global chunk (L % 32) ^ ((row & 1) << 3).
template <int KR>
PT2Q_DEV void x_panel_dma(const float* base, long ld, int d0, int DMAX, int k0, int kend, uint8_t* pan) {
  constexpr int XDMA = XGeo<KR>::DMA;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  typedef __attribute__((address_space(3))) void* lptr;
#pragma unroll
  for (int q = 0; q < XDMA; ++q) {
    const int L = (wave * XDMA + q) * 64 + lane;
    const int kr = L >> 5, p = L & 31;
    const int c = p ^ ((kr & 1) << 3);
    const int k = k0 + kr, d = d0 + 4 * c;
    const bool ok = k < kend && d < DMAX;
    const void* src = ok ? (const void*)(base + (long)k * ld + d) : (const void*)gxz_zero16;
    __builtin_amdgcn_global_load_lds(src, (lptr)(pan + (wave * XDMA + q) * 1024), 16, 0, 0);
  }
}

// Fast staging of a whole in-range panel (rows [k0, k0 + KR) below kend, columns [d0, d0 + 128)
// below DMAX): this lane's byte offsets from the panel's first element, fixed for the launch, and a
// scalar base -- s_mov m0 + one global_load_lds per chunk instead of per-lane address math.
template <int KR>
PT2Q_DEV void x_panel_voff(long ld, uint32_t (&vo)[XGeo<KR>::DMA]) {
  constexpr int XDMA = XGeo<KR>::DMA;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int q = 0; q < XDMA; ++q) {
    const int L = (wave * XDMA + q) * 64 + lane;
    const int kr = L >> 5, c = (L & 31) ^ ((kr & 1) << 3);
    vo[q] = (uint32_t)(((long)kr * ld + 4 * c) * 4);
  }
}

template <int KR>
PT2Q_DEV void x_panel_dma_fast(const float* base, long ld, int d0, int k0, const uint32_t (&vo)[XGeo<KR>::DMA],
                               uint32_t pan) {
  constexpr int XDMA = XGeo<KR>::DMA;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* sb = (const char*)(base + (long)k0 * ld + d0);
#pragma unroll
  for (int q = 0; q < XDMA; ++q)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(vo[q]), "s"(sb),
                 "s"(pan + (uint32_t)((wave * XDMA + q) * 1024))
                 : "memory");
}

template <int OFF>
PT2Q_DEV float x_ld(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

struct XOps {
  float v[4][4];  // ring of 4 k-pair sets: a0, a1, b0, b1
};

// k-pair S (rows 2S, 2S+1 of the stage): its 4 operands were read into set S % 4; the reads of
// pair S+2 go into set (S+2) % 4 before pair S's MFMAs, so their latency hides under them.
template <int S>
PT2Q_DEV void x_read(XOps& o, uint32_t aA0, uint32_t aA1, uint32_t aB0, uint32_t aB1) {
  constexpr int c = S % 4, off = S * 2 * XROW;
  o.v[c][0] = x_ld<off>(aA0);
  o.v[c][1] = x_ld<off>(aA1);
  o.v[c][2] = x_ld<off>(aB0);
  o.v[c][3] = x_ld<off>(aB1);
}

// the next stage's fast DMAs, one A and one B chunk after the first MFMA of k-pair q (q < DMA), so
// their issue sits in MFMA shadows instead of in front of the stage (on = false: nothing)
template <int KR>
struct XStageIO {
  const char* sbA;
  const char* sbB;
  const uint32_t (&voA)[XGeo<KR>::DMA];
  const uint32_t (&voB)[XGeo<KR>::DMA];
  uint32_t mA, mB;
  bool on;
  template <int S>
  PT2Q_DEV void at() {
    if constexpr (S < XGeo<KR>::DMA) {
      if (on) {
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voA[S]), "s"(sbA),
                     "s"(mA + S * 1024)
                     : "memory");
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voB[S]), "s"(sbB),
                     "s"(mB + S * 1024)
                     : "memory");
      }
    }
  }
};

template <int S, int NP, class IO>
PT2Q_DEV void x_chain(f32x16 (&acc)[2][2], XOps& o, uint32_t aA0, uint32_t aA1, uint32_t aB0, uint32_t aB1, IO& io) {
  if constexpr (S == 0) {
    x_read<0>(o, aA0, aA1, aB0, aB1);
    x_read<1>(o, aA0, aA1, aB0, aB1);
    asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(o.v[0][0]), "+v"(o.v[0][1]), "+v"(o.v[0][2]), "+v"(o.v[0][3]));
  }
  if constexpr (S < NP) {
    constexpr int c = S % 4;
    if constexpr (S + 2 < NP) x_read<S + 2>(o, aA0, aA1, aB0, aB1);
    if constexpr (S > 0) {  // pair S-1's registers stay allocated until these reads are issued
      constexpr int p = (S + 3) % 4;
      asm volatile("" ::"v"(o.v[p][0]), "v"(o.v[p][1]), "v"(o.v[p][2]), "v"(o.v[p][3]));
    }
    __builtin_amdgcn_sched_barrier(0);
    // transposed tile: lane <-> C row (16-byte epilogue)
    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(o.v[c][2], o.v[c][0], acc[0][0], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    io.template at<S>();
    __builtin_amdgcn_sched_barrier(0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(o.v[c][3], o.v[c][0], acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(o.v[c][2], o.v[c][1], acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(o.v[c][3], o.v[c][1], acc[1][1], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (S + 1 < NP) {  // pair S+1 landed (pair S+2 may stay in flight)
      constexpr int c1 = (S + 1) % 4;
      if constexpr (S + 2 < NP)
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(o.v[c1][0]), "+v"(o.v[c1][1]), "+v"(o.v[c1][2]), "+v"(o.v[c1][3]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(o.v[c1][0]), "+v"(o.v[c1][1]), "+v"(o.v[c1][2]), "+v"(o.v[c1][3]));
    }
    x_chain<S + 1, NP>(acc, o, aA0, aA1, aB0, aB1, io);
  }
}

// wait until the y youngest stages (D DMAs each, 0 <= y <= 4) may stay in flight
template <int D>
PT2Q_DEV void x_vmwait(int y) {
  switch (y) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * D) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * D) : "memory"); break;
  }
}

struct XArgs {
  GemmDesc g;
  int tiles_m, tiles_n;
  int order;  // 0 row-major tiles, 1 upper (XCD super-tiles), 2 upper by columns (lauum)
};

// One workgroup's tile of item blockIdx.y: operands Ab / Bb, output Cz (the item's bases).
template <int NS, int KR>
PT2Q_DEV void gemmx_tile(const XArgs& X, const float* Ab, const float* Bb, float* const Cz, uint8_t* smem) {
  using GE = XGeo<KR>;
  constexpr int XSTG = GE::STG, XPANEL = GE::PANEL, XDMA = GE::DMA, XK = KR;
  const GemmDesc& g = X.g;
  int ti, tj;
  const int bid = blockIdx.x;
  if (X.order == 2) {  // K starts at the tile column: tj ascending = longest chains first
    tj = (int)((sqrtf(8.0f * (float)bid + 1.0f) - 1.0f) * 0.5f);
    while ((tj + 1) * (tj + 2) / 2 <= bid) ++tj;
    while (tj * (tj + 1) / 2 > bid) --tj;
    ti = bid - tj * (tj + 1) / 2;
  } else if (X.order == 1) {
    x_upper_tile(x_xcd_remap(bid, gridDim.x), X.tiles_n, ti, tj);
  } else {
    ti = bid / X.tiles_n;
    tj = bid % X.tiles_n;
  }
  const int i0 = ti * XT, j0 = tj * XT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1, li = lane & 31, lk = lane >> 5;
  const int kbeg = g.kstart_diag == 2 ? j0 : (g.kstart_diag == 1 ? i0 : 0);
  const int kend = g.K;
  const int nst = kend > kbeg ? (kend - kbeg + XK - 1) / XK : 0;
  // the C tile (chain modes) is loaded first, so that waiting for it does not wait for the DMA
  // prologue issued after it; accumulators: lane <-> C row, register groups of 4 <-> 4
  // consecutive C columns
  const bool chain = g.mode == GEMM_CHAIN_NEG || g.mode == GEMM_CHAIN_POS;
  const float csg = g.mode == GEMM_CHAIN_NEG ? -1.0f : 1.0f;
  f32x4 cv[2][2][4];
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int rn = 0; rn < 2; ++rn) {
      const int row = i0 + wr * 64 + rm * 32 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = j0 + wc * 64 + rn * 32 + 8 * q + 4 * lk;
        const bool in = chain && row < g.M && col < g.N;
        cv[rm][rn][q] = *(const f32x4*)(Cz + (in ? (long)row * g.ldc + col : 0));
      }
    }
  asm volatile("" ::: "memory");
  // prologue DMA: stages 0 .. NS-2 (stage p is whole -- the fast path -- when p < nfull)
  uint32_t voA[XDMA], voB[XDMA];
  x_panel_voff<KR>(g.lda, voA);
  x_panel_voff<KR>(g.ldb, voB);
  const uint32_t ldsb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  const int nfull = (i0 + XT <= g.M && j0 + XT <= g.N) ? (kend - kbeg) / XK : 0;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto stage = [&](int p) {
    if (p < nfull) {
      x_panel_dma_fast<KR>(Ab, g.lda, i0, kbeg + p * XK, voA, ldsb + (uint32_t)((p % NS) * XSTG));
      x_panel_dma_fast<KR>(Bb, g.ldb, j0, kbeg + p * XK, voB, ldsb + (uint32_t)((p % NS) * XSTG + XPANEL));
    } else {
      x_panel_dma<KR>(Ab, g.lda, i0, g.M, kbeg + p * XK, kend, smem + (p % NS) * XSTG);
      x_panel_dma<KR>(Bb, g.ldb, j0, g.N, kbeg + p * XK, kend, smem + (p % NS) * XSTG + XPANEL);
    }
  };
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nst) stage(p);
  f32x16 acc[2][2];
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int rn = 0; rn < 2; ++rn) {
      const int row = i0 + wr * 64 + rm * 32 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = j0 + wc * 64 + rn * 32 + 8 * q + 4 * lk;
        const bool in = chain && row < g.M && col < g.N;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[rm][rn][4 * q + e] = in ? csg * cv[rm][rn][q][e] : 0.0f;
      }
    }
  // per-lane LDS read addresses inside a stage (k-pair 0)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  auto opaddr = [&](int panel, int d) -> uint32_t {  // element (k = lk, column d) of a panel
    const int cch = (d >> 2) ^ (lk << 3);
    return (uint32_t)(panel + lk * XROW + cch * 16 + (d & 3) * 4);
  };
  const uint32_t oA0 = opaddr(0, wr * 64 + li), oA1 = opaddr(0, wr * 64 + 32 + li);
  const uint32_t oB0 = opaddr(XPANEL, wc * 64 + li), oB1 = opaddr(XPANEL, wc * 64 + 32 + li);
  XOps o;
  for (int t = 0; t < nst; ++t) {
    // stage t landed (this wave's DMAs; stage t+1 may stay in flight), then a raw barrier (the
    // fence of __syncthreads would wait vmcnt(0)); the barrier also retires every wave's reads
    // of the slot the next DMA reuses
    // (younger stages in flight: t+1 .. min(t+NS-2, nst-1))
    x_vmwait<2 * XDMA>(min(NS - 2, nst - 1 - t));
    asm volatile("s_barrier" ::: "memory");
    const int tn = t + NS - 1;
    // a whole next stage goes out inside the chain (XStageIO), any other one here
    const bool fastn = tn < nfull;
    if (tn < nst && !fastn) stage(tn);
    XStageIO<KR> sio{(const char*)(Ab + (long)(kbeg + tn * XK) * g.lda + i0),
                     (const char*)(Bb + (long)(kbeg + tn * XK) * g.ldb + j0), voA, voB,
                     ldsb + (uint32_t)((tn % NS) * XSTG + wv * XDMA * 1024),
                     ldsb + (uint32_t)((tn % NS) * XSTG + XPANEL + wv * XDMA * 1024), tn < nst && fastn};
    const uint32_t sb = lds0 + (uint32_t)((t % NS) * XSTG);
    x_chain<0, XK / 2>(acc, o, sb + oA0, sb + oA1, sb + oB0, sb + oB1, sio);
  }
  // epilogue
  const bool mirror = g.upper && g.mirror && ti != tj;
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int rn = 0; rn < 2; ++rn) {
      const int row = i0 + wr * 64 + rm * 32 + li;
      if (row >= g.M) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = j0 + wc * 64 + rn * 32 + 8 * q + 4 * lk;
        if (col >= g.N) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = csg * acc[rm][rn][4 * q + e];
        *(f32x4*)(Cz + (long)row * g.ldc + col) = v;
        if (mirror) {
#pragma unroll
          for (int e = 0; e < 4; ++e) Cz[(long)(col + e) * g.ldc + row] = v[e];
        }
      }
    }
}

template <int NS, int KR>
__global__ __launch_bounds__(256) void gemmx_kernel(XArgs X) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[NS * XGeo<KR>::STG];
  const long zo = (long)blockIdx.y * X.g.bstride;  // batch item (grid.y)
  gemmx_tile<NS, KR>(X, (const float*)X.g.A + zo, (const float*)X.g.B + zo, X.g.C + zo, smem);
}

// Symmetric Grams G[z] = X[z]ᵀX[z] of a batch with their own activation pointers: X[z] (N x m,
// row-major) is the K-major operand on both sides (A(i, k) = X[z][k][i]).
struct XPtrs {
  const float* X[PT2Q_GX_PTRS];
};

template <int NS, int KR>
__global__ __launch_bounds__(256) void gemmx_gram_kernel(XArgs X, XPtrs P) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[NS * XGeo<KR>::STG];
  const float* Xz = P.X[blockIdx.y];
  gemmx_tile<NS, KR>(X, Xz, Xz, X.g.C + (long)blockIdx.y * X.g.bstride, smem);
}

}  // namespace

// A batch of f32 Grams (STORE, upper tiles mirrored) on the LDS-DMA kernel: every element is the
// k-ascending chain over the N rows from 0, as the generic kernels form it (bit-identical).
// E_UNSUPPORTED unless every X[z] is 16-byte aligned and ldx, m are multiples of 4.
int pt2q_launch_gemmx_gram(const float* const* X, long N, int m, long ldx, float* G, long gstride, int batch,
                           hipStream_t st) {
  if (batch <= 0 || batch > PT2Q_GX_PTRS || m <= 0 || N < 0 || N > INT_MAX || ldx < m || !G) return PT2Q_E_ARG;
  auto al = [](const void* p) { return (uintptr_t)p % 16 == 0; };
  if (m % 4 || ldx % 4 || !al(G) || gstride % 4 || (long)m * m > gstride) return PT2Q_E_UNSUPPORTED;
  XPtrs P{};
  for (int z = 0; z < batch; ++z) {
    if (!X[z] && N > 0) return PT2Q_E_ARG;
    if (!al(X[z])) return PT2Q_E_UNSUPPORTED;
    P.X[z] = X[z] ? X[z] : (const float*)G;  // N = 0: never read
  }
  GemmDesc g{};
  g.M = m; g.N = m; g.K = (int)N;
  g.lda = ldx; g.a_layout = LAY_KMAJOR;
  g.ldb = ldx; g.b_layout = LAY_KMAJOR;
  g.in_dtype = PT2Q_F32;
  g.C = G; g.ldc = m;
  g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1;
  g.batch = batch; g.bstride = gstride;
  XArgs A{g, ceil_div(m, XT), ceil_div(m, XT), 1};
  const dim3 grid((unsigned)((long)A.tiles_n * (A.tiles_n + 1) / 2), (unsigned)batch);
  hipLaunchKernelGGL((gemmx_gram_kernel<2, 32>), grid, dim3(256), 0, st, A, P);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

// E_UNSUPPORTED unless: f32, both operands K-major, no output-row gather, mode STORE / CHAIN_NEG /
// CHAIN_POS, 16-byte aligned operands and C with leading dimensions and M, N multiples of 4.
int pt2q_launch_gemmx(const GemmDesc& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return PT2Q_OK;
  auto al = [](const void* p) { return (uintptr_t)p % 16 == 0; };
  if (g.in_dtype != PT2Q_F32 || g.a_layout != LAY_KMAJOR || g.b_layout != LAY_KMAJOR || g.crow ||
      !(g.mode == GEMM_STORE || g.mode == GEMM_CHAIN_NEG || g.mode == GEMM_CHAIN_POS) ||
      !al(g.A) || !al(g.B) || !al(g.C) || g.lda % 4 || g.ldb % 4 || g.ldc % 4 || g.M % 4 ||
      g.N % 4 || g.K < 0 || (g.mirror && !g.upper) || (g.kstart_diag == 2 && !g.upper))
    return PT2Q_E_UNSUPPORTED;
  XArgs X{g, ceil_div(g.M, XT), ceil_div(g.N, XT), 0};
  long tiles;
  if (g.upper) {
    if (X.tiles_m != X.tiles_n) return PT2Q_E_ARG;
    tiles = (long)X.tiles_n * (X.tiles_n + 1) / 2;
    X.order = g.kstart_diag == 2 ? 2 : 1;
  } else {
    tiles = (long)X.tiles_m * X.tiles_n;
  }
  const dim3 grid((unsigned)tiles, (unsigned)(g.batch > 1 ? g.batch : 1));
  switch (pt2q_tuning().gemmx_stages) {
    case 3: hipLaunchKernelGGL((gemmx_kernel<3, 32>), grid, dim3(256), 0, st, X); break;  // 96 KiB
    case 4: hipLaunchKernelGGL((gemmx_kernel<4, 16>), grid, dim3(256), 0, st, X); break;  // 64 KiB, 2 WGs/CU
    case 5: hipLaunchKernelGGL((gemmx_kernel<5, 16>), grid, dim3(256), 0, st, X); break;  // 80 KiB, 2 WGs/CU
    default: hipLaunchKernelGGL((gemmx_kernel<2, 32>), grid, dim3(256), 0, st, X); break;  // 64 KiB, 2 WGs/CU
  }
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}
