// Ternary-weight linear layer for inference (reference model.py:17-127
// TernaryLinear, model.py:174-225 replace_linear_with_ternary).
//
//   y[t][i] = Σ_p Wd[i][p] · x[t][g[p]] + bias[i],   Wd[i][p] = TX(α[i][p/bs]·c[i][p] + μ[i][p/bs])
//
// p runs over "positions" (the input columns in block order), g maps a position to its input
// column and c ∈ {-1, 0, +1} are the codes at that position.  The correct reconstruction
// (gptq.py:201-230) uses g = perm, c[i][p] = T[i][perm[p]]; the reference's TernaryLinear
// forward (which permutes twice) is the same formula with g = perm∘perm and
// c[i][p] = T[i][p], so one kernel serves both.  Wd is rounded to the activation dtype TX
// exactly where the reference materialises its weight in alpha's dtype (model.py:97-110).
//
// Weights stay 2-bit packed in HBM (n x P/4 bytes, 16x smaller than fp32): each lane loads the
// 64 codes it needs for a 128-position block with ONE 16-byte load (the packing below puts a
// lane's codes together) and dequantises them in registers straight into the operand of
// v_mfma_f32_32x32x16_{f16,bf16}; activations are pre-gathered into position order (x_sel).
// No LDS.  Decode-sized token counts split K across workgroups; partial sums are reduced in a
// fixed order (deterministic).
#include "common.hpp"
#include "internal.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int TL_PB = 128;  // positions per packed block (one 16-byte load per lane)

// Packed layout: row i, block kb (128 positions), half h (0/1), group g (0..7), j (0..7):
// position p = 128 kb + 16 g + 8 h + j lives at byte  i*(P/4) + 32 kb + 16 h + 2 g + j/4,
// bits 2*(j%4), code stored as c + 1 ∈ {0, 1, 2}.
__global__ void tl_pack_kernel(const int8_t* T, long ldt, int n, int m, const int64_t* perm,
                               int mode, int P, uint8_t* out) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one output byte
  const long rowbytes = P / 4;
  if (q >= (long)n * rowbytes) return;
  const int i = (int)(q / rowbytes);
  const int b = (int)(q % rowbytes);
  const int kb = b / 32, h = (b % 32) / 16, g = (b % 16) / 2, j0 = (b % 2) * 4;
  uint8_t v = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int p = 128 * kb + 16 * g + 8 * h + j0 + s;
    int c = 0;
    if (p < m) {
      const long col = (mode == 0) ? perm[p] : p;  // correct: T[i][perm[p]]; compat: T[i][p]
      c = T[(long)i * ldt + col];
    }
    v |= (uint8_t)((c + 1) << (2 * s));
  }
  out[q] = v;
}

// g[p] (int32): correct mode perm[p]; compat mode perm[perm[p]]; -1 for padding positions
__global__ void tl_gather_index_kernel(const int64_t* perm, int m, int mode, int P, int* g) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  if (p >= m) {
    g[p] = -1;
    return;
  }
  const long a = perm[p];
  g[p] = (int)((mode == 0) ? a : perm[a]);
}

// x_sel[t][p] = x[t][g[p]] (0 for padding), 16-bit elements
__global__ void tl_gather_x_kernel(const uint16_t* x, long ldx, int tokens, const int* g, int P,
                                   uint16_t* xs) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)tokens * P) return;
  const int t = (int)(q / P), p = (int)(q % P);
  const int c = g[p];
  xs[q] = (c >= 0) ? x[(long)t * ldx + c] : (uint16_t)0;
}

template <bool BF16>
PT2Q_DEV uint32_t to_bits(float v) {
  if constexpr (BF16) {
    __bf16 h = (__bf16)v;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    return u;
  } else {
    _Float16 h = (_Float16)v;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    return u;
  }
}

// One wave = 32 output features x 32*NT tokens (the features' A operand is dequantised once and
// reused by the NT token tiles); 4 waves stack along features (128 features per workgroup).
// Dequantisation: per (row, block) the three possible weights TX(mu - alpha), TX(mu),
// TX(mu + alpha) (= TX(alpha*c + mu) for c = -1, 0, 1, the reference's rounding) sit in two
// registers as an 8-byte table; a code pair (c0+1, c1+1) becomes a v_perm_b32 byte selector
// (q * 0x202 + 0x01000100), so two weights cost about three VALU ops.
// blockIdx.z = K split: positions [z*kchunk, min(P, (z+1)*kchunk)).
template <bool BF16, int NT>
__global__ __launch_bounds__(256) void tl_gemm_kernel(const uint8_t* codes, int P, const float* alpha,
                                                      const float* mu, int B, int bs,
                                                      const uint16_t* xs, int tokens, int n,
                                                      int kchunk, float* part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int i = blockIdx.x * 128 + w * 32 + r;  // A row (output feature) of this lane
  const bool irow = i < n;
  const int p0 = blockIdx.z * kchunk, p1 = min(P, p0 + kchunk);
  const uint8_t* crow = codes + (long)(irow ? i : 0) * (P / 4);
  const float* arow = alpha + (long)(irow ? i : 0) * B;
  const float* mrow = mu + (long)(irow ? i : 0) * B;
  const uint16_t* xrow[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int t = (blockIdx.y * NT + u) * 32 + r;
    xrow[u] = xs + (long)(t < tokens ? t : 0) * P;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[u][e] = 0.0f;
  int tblk = -1;
  uint32_t tab0 = 0, tab1 = 0;
  for (int kb = p0 / TL_PB; kb < p1 / TL_PB; ++kb) {
    const u32x4 cw = *(const u32x4*)(crow + 32 * kb + 16 * h);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int pg = TL_PB * kb + 16 * g;
      const int blk = pg / bs;
      if (blk != tblk) {  // new scale block: rebuild the weight table
        tblk = blk;
        const float a = arow[blk], mm = mrow[blk];
        tab0 = to_bits<BF16>(mm - a) | (to_bits<BF16>(mm) << 16);
        tab1 = to_bits<BF16>(mm + a);
      }
      const uint32_t cb = (cw[g >> 1] >> (16 * (g & 1))) & 0xffffu;  // 8 codes, 2 bits each
      uint32_t wv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t q = ((cb >> (4 * j)) & 3u) | (((cb >> (4 * j + 2)) & 3u) << 16);
        wv[j] = __builtin_amdgcn_perm(tab1, tab0, q * 0x202u + 0x01000100u);
      }
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const u32x4 xv = *(const u32x4*)(xrow[u] + pg + 8 * h);
        if constexpr (BF16) {
          bf16x8 A, X;
          __builtin_memcpy(&A, wv, 16);
          __builtin_memcpy(&X, &xv, 16);
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, X, acc[u], 0, 0, 0);
        } else {
          f16x8 A, X;
          __builtin_memcpy(&A, wv, 16);
          __builtin_memcpy(&X, &xv, 16);
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, X, acc[u], 0, 0, 0);
        }
      }
    }
  }
  // D[row][col]: col = token (lane & 31), row = feature (e&3) + 8(e>>2) + 4h
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int tt = (blockIdx.y * NT + u) * 32 + r;
    if (tt >= tokens) continue;
    float* prow = part + ((long)blockIdx.z * tokens + tt) * n;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ii = blockIdx.x * 128 + w * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (ii < n) prow[ii] = acc[u][e];
    }
  }
}

// Prefill (many tokens): one workgroup = 256 features x 128 tokens, 4 waves of 64 features x
// 128 tokens (2 x 4 MFMA tiles, D[token][feature]: lane <-> feature, so the epilogue stores 32
// consecutive features per half-wave).  The gathered activations go global -> LDS by LDS-DMA in
// stages of 64 positions x 128 tokens (16 KiB, ring of 3; 16-byte chunks XOR-swizzled by
// (token >> 1) & 7, so the 16 lanes a ds_read_b128 serves per clock hit 16 distinct 4-bank
// groups) and are shared by the 4 waves;
// every wave dequantises its own 64 features per k-step from the 2-bit codes through the same
// v_perm_b32 tables as tl_gemm_kernel.  Codes and scales of the next 128-position block come
// one block ahead by LDS-DMA as well (plain loads would make the compiler wait vmcnt(0) -- every
// DMA in flight -- before their first use); the hand-counted vmcnt waits below cover them.
// Needs bs % 128 == 0 (a table per 128-position block); y (+ bias) is written directly, no split
// partials.
constexpr int TP_F = 256, TP_T = 128, TP_KS = 64;
constexpr int TP_ROW = TP_KS * 2;            // 128 B per token row of a stage
constexpr int TP_STG = TP_T * TP_ROW;        // 16 KiB
constexpr int TP_NS = 3;
constexpr int TP_DMA = TP_STG / (256 * 16);  // DMA instructions per thread per stage (4)
constexpr int TP_CB = TP_F * 32;             // codes of one 128-position block: 32 B per feature
constexpr int TP_BLK = TP_CB + 2 * TP_F * 4; // + alpha and mu per feature (10 KiB)
constexpr int TP_FETCH = 4;                  // DMA instructions per thread per block (2 codes, alpha, mu)

__device__ uint4 tp_zero16;  // DMA source past the data (zero-initialised)

template <int OFF>
PT2Q_DEV u32x4 tp_ld(uint32_t addr) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

PT2Q_DEV float tp_ldf(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

template <bool BF16>
PT2Q_DEV void tp_table(float a, float mm, uint32_t& t0, uint32_t& t1) {
  t0 = to_bits<BF16>(mm - a) | (to_bits<BF16>(mm) << 16);
  t1 = to_bits<BF16>(mm + a);
}

// 8 weights (one 16-position group of a lane's half) from 8 packed codes
PT2Q_DEV void tp_decode(uint32_t cb, uint32_t t0, uint32_t t1, uint32_t (&wv)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t q = ((cb >> (4 * j)) & 3u) | (((cb >> (4 * j + 2)) & 3u) << 16);
    wv[j] = __builtin_amdgcn_perm(t1, t0, q * 0x202u + 0x01000100u);
  }
}

template <bool BF16, typename TY>
__global__ __launch_bounds__(256, 2) void tl_prefill_kernel(const uint8_t* codes, int P, const float* alpha,
                                                            const float* mu, int B, int bs, const uint16_t* xs,
                                                            int tokens, int n, const float* bias, TY* y,
                                                            long ldy) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[TP_NS * TP_STG + 2 * TP_BLK];
  typedef __attribute__((address_space(3))) void* lptr;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(w);
  const int r = lane & 31, h = lane >> 5;
  const int fb = blockIdx.x * TP_F;  // the workgroup's first feature
  const int t0 = blockIdx.y * TP_T;
  const int nst = P / TP_KS;  // P is a multiple of 128: an even number of stages
  // activations of stage st: thread's q-th chunk = LDS slot L = (w * TP_DMA + q) * 64 + lane,
  // token row L / 8, holding global chunk (L % 8) ^ ((row >> 1) & 7)
  auto dma = [&](int st) {
    uint8_t* slot = smem + (st % TP_NS) * TP_STG;
#pragma unroll
    for (int q = 0; q < TP_DMA; ++q) {
      const int L = (wv * TP_DMA + q) * 64 + lane;
      const int row = L >> 3, c = (L & 7) ^ ((row >> 1) & 7);
      const int t = t0 + row;
      const void* src = t < tokens ? (const void*)(xs + (long)t * P + st * TP_KS + 8 * c) : (const void*)&tp_zero16;
      __builtin_amdgcn_global_load_lds(src, (lptr)(slot + (wv * TP_DMA + q) * 1024), 16, 0, 0);
    }
  };
  // codes (feature fl at fl * 32 + 16 half) and scales (alpha[fl], mu[fl]) of block kb, by
  // LDS-DMA into block slot kb % 2: TP_FETCH instructions per thread, issued in this order
  auto fetch = [&](int kb) {
    uint8_t* bsl = smem + TP_NS * TP_STG + (kb & 1) * TP_BLK;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int L = (wv * 2 + q) * 64 + lane;
      const int f = fb + (L >> 1);
      const void* src = f < n ? (const void*)(codes + (long)f * (P / 4) + 32 * kb + 16 * (L & 1))
                              : (const void*)&tp_zero16;
      __builtin_amdgcn_global_load_lds(src, (lptr)(bsl + (wv * 2 + q) * 1024), 16, 0, 0);
    }
    const int f = fb + wv * 64 + lane, blk = (kb * 128) / bs;
    const void* sa = f < n ? (const void*)(alpha + (long)f * B + blk) : (const void*)&tp_zero16;
    const void* sm = f < n ? (const void*)(mu + (long)f * B + blk) : (const void*)&tp_zero16;
    __builtin_amdgcn_global_load_lds(sa, (lptr)(bsl + TP_CB + wv * 256), 4, 0, 0);
    __builtin_amdgcn_global_load_lds(sm, (lptr)(bsl + TP_CB + TP_F * 4 + wv * 256), 4, 0, 0);
  };
  float bvs[2];  // bias of the lane's two features (waited for before any DMA is in flight)
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int f = fb + wv * 64 + 32 * a + r;
    bvs[a] = (bias && f < n) ? bias[f] : 0.0f;
  }
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(bvs[0]), "+v"(bvs[1])::"memory");
  fetch(0);
  dma(0);
  if (nst > 1) dma(1);
  f32x16 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][u][e] = 0.0f;
  // lane's LDS byte offset of k-step s inside a stage (token row r of token tile 0)
  uint32_t offs[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) offs[s2] = r * TP_ROW + (((2 * s2 + h) ^ ((r >> 1) & 7)) * 16);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  const uint32_t blk0 = lds0 + TP_NS * TP_STG;
  u32x4 cw[2];
  uint32_t tab0[2], tab1[2];
  for (int st = 0; st < nst; ++st) {
    const bool blk_start = (st & 1) == 0;
    // stage st landed.  Issue order: at an even stage e [block fetch for e/2 + 1][DMA e+2], at
    // an odd one [DMA e+2].  Younger than stage st's DMA: at an even st, stage st+1's DMA; at
    // an odd st, the block fetch and stage st+1's DMA, both issued at st-1.  At an even st the
    // fetch of this block (issued at st-2, before stage st's DMA) has landed too.
    if (st + 1 >= nst)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (blk_start)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TP_DMA) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TP_DMA + TP_FETCH) : "memory");
    asm volatile("s_barrier" ::: "memory");
    if (blk_start) {  // this block's codes and tables from LDS, then fetch the next block
      const uint32_t bsl = blk0 + ((st >> 1) & 1) * TP_BLK;
      float av[2], mv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int fl = wv * 64 + 32 * a + r;
        cw[a] = tp_ld<0>(bsl + fl * 32 + 16 * h);
        av[a] = tp_ldf(bsl + TP_CB + fl * 4);
        mv[a] = tp_ldf(bsl + TP_CB + TP_F * 4 + fl * 4);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cw[0]), "+v"(cw[1]), "+v"(av[0]), "+v"(av[1]), "+v"(mv[0]),
                   "+v"(mv[1])::"memory");
#pragma unroll
      for (int a = 0; a < 2; ++a) tp_table<BF16>(av[a], mv[a], tab0[a], tab1[a]);
      if (st + 2 < nst) fetch(st / 2 + 1);
    }
    if (st + 2 < nst) dma(st + 2);
    const uint32_t sb = lds0 + (uint32_t)((st % TP_NS) * TP_STG);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const uint32_t ad = sb + offs[s2];
      u32x4 xv[4];
      xv[0] = tp_ld<0>(ad);
      xv[1] = tp_ld<32 * TP_ROW>(ad);
      xv[2] = tp_ld<64 * TP_ROW>(ad);
      xv[3] = tp_ld<96 * TP_ROW>(ad);
      const int g = (st & 1) * 4 + s2;  // 16-position group inside the 128-position block
      uint32_t wq[2][4];
#pragma unroll
      for (int a = 0; a < 2; ++a) tp_decode((cw[a][g >> 1] >> (16 * (g & 1))) & 0xffffu, tab0[a], tab1[a], wq[a]);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xv[0]), "+v"(xv[1]), "+v"(xv[2]), "+v"(xv[3]));
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if constexpr (BF16) {
            bf16x8 Wb, Xb;
            __builtin_memcpy(&Wb, wq[a], 16);
            __builtin_memcpy(&Xb, &xv[u], 16);
            acc[a][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Xb, Wb, acc[a][u], 0, 0, 0);
          } else {
            f16x8 Wb, Xb;
            __builtin_memcpy(&Wb, wq[a], 16);
            __builtin_memcpy(&Xb, &xv[u], 16);
            acc[a][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Xb, Wb, acc[a][u], 0, 0, 0);
          }
        }
    }
  }
  // D[token][feature]: feature = lane & 31 (+ 32 a), token = (e & 3) + 8 (e >> 2) + 4 h (+ 32 u)
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int f = fb + wv * 64 + 32 * a + r;
    if (f >= n) continue;
    const float bv = bvs[a];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int t = t0 + 32 * u + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (t < tokens) y[(long)t * ldy + f] = (TY)(bias ? acc[a][u][e] + bv : acc[a][u][e]);
      }
  }
}

// y[t][i] = ((part[0] + part[1]) + ...) + bias  (split order fixed), stored as fp32 or TX
template <typename TY>
__global__ void tl_reduce_kernel(const float* part, int splits, int tokens, int n,
                                 const float* bias, TY* y, long ldy) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)tokens * n) return;
  const int t = (int)(q / n), i = (int)(q % n);
  float s = part[q];
  for (int z = 1; z < splits; ++z) s = s + part[(long)z * tokens * n + q];
  if (bias) s = s + bias[i];
  y[(long)t * ldy + i] = (TY)s;
}

}  // namespace

extern "C" size_t pt2q_ternary_linear_positions(int m) { return (size_t)ceil_div(m, TL_PB) * TL_PB; }

extern "C" int pt2q_ternary_pack(const int8_t* T, int64_t ldt, int n, int m, const int64_t* perm,
                                 int mode, uint8_t* codes, int* gather, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!T || !perm || !codes || !gather || n <= 0 || m <= 0 || ldt < m || (mode != 0 && mode != 1))
    return PT2Q_E_ARG;
  const int P = (int)pt2q_ternary_linear_positions(m);
  const long nbytes = (long)n * (P / 4);
  hipLaunchKernelGGL(tl_pack_kernel, dim3(ceil_div(nbytes, 256)), dim3(256), 0, st, T, (long)ldt, n,
                     m, perm, mode, P, codes);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(tl_gather_index_kernel, dim3(ceil_div(P, 256)), dim3(256), 0, st, perm, m, mode,
                     P, gather);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

namespace {
// Launch plan shared by the workspace query and the launcher: K split so that decode-sized calls
// still put ~2 workgroups on every CU (prefill-sized calls get splits = 1), and token tiles per
// wave (each dequantised operand reused across up to 4 MFMA token tiles).
struct TlPlan {
  int splits, kchunk, NT;
};
TlPlan tl_plan(int tokens, int n, int m) {
  const int P = (int)pt2q_ternary_linear_positions(m);
  const int tiles = ceil_div(n, 128) * ceil_div(tokens, tokens >= 512 ? 128 : (tokens >= 128 ? 64 : 32));
  const int nkb = P / TL_PB;
  int splits = 1;
  while (splits < 16 && tiles * splits < 512 && nkb / (splits * 2) >= 2) splits *= 2;
  TlPlan p;
  p.kchunk = ceil_div(nkb, splits) * TL_PB;
  p.splits = ceil_div(P, p.kchunk);
  p.NT = tokens >= 512 ? 4 : (tokens >= 128 ? 2 : 1);
  return p;
}
}  // namespace

extern "C" size_t pt2q_ternary_linear_workspace_bytes(int tokens, int n, int m) {
  if (tokens <= 0 || n <= 0 || m <= 0) return 0;
  const size_t P = pt2q_ternary_linear_positions(m);
  const TlPlan pl = tl_plan(tokens, n, m);
  // gathered activations (tokens x P 16-bit) + the split partial sums (splits x tokens x n fp32)
  return ((size_t)tokens * P * 2 + 255) / 256 * 256 + (size_t)pl.splits * tokens * n * 4 + 256;
}

extern "C" int pt2q_ternary_linear(const void* x, int xdtype, int tokens, int64_t ldx, int n, int m,
                                   const uint8_t* codes, const int* gather, const float* alpha,
                                   const float* mu, int B, int bs, const float* bias, void* y,
                                   int ydtype, int64_t ldy, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!x || !codes || !gather || !alpha || !mu || !y || tokens <= 0 || n <= 0 || m <= 0 ||
      ldx < m || ldy < n || B <= 0 || bs <= 0)
    return PT2Q_E_ARG;
  if (xdtype != PT2Q_F16 && xdtype != PT2Q_BF16) return PT2Q_E_UNSUPPORTED;
  if (ydtype != xdtype && ydtype != PT2Q_F32) return PT2Q_E_ARG;
  if (bs < m && bs % 16 != 0) return PT2Q_E_UNSUPPORTED;  // alpha constant within a 16-group
  if ((long)ceil_div(m, bs < m ? bs : m) > B) return PT2Q_E_ARG;
  const int P = (int)pt2q_ternary_linear_positions(m);
  const int bse = bs < m ? bs : P;  // per-channel: one scale for every position
  if (workspace_bytes < pt2q_ternary_linear_workspace_bytes(tokens, n, m)) return PT2Q_E_WORKSPACE;
  uint16_t* xs = (uint16_t*)workspace;
  float* part = (float*)((char*)workspace + ((size_t)tokens * P * 2 + 255) / 256 * 256);
  hipLaunchKernelGGL(tl_gather_x_kernel, dim3(ceil_div((long)tokens * P, 256)), dim3(256), 0, st,
                     (const uint16_t*)x, (long)ldx, tokens, gather, P, xs);
  PT2Q_LAUNCH_CHECK();
  if (tokens >= 256 && bse % 128 == 0) {
    auto launch_p = [&](auto kern, auto* yp) {
      hipLaunchKernelGGL(kern, dim3(ceil_div(n, TP_F), ceil_div(tokens, TP_T)), dim3(256), 0, st, codes, P, alpha,
                         mu, B, bse, xs, tokens, n, bias, yp, (long)ldy);
    };
    if (ydtype == PT2Q_F32)
      xdtype == PT2Q_BF16 ? launch_p(tl_prefill_kernel<true, float>, (float*)y)
                          : launch_p(tl_prefill_kernel<false, float>, (float*)y);
    else if (ydtype == PT2Q_BF16)
      launch_p(tl_prefill_kernel<true, __bf16>, (__bf16*)y);
    else
      launch_p(tl_prefill_kernel<false, _Float16>, (_Float16*)y);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  const TlPlan pl = tl_plan(tokens, n, m);
  const int splits = pl.splits, kchunk = pl.kchunk, NT = pl.NT;
  dim3 grid(ceil_div(n, 128), ceil_div(tokens, 32 * NT), splits);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, codes, P, alpha, mu, B, bse, xs, tokens, n,
                       kchunk, part);
  };
  if (xdtype == PT2Q_BF16)
    NT == 4 ? launch(tl_gemm_kernel<true, 4>) : NT == 2 ? launch(tl_gemm_kernel<true, 2>)
                                                       : launch(tl_gemm_kernel<true, 1>);
  else
    NT == 4 ? launch(tl_gemm_kernel<false, 4>) : NT == 2 ? launch(tl_gemm_kernel<false, 2>)
                                                        : launch(tl_gemm_kernel<false, 1>);
  PT2Q_LAUNCH_CHECK();
  const long tot = (long)tokens * n;
  if (ydtype == PT2Q_F32)
    hipLaunchKernelGGL(tl_reduce_kernel<float>, dim3(ceil_div(tot, 256)), dim3(256), 0, st, part,
                       splits, tokens, n, bias, (float*)y, (long)ldy);
  else if (ydtype == PT2Q_BF16)
    hipLaunchKernelGGL(tl_reduce_kernel<__bf16>, dim3(ceil_div(tot, 256)), dim3(256), 0, st, part,
                       splits, tokens, n, bias, (__bf16*)y, (long)ldy);
  else
    hipLaunchKernelGGL(tl_reduce_kernel<_Float16>, dim3(ceil_div(tot, 256)), dim3(256), 0, st, part,
                       splits, tokens, n, bias, (_Float16*)y, (long)ldy);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}
