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
