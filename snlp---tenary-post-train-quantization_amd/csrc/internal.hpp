// Internal (non-exported) launchers shared between the libpt2q translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ---- Grouped block loops (pt2q_quantize_blocks_group): one launch per block step serves up to
// PT2Q_GROUP_MAX linears of one shape, grid.z = linear z.  Every per-linear pointer that lives
// in the linear's workspace slice moves by z * ws bytes; the raw Gram and the inverse Hessian
// come from per-linear tables.  count == 0 (and blockIdx.z == 0): a plain single-linear launch.
constexpr int PT2Q_GROUP_MAX = 16;
struct Grp {
  long ws;     // bytes between consecutive linears' workspace slices
  int count;   // linears in the group (0: not a grouped launch)
  const float* G[PT2Q_GROUP_MAX];     // raw Gram of linear z (AGA S1 source)
  const float* Hinv[PT2Q_GROUP_MAX];  // inverse Hessian of linear z (error-feedback coefficients)
};
template <class T>
__device__ __forceinline__ T* zws(T* p, long ws) {  // nullptr stays nullptr
  return p ? (T*)((char*)p + (long)blockIdx.z * ws) : p;
}
inline unsigned grp_z(const Grp* g) { return g && g->count > 0 ? (unsigned)g->count : 1u; }
inline Grp grp_or_none(const Grp* g) {
  if (g) return *g;
  Grp z{};
  return z;
}

// ---- ATQ (atq.hip)
// per-channel block (b = m > 512) on the caller's row-major W, outputs in place (atq.hip)
// per-channel rows on the caller's row-major W, codes held on-chip (atq_pc.hip)
bool pt2q_atq_pc_supported(const void* W, int wdtype, long ldw, int m);
int pt2q_launch_atq_pc(const void* W, int wdtype, long ldw, int n, int m, const float* S1, const float* d,
                       int max_iter, float* alpha, float* mu, void* T, int tdtype, long ldt, int* iters,
                       int* counters, hipStream_t st);
int pt2q_launch_atq_wide_rm(const void* W, int wdtype, long ldw, int n, int b, const float* S1, const float* d,
                            int max_iter, float* alpha, float* mu, void* T, int tdtype, long ldt, int* iters,
                            int* counters, hipStream_t st);
// grouped per-channel rows: up to PT2Q_PC_GROUP_MAX linears of one width m and W dtype (row counts
// may differ) in one launch sequence; S1 / d per linear (nullable S1: no AGA); counters (2 ints,
// zeroed) and *iters (zeroed) per linear
constexpr int PT2Q_PC_GROUP_MAX = 16;
struct PcLinear {
  const void* W;
  long ldw;
  int n;
  const float* S1;
  const float* d;
  float* alpha;
  float* mu;
  void* T;
  long ldt;
  int* iters;
  int* counters;
  int64_t* perm;  // the setup's [0, m) (pt2q_quantize_perchannel_group), unused by the kernels
};
int pt2q_launch_atq_pc_group(int count, const PcLinear* lin, int wdtype, int m, int max_iter, int tdtype,
                             hipStream_t st);
int pt2q_launch_atq_rm_group(int count, const PcLinear* lin, int wdtype, int m, int max_iter, int tdtype,
                             hipStream_t st);
int pt2q_launch_atq_block(const float* Wt, long ldw, int n, const int* blk, int b,
                          const float* S1, const float* d, int max_iter, float* alpha, float* mu,
                          int8_t* Tt, long ldt, float* Et, long lde, int* iters, int* counters,
                          hipStream_t st, const float* Hinv = nullptr, long ldh = 0,
                          const int* rem = nullptr, int nr = 0, float* C = nullptr, long ldc = 0,
                          int* iters_part = nullptr,  // 4 ceil(n/16) ints of scratch (one per wave), nullable
                          // variant M, b <= 128: S1/d (into S1, d) formed inside the launch from
                          // the raw Gram G; s1sync: 2 zeroed ints
                          const float* G = nullptr, long ldg = 0, int* s1sync = nullptr,
                          int* status = nullptr,  // status word (stall reporting), nullable
                          const Grp* grp = nullptr);

// ---- SSR / selection (ssr.hip)
// cnt (nullable): pt2q_ssr_counter_ints(n) zeroed ints -> one fused wbar launch (self-resetting)
// pre: part already holds the chunk partials of rem (written by the error feedback of the previous
// block, pt2q_launch_ef with part); only their sum and the norm remain (needs the fused path)
int pt2q_launch_ssr_similarity(const float* Wt, long ldw, int n, const int* rem, int r,
                               float* part, float* wn, float* sim, hipStream_t st, int* cnt = nullptr,
                               const Grp* grp = nullptr, bool pre = false);
inline int pt2q_ssr_counter_ints(int n) { return (n + 255) / 256 + 1; }
int pt2q_launch_ssr_topk(const float* sim, const int* rem, int r, int b, int* blk, int* newrem,
                         int64_t* perm_out, hipStream_t st, const float* G = nullptr, long ldg = 0,
                         float* S1 = nullptr, float* d = nullptr, int* sync = nullptr,
                         int* status = nullptr, const Grp* grp = nullptr);
int pt2q_launch_select_seq(int mode, int p0, int bs, int m, const int* rem, int* blk,
                           int* newrem, int64_t* perm_out, hipStream_t st, const Grp* grp = nullptr);
int pt2q_launch_s1_batched(const float* G, long ldg, int m, int batch, long sG, float* S1d, hipStream_t st,
                           bool upper = false);
int pt2q_launch_aga_s1(int src, const float* A, long lda, const int* blk, int b, float* S1,
                       float* d, hipStream_t st);
int pt2q_launch_ef_coeffs(const float* Hinv, long ldh, const int* blk, int bs, const int* rem,
                          int nr, float* C, long ldc, hipStream_t st);
size_t pt2q_ssr_scratch_floats(int n, int m);

// ---- GEMM (gemm.hip)
enum GemmMode { GEMM_STORE = 0, GEMM_ADD = 1, GEMM_SUB = 2, GEMM_CHAIN_NEG = 3, GEMM_CHAIN_POS = 4 };
enum GemmLayout { LAY_KMAJOR = 0, LAY_ROWMAJOR = 1 };
struct GemmDesc {
  int M, N, K;
  const void* A;  // element (i,k): KMAJOR A[k*lda + i], ROWMAJOR A[i*lda + k]
  long lda;
  int a_layout;
  const void* B;  // element (k,j): KMAJOR B[k*ldb + j], ROWMAJOR B[j*ldb + k]
  long ldb;
  int b_layout;
  int in_dtype;   // PT2Q_F32 / PT2Q_F16 / PT2Q_BF16 (applies to both A and B)
  float* C;       // C[crow(i)*ldc + j]
  long ldc;
  const int* crow;  // nullable output-row gather
  int mode;
  int upper;        // compute only tiles with tile_i <= tile_j
  int mirror;       // with upper: also write C[j][i] (full symmetric output)
  int kstart_diag;  // skip K below min(tile row start): exact for triangular operands (zeros)
  int batch;        // > 1: that many independent GEMMs, item z at A/B/C + z * bstride elements
  long bstride;     //      (gemmx and the rank-<=128 update run them in one launch, grid.y = z)
};
int pt2q_launch_gemm(const GemmDesc& g, hipStream_t st);
// batch (<= 128) f32 Grams G + z * gstride = X[z]ᵀX[z] (N x m, ld ldx; G ld m), bit-equal to pt2q_gram per item
int pt2q_launch_gram_f32_batched(const float* const* X, long N, int m, long ldx, float* G, long gstride, int batch,
                                 hipStream_t st);
// block error feedback Wt[crow[e]][i] -= sum_k Ck[k][e] Et[k][i] (ef.hip); E_UNSUPPORTED if bs > 128
// part (nullable): also the w-bar chunk partials of the updated rows, part[c][i] for i < n (the
// next block's SSR mean over crow, ssr.hip wbar_chunk order)
int pt2q_launch_ef(const float* Ck, long ldk, const float* Et, float* Wt, long ldw, long wt_rows,
                   const int* crow, int nr, int bs, hipStream_t st, const Grp* grp = nullptr,
                   float* part = nullptr, int n = 0);
// two independent f32 GEMMs in one launch (either may be empty)
// dA != nullptr: also factor the diagonal block (dp0, dp0) of dA (nb dnb) in the same launch if
// g0's first tile is that block; *fused reports whether it did (else launch the factor).
int pt2q_launch_gemm2(const GemmDesc& g0, const GemmDesc& g1, hipStream_t st, float* dA = nullptr,
                      long dld = 0, int dp0 = 0, int dnb = 0, int* info = nullptr,
                      bool* fused = nullptr);
// f32 chain GEMM with K-major operands, LDS-DMA staged (gemmx.hip); E_UNSUPPORTED if the desc
// does not fit it (then use pt2q_launch_gemm)
int pt2q_launch_gemmx(const GemmDesc& g, hipStream_t st);
// a batch of f32 Grams with their own activation pointers on the same kernel (gemmx.hip)
constexpr int PT2Q_GX_PTRS = 128;
int pt2q_launch_gemmx_gram(const float* const* X, long N, int m, long ldx, float* G, long gstride, int batch,
                           hipStream_t st);
// symmetric Gram (STORE/ADD); flags (nullable): pt2q_gram_flags_ints(m) ints of scratch
// status (nullable): the caller's status word for stall reports (else a word of the flag area)
int pt2q_launch_gram(const GemmDesc& g, int* flags, hipStream_t st, int* status = nullptr);
size_t pt2q_gram_flags_ints(int m);
// 16-bit-input Gram on the 16-bit MFMA (gram16.hip): every shape, STORE / ADD / CHAIN_POS
int pt2q_launch_gram16(const GemmDesc& g, int* flags, hipStream_t st, int* status = nullptr);
size_t pt2q_gram16_flags_ints(int m);
int pt2q_launch_gram16_batched(const void* const* X, int dtype, long N, int m, long ldx, float* G, long gstride,
                               int batch, hipStream_t st, bool upper = false);

// ---- misc (misc.hip)
int pt2q_launch_transpose_to_f32(const void* src, int dtype, long lds, int rows, int cols,
                                 float* dst, long ldd, hipStream_t st);
int pt2q_launch_transpose_i8(const int8_t* src, long lds, int rows, int cols, void* dst, int ddtype,
                             long ldd, hipStream_t st);
int pt2q_launch_transpose_f32(const float* src, long lds, int rows, int cols, float* dst, long ldd,
                              hipStream_t st);
// batch > 1 (m <= SUMN_LDS_MAX, damp given): items at G / H + z * bs, damp[z], in one launch pair
int pt2q_launch_prepare_hessian(const float* G, long ldg, int m, long nsamples, float percdamp,
                                float* H, long ldh, float* damp, hipStream_t st, bool upper_only = false,
                                int batch = 1, long bs = 0);

// ---- Cholesky (chol.hip)
// batch > 1: that many independent inverses, all packed (ld = m, item z at + z * m * m, info + z)
int pt2q_launch_cholesky_inverse(const float* H, long ldh, int m, float* Hinv, long ldhi,
                                 float* U, float* Ui, int* info, hipStream_t st, bool h_upper_form = false,
                                 int batch = 1);
