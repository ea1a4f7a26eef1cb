// Cholesky factorisation and inverse of the damped Hessian (main.py:136-139, gptq.py:101-103:
// torch.linalg.cholesky + torch.cholesky_inverse) under the PT2Q contract:
//
//   U (upper, H = UᵀU):  acc = H[k][i]; for j < k ascending: acc = fmaf(-U[j][k], U[j][i], acc);
//                        U[k][k] = sqrt(acc) (breakdown if !(acc > 0)); U[k][i] = acc / U[k][k]
//   Uinv = U⁻¹:          Uinv[k][k] = 1/U[k][k]; Uinv[k][i] = -(j-ascending chain over
//                        j in [k,i) of Uinv[k][j]*U[j][i]) / U[i][i]
//   Hinv = Uinv·Uinvᵀ:   Hinv[i][k] = j-ascending chain over j >= max(i,k) of Uinv[i][j]*Uinv[k][j]
//
// Blocked right-looking with NB = 64 blocks inside panels of CP = 512 / 1024 rows; the strip updates
// inside a panel run on the rank-<=128 kernel (gemm.hip), the panel-wide updates and lauum on
// the LDS-DMA f32 GEMM (gemmx.hip).  Their k-ordered chains keep every element bit-identical to
// the unblocked definition above (oracle/pt2q_oracle.c).
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

#include "common.hpp"
#include "internal.hpp"
#include "chol_diag.hpp"

namespace {

using pt2q_chol::NB;

// Diagonal-block factor (chol_diag.hpp) as a kernel of its own: the first block, and any block
// whose producing update did not run the fused factor.
__global__ __launch_bounds__(256) void chol_diag_kernel(float* A, long lda, int p0, int nb,
                                                        int* info, long bst) {
  __shared__ __attribute__((aligned(16))) float urow[3][pt2q_chol::DG][NB];
  A += (long)blockIdx.y * bst;  // batch item (grid.y)
  info += blockIdx.y;
  const float* D = A + (long)p0 * lda + p0;
  pt2q_chol::diag_factor([&](int r, int c) { return D[(long)r * lda + c]; }, A, lda, p0, nb, info, urow);
}

constexpr int LPR = 4;           // lanes cooperating on one panel column / inverse row

// Broadcast lane `owner` of each aligned group of 4 lanes (one DPP quad_perm move instead of a
// ds_bpermute round trip through LDS).  owner is a compile-time constant after unrolling.
template <int O>
PT2Q_DEV float quad_bcast_c(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), O * 0x55, 0xF, 0xF, false));
}
PT2Q_DEV float quad_bcast(float v, int owner) {
  return owner == 0 ? quad_bcast_c<0>(v)
                    : owner == 1 ? quad_bcast_c<1>(v) : owner == 2 ? quad_bcast_c<2>(v) : quad_bcast_c<3>(v);
}
constexpr int SEG = NB / LPR;    // entries owned per lane

// Loads the nb x nb diagonal block at (r0, r0) as its STRICT upper part Dus (zero on and below
// the diagonal) plus the diagonal dg (identity padding beyond nb: dg = 1, Dus = 0).  With the
// zeros in place the step loops below need no masks or branches: an fmaf with a zero factor is
// an exact no-op on every nonzero chain (only the sign of an exact zero can differ, which the
// contract treats as equal).  256 threads: all 16 loads of a thread are in flight together.
PT2Q_DEV void load_diag_block(float (*Dus)[NB + 4], float* dg, const float* A, long lda, int r0,
                              int nb) {
  constexpr int PER = NB * NB / 256;
  float v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = threadIdx.x + 256 * u, r = q / NB, c = q % NB;
    const bool in = r < nb && c < nb && r <= c;
    v[u] = A[in ? (long)(r0 + r) * lda + r0 + c : (long)r0 * lda + r0];
    v[u] = in ? v[u] : ((r == c) ? 1.0f : 0.0f);
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = threadIdx.x + 256 * u, r = q / NB, c = q % NB;
    Dus[r][c] = (c > r) ? v[u] : 0.0f;
    if (r == c) dg[r] = v[u];
  }
}

// Panel rows [p0, p0+nb) for columns i >= p0+nb: forward substitution against the factored
// diagonal block, continuing each element's chain from the already-updated A value.  Four
// lanes share a column (16 rows each); the lane owning row k divides and broadcasts x_k.
PT2Q_DEV void chol_panel_load(const float* A, long lda, int p0, int nb, int m, int bid, float (&x)[SEG]) {
  const int i = p0 + nb + (bid * (int)blockDim.x + (int)threadIdx.x) / LPR;
  const int sub = threadIdx.x & (LPR - 1);
  const bool valid = i < m;
#pragma unroll
  for (int s = 0; s < SEG; ++s) {
    int k = sub * SEG + s;
    const bool in = valid && k < nb;
    x[s] = A[in ? (long)(p0 + k) * lda + i : (long)p0 * lda + p0];  // branch-free loads
    x[s] = in ? x[s] : 0.0f;
  }
}

PT2Q_DEV void chol_panel(float* A, long lda, int p0, int nb, int m, int bid,
                         float (*Dus)[NB + 4], float* dg, float (&x)[SEG]) {
  const int i = p0 + nb + (bid * (int)blockDim.x + (int)threadIdx.x) / LPR;
  const int sub = threadIdx.x & (LPR - 1);
  const bool valid = i < m;
  // row k+1 of the diagonal block and dg[k+1] are read during step k (software pipeline: the
  // LDS latency stays off the divide -> broadcast -> fma chain)
  float cur[SEG], nxt[SEG];
  float dcur = dg[0], dnxt = 0.0f;
#pragma unroll
  for (int s = 0; s < SEG; ++s) cur[s] = Dus[0][sub * SEG + s];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int owner = k / SEG, ks = k % SEG;
    if (k + 1 < NB) {
#pragma unroll
      for (int s = 0; s < SEG; ++s) nxt[s] = Dus[k + 1][sub * SEG + s];
      dnxt = dg[k + 1];
    }
    const float xk = quad_bcast(x[ks] / dcur, owner);
    x[ks] = (sub == owner) ? xk : x[ks];
#pragma unroll
    for (int s = 0; s < SEG; ++s) x[s] = fmaf(-cur[s], xk, x[s]);
#pragma unroll
    for (int s = 0; s < SEG; ++s) cur[s] = nxt[s];
    dcur = dnxt;
  }
  if (!valid) return;
#pragma unroll
  for (int s = 0; s < SEG; ++s) {
    int k = sub * SEG + s;
    if (k < nb) A[(long)(p0 + k) * lda + i] = x[s];
  }
}

// In-block part of the triangular inverse for column block [c0, c0+nb): rows k < c0+nb.
// The inverse is kept TRANSPOSED, UiT[i][k] = Uinv[k][i] (lower triangular), so that every
// product that reads it has K-major operands (gemmx.hip).  UiT[c0..][k] holds the running chains
// for k < c0 (zero otherwise).  Four lanes share a row k of Uinv.
// For rows inside the block, columns left of the diagonal start at zero and only ever receive
// zero terms, so they need no mask until the final store.
PT2Q_DEV void trtri_load(const float* UiT, long ldi, int c0, int nb, int bid, float (&acc)[SEG]) {
  const int k = (bid * (int)blockDim.x + (int)threadIdx.x) / LPR;
  const int sub = threadIdx.x & (LPR - 1);
  const bool valid = k < c0 + nb;
#pragma unroll
  for (int s = 0; s < SEG; ++s) {
    int q = sub * SEG + s;
    const bool in = valid && k < c0 && q < nb;
    acc[s] = UiT[in ? (long)(c0 + q) * ldi + k : 0];  // branch-free loads; Uinv[k][c0+q]
    acc[s] = in ? acc[s] : 0.0f;
  }
}

PT2Q_DEV void trtri_inblock(float* Ui, long ldi, int c0, int nb, int bid, float (*Dus)[NB + 4],
                            float* dg, float (&acc)[SEG]) {
  const int k = (bid * (int)blockDim.x + (int)threadIdx.x) / LPR;
  const int sub = threadIdx.x & (LPR - 1);
  const bool valid = k < c0 + nb;
  const int jb = (k > c0) ? k - c0 : 0;  // first in-block j (local)
  float cur[SEG], nxt[SEG];  // software-pipelined rows, as in chol_panel
  float dcur = dg[0], dnxt = 0.0f;
#pragma unroll
  for (int s = 0; s < SEG; ++s) cur[s] = Dus[0][sub * SEG + s];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int owner = j / SEG, js = j % SEG;
    if (j + 1 < NB) {
#pragma unroll
      for (int s = 0; s < SEG; ++s) nxt[s] = Dus[j + 1][sub * SEG + s];
      dnxt = dg[j + 1];
    }
    const float mine = (c0 + j == k) ? 1.0f / dcur : -acc[js] / dcur;
    const float xj = quad_bcast(mine, owner);
    acc[js] = (sub == owner) ? xj : acc[js];
#pragma unroll
    for (int s = 0; s < SEG; ++s) acc[s] = fmaf(xj, cur[s], acc[s]);
#pragma unroll
    for (int s = 0; s < SEG; ++s) cur[s] = nxt[s];
    dcur = dnxt;
  }
  if (!valid) return;
#pragma unroll
  for (int s = 0; s < SEG; ++s) {
    int q = sub * SEG + s;
    if (q < nb) Ui[(long)(c0 + q) * ldi + k] = (q >= jb) ? acc[s] : 0.0f;  // UiT[c0+q][k]
  }
}

// Block J after its diagonal factor: workgroups [0, npanel) solve the panel (rows of block J
// right of it), the rest run the in-block triangular inverse of block J (which needs only the
// factored diagonal block and the inverse chains of earlier blocks) -- one launch.
__global__ __launch_bounds__(256) void chol_panel_trtri_kernel(float* U, long ld, int p0, int nb,
                                                               int m, float* Ui, int npanel, long bst) {
  __shared__ __attribute__((aligned(16))) float Dus[NB][NB + 4];
  __shared__ float dg[NB];
  U += (long)blockIdx.y * bst;  // batch item (grid.y)
  Ui += (long)blockIdx.y * bst;
  const bool panel = (int)blockIdx.x < npanel;
  float x[SEG];  // this thread's chains, loaded together with the diagonal block
  if (panel)
    chol_panel_load(U, ld, p0, nb, m, blockIdx.x, x);
  else
    trtri_load(Ui, ld, p0, nb, blockIdx.x - npanel, x);
  load_diag_block(Dus, dg, U, ld, p0, nb);
  __syncthreads();
  if (panel)
    chol_panel(U, ld, p0, nb, m, blockIdx.x, Dus, dg, x);
  else
    trtri_inblock(Ui, ld, p0, nb, blockIdx.x - npanel, Dus, dg, x);
}

// The same block step with one lane per panel column / inverse row (whole 64-row blocks only):
// the lane keeps all 64 chains in registers, so it needs no broadcast and no padded zero terms.
// The factored diagonal block is staged in LDS once per workgroup; every lane of a wave reads the
// same U[k][j] (ds_read_b128 broadcasts, four entries per read).  Each chain takes exactly the
// terms of the kernel above in the same order (that kernel's extra terms are zero factors, exact
// no-ops), so the bits are equal.  Packed FMAs update two chains per instruction.
typedef float f32x2 __attribute__((ext_vector_type(2)));

typedef float f32x4 __attribute__((ext_vector_type(4)));
#include "chol_lane.inc"  // lane_stream_panel / lane_stream_inverse (tools/gen_chol_lane.py)

PT2Q_DEV void lane_stage_block(float (*Ds)[NB], const float* U, long ld, int p0) {
  const float* D = U + (long)p0 * ld + p0;
#pragma unroll
  for (int u = 0; u < NB * NB / 4 / 256; ++u) {
    const int q = (int)threadIdx.x + 256 * u, r = q / (NB / 4), c4 = q % (NB / 4);
    *(float4*)&Ds[r][4 * c4] = *(const float4*)(D + (long)r * ld + 4 * c4);
  }
}

PT2Q_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// panel column i = p0 + NB + t
PT2Q_DEV void lane_panel(float* U, long ld, int p0, int m, int t, float (*Ds)[NB]) {
  const int i = p0 + NB + t;
  const bool valid = i < m;
  const float* col = U + (long)p0 * ld + (valid ? i : p0);
  f32x2 xp[NB / 2];
#pragma unroll
  for (int r = 0; r < NB / 2; ++r) xp[r] = f32x2{col[(long)(2 * r) * ld], col[(long)(2 * r + 1) * ld]};
  lane_stage_block(Ds, U, ld, p0);  // (the chains' loads in flight meanwhile)
  __syncthreads();
  lane_stream_panel(xp, lds_addr(&Ds[0][0]));
  if (!valid) return;
#pragma unroll
  for (int r = 0; r < NB / 2; ++r) {
    U[(long)(p0 + 2 * r) * ld + i] = xp[r].x;
    U[(long)(p0 + 2 * r + 1) * ld + i] = xp[r].y;
  }
}

// inverse row k: UiT[p0 + q][k] = Uinv[k][p0 + q], earlier blocks' chains for k < p0, zero otherwise
PT2Q_DEV void lane_inverse(const float* U, float* Ui, long ld, int p0, int k, float (*Ds)[NB]) {
  const bool prior = k < p0;
  const float* row = Ui + (long)p0 * ld + (prior ? k : 0);
  f32x2 xp[NB / 2];
#pragma unroll
  for (int q = 0; q < NB / 2; ++q) {
    const float a = row[(long)(2 * q) * ld], b = row[(long)(2 * q + 1) * ld];  // branch-free loads
    xp[q] = prior ? f32x2{a, b} : f32x2{0.0f, 0.0f};
  }
  lane_stage_block(Ds, U, ld, p0);
  __syncthreads();
  const int kl = k - p0;  // the row's own diagonal step (none for k < p0)
  lane_stream_inverse(xp, lds_addr(&Ds[0][0]), kl);
  if (k >= p0 + NB) return;
  const int jb = kl > 0 ? kl : 0;
#pragma unroll
  for (int q = 0; q < NB / 2; ++q) {
    Ui[(long)(p0 + 2 * q) * ld + k] = (2 * q >= jb) ? xp[q].x : 0.0f;  // UiT[p0+q][k]
    Ui[(long)(p0 + 2 * q + 1) * ld + k] = (2 * q + 1 >= jb) ? xp[q].y : 0.0f;
  }
}

// 256-thread workgroups: [0, npanel) one panel column per lane (columns p0 + NB + ...), the rest
// one row k < p0 + NB of the inverse per lane.
__global__ __launch_bounds__(256) void chol_panel_trtri_lane_kernel(float* U, long ld, int p0, int m, float* Ui,
                                                                    int npanel, long bst) {
  __shared__ __attribute__((aligned(16))) float Ds[NB][NB];
  U += (long)blockIdx.y * bst;  // batch item (grid.y)
  Ui += (long)blockIdx.y * bst;
  if ((int)blockIdx.x < npanel)
    lane_panel(U, ld, p0, m, (int)blockIdx.x * 256 + (int)threadIdx.x, Ds);
  else
    lane_inverse(U, Ui, ld, p0, ((int)blockIdx.x - npanel) * 256 + (int)threadIdx.x, Ds);
}

__global__ void copy_upper_kernel(const float* H, long ldh, float* A, long lda, int m, long bst) {
  H += (long)blockIdx.y * bst;  // batch item (grid.y)
  A += (long)blockIdx.y * bst;
  long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)m * m) return;
  int r = (int)(q / m), c = (int)(q % m);
  A[(long)r * lda + c] = (c >= r) ? H[(long)r * ldh + c] : 0.0f;
}

}  // namespace

namespace {

// U[r0.., c0..] (rows x cols) -= U[p0 + k][r0 + i] * U[p0 + k][c0 + j] over the nb rows from p0
// (one or two blocks; chains continue from U, k ascending).  upper: the square trailing
// triangle; otherwise the full rectangle (the strictly-lower part of U is scratch).
GemmDesc trailing_desc(float* U, long ld, int p0, int nb, int r0, int rows, int c0, int cols,
                       bool upper = true, int batch = 1) {
  GemmDesc g{};
  g.batch = batch; g.bstride = ld * ld;
  g.M = rows; g.N = cols; g.K = nb;
  g.A = U + (long)p0 * ld + r0; g.lda = ld; g.a_layout = LAY_KMAJOR;
  g.B = U + (long)p0 * ld + c0; g.ldb = ld; g.b_layout = LAY_KMAJOR;
  g.in_dtype = PT2Q_F32;
  g.C = U + (long)r0 * ld + c0; g.ldc = ld;
  g.mode = GEMM_CHAIN_NEG; g.upper = upper ? 1 : 0; g.mirror = 0;
  return g;
}

// Inverse chains of columns [c1, c1 + cols) (rows of UiT), over rows k < nk of Uinv, get the terms
// j in [j0, j0 + K) (ascending):  UiT[c][k] += sum_j U[j][c] * UiT[j][k].
GemmDesc trtri_desc(const float* U, float* UiT, long ld, int j0, int K, int c1, int cols, int nk,
                    int batch = 1) {
  GemmDesc g{};
  g.batch = batch; g.bstride = ld * ld;
  g.M = cols; g.N = nk; g.K = K;
  g.A = U + (long)j0 * ld + c1; g.lda = ld; g.a_layout = LAY_KMAJOR;   // (c, j) = U[j0+j][c1+c]
  g.B = UiT + (long)j0 * ld; g.ldb = ld; g.b_layout = LAY_KMAJOR;      // (j, k) = UiT[j0+j][k]
  g.in_dtype = PT2Q_F32;
  g.C = UiT + (long)c1 * ld; g.ldc = ld;
  g.mode = GEMM_CHAIN_POS;
  return g;
}

// Large chain GEMMs (panel-wide updates, lauum): the LDS-DMA kernel where it applies and pays.
int launch_big(const GemmDesc& g, hipStream_t st) {
  const long tiles = (long)ceil_div(g.M, 128) * ceil_div(g.N, 128) / (g.upper ? 2 : 1) * (g.batch > 1 ? g.batch : 1);
  if (tiles >= 64 && g.K >= 128) {
    const int rc = pt2q_launch_gemmx(g, st);
    if (rc != PT2Q_E_UNSUPPORTED) return rc;
  }
  return pt2q_launch_gemm(g, st);
}

}  // namespace

// The side stream of the look-ahead below and its two events, `fork` (main -> side) and `join`
// (side -> main): one set per (device, caller stream), created on first use, so concurrent
// callers on different streams (UnitPipeline lanes, host threads) neither serialise their side
// work behind each other nor share events.  Under hipGraph capture the event wait pulls the side
// stream into the capture and the final join brings it back.
struct CholSide {
  hipStream_t st = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

int chol_side(hipStream_t caller, CholSide*& out) {
  static std::map<std::pair<int, hipStream_t>, CholSide> sides;
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return PT2Q_E_HIP;
  std::lock_guard<std::mutex> lock(mu);
  CholSide& c = sides[{dev, caller}];  // std::map: references stay valid as entries are added
  if (!c.st) {
    int lo = 0, hi = 0;  // the side stream yields to the critical path: the lowest priority
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c.st, hipStreamNonBlocking, lo) != hipSuccess ||
        hipEventCreateWithFlags(&c.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c.join, hipEventDisableTiming) != hipSuccess)
      return PT2Q_E_HIP;
  }
  out = &c;
  return PT2Q_OK;
}

// Main stream: per 64-wide block J a panel solve + in-block triangular inverse launch and a strip
// update launch (which also factors the next diagonal block); per 512- or 1024-row panel P the
// rank-CP terms of P go first to the NEXT panel's rows (main stream, on the critical path), and
// to every row beyond it on a side stream, where they overlap the factorisation of panel P+1
// (which touches only its own rows of U and of the inverse).  Before panel P+1's terms reach
// those rows, the main stream joins the side stream, so every chain still takes panel P's terms
// before panel P+1's: the order, and every bit, are those of the one-stream schedule.  The
// inverse (kept transposed, UiT) is built right-looking by column blocks as soon as rows of
// block J are final.
int pt2q_launch_cholesky_inverse(const float* H, long ldh, int m, float* Hinv, long ldhi,
                                 float* U, float* Ui, int* info, hipStream_t st, bool h_upper_form,
                                 int batch) {
  const long ld = m;  // U and Ui are packed m x m
  const long bst = ld * ld;  // batch item stride of every matrix (batch > 1: all packed)
  if (batch < 1 || (batch > 1 && (ldh != ld || ldhi != ld))) return PT2Q_E_ARG;
  if (hipMemsetAsync(info, 0, sizeof(int) * batch, st) != hipSuccess) return PT2Q_E_HIP;
  if (hipMemsetAsync(Ui, 0, sizeof(float) * (size_t)m * m * batch, st) != hipSuccess) return PT2Q_E_HIP;
  if (!(h_upper_form && H == U && ldh == ld)) {  // (else H already is the upper work matrix)
    hipLaunchKernelGGL(copy_upper_kernel, dim3(ceil_div((long)m * m, 256), batch), dim3(256), 0, st, H, ldh,
                       U, ld, m, bst);
    PT2Q_LAUNCH_CHECK();
  }
  int rc;
  const Pt2qTuning& tu = pt2q_tuning();
  // panel solve + in-block inverse of the block at p0 (its diagonal factor done: `factored`)
  auto factor = [&](int p0, int nb, bool factored) -> int {
    if (!factored) {
      hipLaunchKernelGGL(chol_diag_kernel, dim3(1, batch), dim3(256), 0, st, U, ld, p0, nb, info, bst);
      PT2Q_LAUNCH_CHECK();
    }
    const int rest = m - p0 - nb;
    if (nb == NB && tu.chol_lane) {  // whole blocks: one lane per column / row
      const int npanel = rest > 0 ? (int)ceil_div((long)rest, 256) : 0;
      const int ninv = (int)ceil_div((long)(p0 + nb), 256);
      hipLaunchKernelGGL(chol_panel_trtri_lane_kernel, dim3(npanel + ninv, batch), dim3(256), 0, st, U, ld, p0, m,
                         Ui, npanel, bst);
      PT2Q_LAUNCH_CHECK();
      return PT2Q_OK;
    }
    const int npanel = rest > 0 ? (int)ceil_div((long)rest * LPR, 256) : 0;
    const int ninv = (int)ceil_div((long)(p0 + nb) * LPR, 256);
    hipLaunchKernelGGL(chol_panel_trtri_kernel, dim3(npanel + ninv, batch), dim3(256), 0, st, U, ld, p0, nb,
                       m, Ui, npanel, bst);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  };
  // Panels of CP rows: inside a panel, 64-blocks right-looking restricted to the panel (the
  // block's rows of U solved across the full width; the panel's later rows of U and later
  // columns of the inverse get the block's terms by rank-64 strip updates, whose first tile is
  // the next diagonal block, factored in the same launch); after the panel, its rank-CP terms
  // (gemmx) as described above.  Every chain takes its terms in ascending k.
  const int tp = tu.chol_panel;
  // look-ahead from m > 6144 (measured: 4096 3.07 -> 3.24 ms with it, 11008 19.7 -> 18.6 ms with
  // it and 512-row panels); panel rows (a multiple of NB): 512, or 1024 for a large m alone
  // (a batch fills the chip by itself: no look-ahead)
  const bool ahead = tu.chol_lookahead && m > 6144 && batch == 1;
  const int CP = tp >= NB ? tp / NB * NB : (m > 6144 && !ahead ? 1024 : 512);
  CholSide* side = nullptr;
  if (ahead && m > CP + CP && (rc = chol_side(st, side)) != PT2Q_OK) return rc;
  bool factored = false, pending = false;  // pending: side-stream terms not yet joined
  auto join = [&]() -> int {
    if (pending && hipStreamWaitEvent(st, side->join, 0) != hipSuccess) return PT2Q_E_HIP;
    pending = false;
    return PT2Q_OK;
  };
  // sub-panels of SP rows (a multiple of NB dividing CP): a block's rank-64 strip update reaches
  // only the rows of its sub-panel; the rest of the panel takes the sub-panel's terms as one
  // rank-SP chain GEMM once the sub-panel is done -- the same terms in the same ascending order
  // (inverse columns of later sub-panels get the zero terms of rows below their diagonal, exact
  // no-ops), with a quarter of the strip updates' read-modify-write traffic at SP = CP / 4.
  const int SPt = tu.chol_subpanel >= NB ? tu.chol_subpanel / NB * NB : CP;
  const int SP = (SPt < CP && CP % SPt == 0) ? SPt : CP;
  for (int P0 = 0; P0 < m; P0 += CP) {
    const int Pend = (m - P0 < CP) ? m : P0 + CP;
    for (int Q0 = P0; Q0 < Pend; Q0 += SP) {
      const int Qend = (Pend - Q0 < SP) ? Pend : Q0 + SP;
      for (int p0 = Q0; p0 < Qend; p0 += NB) {
        const int nb = (Qend - p0 < NB) ? Qend - p0 : NB;
        if ((rc = factor(p0, nb, factored)) != PT2Q_OK) return rc;
        factored = false;
        const int p1 = p0 + nb;
        if (p1 >= Qend) break;
        const int nb1 = (Qend - p1 < NB) ? Qend - p1 : NB;
        // U rows [p1, Qend) x columns [p1, m) and inverse columns [p1, Qend) x rows [0, p1)
        if ((rc = pt2q_launch_gemm2(trailing_desc(U, ld, p0, nb, p1, Qend - p1, p1, m - p1, false, batch),
                                    trtri_desc(U, Ui, ld, p0, nb, p1, Qend - p1, p1, batch), st, U, ld, p1,
                                    nb1, info, &factored)) != PT2Q_OK)
          return rc;
      }
      if (Qend >= Pend) break;
      // the sub-panel's terms: U rows [Qend, Pend) x columns [Qend, m), inverse columns
      // [Qend, Pend) x rows [0, Qend)
      const int K = Qend - Q0;
      if ((rc = launch_big(trailing_desc(U, ld, Q0, K, Qend, Pend - Qend, Qend, m - Qend, false, batch), st)) !=
          PT2Q_OK)
        return rc;
      if ((rc = launch_big(trtri_desc(U, Ui, ld, Q0, K, Qend, Pend - Qend, Qend, batch), st)) != PT2Q_OK) return rc;
    }
    if (Pend >= m) break;
    const int K = Pend - P0, rest = m - Pend;
    // rows the side stream still owes earlier panels' terms must have them first
    if ((rc = join()) != PT2Q_OK) return rc;
    // the next panel's rows [Pend, Pend2) -- or all remaining rows without a side stream
    const int Pend2 = side ? std::min(m, Pend + CP) : m;
    if ((rc = launch_big(trailing_desc(U, ld, P0, K, Pend, Pend2 - Pend, Pend, rest, Pend2 < m ? false : true,
                                       batch), st)) != PT2Q_OK)
      return rc;
    if ((rc = launch_big(trtri_desc(U, Ui, ld, P0, K, Pend, Pend2 - Pend, Pend, batch), st)) != PT2Q_OK) return rc;
    if (Pend2 < m) {  // every row beyond, on the side stream
      if (hipEventRecord(side->fork, st) != hipSuccess || hipStreamWaitEvent(side->st, side->fork, 0) != hipSuccess)
        return PT2Q_E_HIP;
      if ((rc = launch_big(trailing_desc(U, ld, P0, K, Pend2, m - Pend2, Pend2, m - Pend2), side->st)) != PT2Q_OK)
        return rc;
      if ((rc = launch_big(trtri_desc(U, Ui, ld, P0, K, Pend2, m - Pend2, Pend), side->st)) != PT2Q_OK) return rc;
      if (hipEventRecord(side->join, side->st) != hipSuccess) return PT2Q_E_HIP;
      pending = true;
    }
  }
  if ((rc = join()) != PT2Q_OK) return rc;
  // Hinv = Uinv Uinvᵀ (upper tiles, mirrored): Hinv[i][k] = chain over j >= max(i, k) of
  // UiT[j][i] * UiT[j][k]
  GemmDesc g{};
  g.M = m; g.N = m; g.K = m;
  g.A = Ui; g.lda = ld; g.a_layout = LAY_KMAJOR;   // (i, j) = UiT[j][i]
  g.B = Ui; g.ldb = ld; g.b_layout = LAY_KMAJOR;   // (j, k) = UiT[j][k]
  g.in_dtype = PT2Q_F32;
  g.C = Hinv; g.ldc = ldhi;
  g.mode = GEMM_STORE; g.upper = 1; g.mirror = 1; g.kstart_diag = 2;
  g.batch = batch; g.bstride = bst;
  return launch_big(g, st);
}
