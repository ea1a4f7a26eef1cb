// Exported C ABI of libpt2q (include/pt2q.h): argument checks, workspace carving and the
// per-layer launch schedule.  All launches are stream-ordered; nothing here synchronises or
// allocates, so a caller may capture a whole layer into a hipGraph.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>
#include <climits>

#include "common.hpp"
#include "internal.hpp"

namespace {

// Tuning, read once at library load -- see Pt2qTuning.  Release builds read only the debug
// spin cap; every kernel-selecting variable is a development-build (PT2Q_DEV_PROBES) override.
Pt2qTuning load_tuning() {
  Pt2qTuning t;
#ifdef PT2Q_DEV_PROBES
  auto geti = [](const char* k, int& v) {
    if (const char* e = std::getenv(k)) v = std::atoi(e);
  };
  auto getb = [](const char* k, bool& v) {
    if (const char* e = std::getenv(k)) v = e[0] != '0';
  };
  // Kernel-selecting overrides and knock-outs: read only by a development build (make
  // DEV_PROBES=1, tools/build_dev_lib.sh).  The release library runs the defaults of Pt2qTuning
  // whatever the environment holds, so no variable can switch it onto a kernel variant the GPU
  // tests do not cover (or onto a knock-out whose results are garbage).
  geti("PT2Q_GRAM_SUPER", t.gram_super);
  geti("PT2Q_GRAM_GROUPS", t.gram_groups);
  geti("PT2Q_GRAM_CUS", t.gram_cus);
  getb("PT2Q_GRAM_STREAMK", t.gram_split);
  getb("PT2Q_GRAM_PAIR", t.gram_pair);
  getb("PT2Q_GRAM_DP", t.gram_dp);
  getb("PT2Q_GRAM_WIDE", t.gram_wide);
  geti("PT2Q_GRAM_SEGLEN", t.gram_seglen);
  geti("PT2Q_GEMM_TILE", t.gemm_tile);
  getb("PT2Q_RANK_UPDATE", t.rank_update);
  geti("PT2Q_CHOL_PANEL", t.chol_panel);
  geti("PT2Q_CHOL_SUBPANEL", t.chol_subpanel);
  getb("PT2Q_CHOL_LOOKAHEAD", t.chol_lookahead);
  getb("PT2Q_WBAR_FUSED", t.wbar_fused);
  getb("PT2Q_SIM_SPLIT", t.sim_split);
  getb("PT2Q_EF_WBAR", t.ef_wbar);
  geti("PT2Q_GEMMX_STAGES", t.gemmx_stages);
  getb("PT2Q_GEMMX_GRAM", t.gemmx_gram);
  getb("PT2Q_CHOL_LANE", t.chol_lane);
  getb("PT2Q_S1_IN_ATQ", t.s1_in_atq);
  getb("PT2Q_EF_GEMM", t.ef_kernel);
  geti("PT2Q_WIDE_WAVES", t.wide_waves);
  geti("PT2Q_ATQ_OCC", t.atq_occ);
  getb("PT2Q_ATQ_VEC", t.atq_vec);
  getb("PT2Q_GRAM_ORDER", t.gram_order);
  getb("PT2Q_ATQ_PC", t.atq_pc);
  getb("PT2Q_ATQ_PC_REGS", t.atq_pc_regs);
  geti("PT2Q_EF_V2", t.ef_v2);
  // knock-outs (tools/ef2_knock.sh, tools/atq_knock.sh; results garbage)
  geti("PT2Q_EF2_PROBE", t.ef2_probe);
  geti("PT2Q_ATQ_PROBE", t.atq_probe);
  geti("PT2Q_EF2_STAGGER", t.ef2_stagger);
  geti("PT2Q_EF2_PER_CU", t.ef2_per_cu);
  geti("PT2Q_EF2_TEAMS", t.ef2_teams);
  geti("PT2Q_EF2_TEAM_OFFSET", t.ef2_team_offset);
  getb("PT2Q_EF2_G1LDS", t.ef2_g1lds);
  if (t.ef2_per_cu != 1) t.ef2_per_cu = 2;
  if (t.wide_waves != 8) t.wide_waves = 4;
  if (t.atq_occ != 0) t.atq_occ = 6;
#endif
  // release and development: the stall-reporting test hook (tests/test_gpu_status.py)
  if (const char* e = std::getenv("PT2Q_DEBUG_SPIN_CAP")) {
    const long c = std::atol(e);
    if (c >= 0) t.spin_cap_long = t.spin_cap_short = t.spin_cap_fallback = c;
  }
  return t;
}

}  // namespace

const Pt2qTuning& pt2q_tuning() {
  static const Pt2qTuning t = load_tuning();
  return t;
}

namespace {

const Pt2qTuning& g_tuning_at_load = pt2q_tuning();  // forces the read at dlopen

struct Carve {
  char* p;
  size_t left;
  bool ok = true;
  bool dry = false;  // count only (used bytes in `used`)
  size_t used = 0;
  template <typename T>
  T* take(size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~(size_t)255;
    used += bytes;
    if (dry) return nullptr;
    if (!p || bytes > left) {
      ok = false;
      return nullptr;
    }
    T* r = (T*)p;
    p += bytes;
    left -= bytes;
    return r;
  }
};

inline long round_up(long a, long b) { return (a + b - 1) / b * b; }

// ---- stage timing (measurement only, pt2q_stage_timing): while enabled, the launches of each
// block-loop stage are bracketed by a pair of HIP events on their stream.  One host thread, no
// graph capture; read back after the stream has drained.
struct StageRec {
  int stage;
  hipEvent_t a, b;
};
struct StageLog {
  bool on = false;
  std::vector<StageRec> recs;
  std::vector<hipEvent_t> pool;
  size_t next = 0;
  hipEvent_t take() {
    if (next == pool.size()) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[next++];
  }
};
StageLog& stage_log() {
  static StageLog l;
  return l;
}
struct StageScope {
  int stage;
  hipStream_t st;
  hipEvent_t a = nullptr;
  StageScope(int s, hipStream_t stream) : stage(s), st(stream) {
    StageLog& l = stage_log();
    if (l.on && (a = l.take()) && hipEventRecord(a, st) != hipSuccess) a = nullptr;
  }
  void close() {
    if (!a) return;
    StageLog& l = stage_log();
    hipEvent_t b = l.take();
    if (b && hipEventRecord(b, st) == hipSuccess) l.recs.push_back({stage, a, b});
    a = nullptr;
  }
  ~StageScope() { close(); }
};

struct BlockWs {
  int* status;  // the call's status word (stall reports)
  float* Wt;
  int8_t* Tt;
  float* Et;
  float* Ck;
  float* alpha_t;
  float* mu_t;
  float* S1;
  float* d;
  float* ssr;
  int* rem[2];
  int* blk;
  int* counters;
  int* iters;
  int* iters_part;
  float* hb;  // variant G, blocks > 128: the gathered H[blk][blk] and S = H_bbᵀH_bb (bb x bb)
  float* hS;
  long ldw;
};

// Whether the error feedback may hand the next block's SSR its w-bar partials (ef.hip / ssr.hip
// pre path: the fused w-bar launch's conditions; PT2Q_EF_WBAR=0 keeps the separate pass).
inline bool ef_wbar_ok(int n, long ldw, const float* Wt) {
  const Pt2qTuning& t = pt2q_tuning();
  return t.ef_wbar && t.wbar_fused && t.ef_kernel && n <= 16384 && n % 4 == 0 && ldw % 4 == 0 &&
         (uintptr_t)Wt % 16 == 0;
}

// variant G's AGA matrix for blocks wider than one workgroup's LDS holds (> 128 columns)
inline bool hess_wide(int flags, int bb) { return (flags & PT2Q_AGA_MASK) == PT2Q_AGA_HESS && bb > 128; }

bool carve_blocks(Carve& c, int n, int m, int b, BlockWs& w, int flags = 0) {
  const long ldw = round_up(n, 64);
  const int bb = b < m ? b : m;
  const int B = b < m ? ceil_div(m, b) : 1;
  w.ldw = ldw;
  w.Wt = c.take<float>((size_t)m * ldw);
  w.Tt = c.take<int8_t>((size_t)m * ldw);
  // E and the feedback coefficients exist only when a block leaves columns behind (B > 1)
  w.Et = c.take<float>(B > 1 ? (size_t)bb * ldw : 1);
  w.Ck = c.take<float>(B > 1 ? (size_t)bb * m : 1);
  w.alpha_t = c.take<float>((size_t)B * n);
  w.mu_t = c.take<float>((size_t)B * n);
  w.S1 = c.take<float>((size_t)bb);
  w.d = c.take<float>(1);
  w.ssr = c.take<float>(pt2q_ssr_scratch_floats(n, m));
  w.rem[0] = c.take<int>((size_t)m);
  w.rem[1] = c.take<int>((size_t)m);
  w.blk = c.take<int>((size_t)bb);
  // [2k, 2k+1] ATQ; [2B+2k, 2B+2k+1] top-k/S1 sync; [4B ..) the wbar hand-off counters
  w.counters = c.take<int>((size_t)4 * B + pt2q_ssr_counter_ints(n));
  w.iters = c.take<int>((size_t)B);
  w.iters_part = c.take<int>((size_t)ceil_div(n, 16) * 4);  // one per ATQ wave (4 waves of 4 rows per workgroup)
  w.hb = w.hS = nullptr;
  if (hess_wide(flags, bb)) {
    w.hb = c.take<float>((size_t)bb * bb);
    w.hS = c.take<float>((size_t)bb * bb);
  }
  return c.ok;
}

size_t blocks_bytes(int n, int m, int b, int flags = 0) {  // a dry run of carve_blocks
  Carve c{nullptr, 0};
  c.dry = true;
  BlockWs w;
  carve_blocks(c, n, m, b, w, flags);
  return c.used;
}

// hb[t][j] = A[blk[t]][blk[j]] (bs x bs, ld bs): variant G's X_block = H[blk][:, blk] (gptq.py:147)
__global__ void gather_block_kernel(const float* A, long lda, const int* blk, int bs, float* hb) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, t = blockIdx.y;
  if (j < bs) hb[(long)t * bs + j] = A[(long)blk[t] * lda + blk[j]];
}

// S1 = (H_bbᵀH_bb)·1, d = 1ᵀS1 for blocks > 128 columns (quantizer.py:202-218 with X = H_bb):
// S on the f32 MFMA GEMM (t-ascending fmaf chains, as aga_s1_kernel's src 2), then the row sums
// in l order and d in j order (pt2q_launch_aga_s1 src 1 on S itself).
int hess_block_s1(const float* A, long lda, const int* blk, int bs, BlockWs& w, hipStream_t st) {
  hipLaunchKernelGGL(gather_block_kernel, dim3(ceil_div(bs, 256), bs), dim3(256), 0, st, A, lda, blk, bs, w.hb);
  PT2Q_LAUNCH_CHECK();
  GemmDesc g{};
  g.M = bs; g.N = bs; g.K = bs;
  g.A = w.hb; g.lda = bs; g.a_layout = LAY_KMAJOR;  // (j, t) = hb[t][j]
  g.B = w.hb; g.ldb = bs; g.b_layout = LAY_KMAJOR;  // (t, l) = hb[t][l]
  g.in_dtype = PT2Q_F32;
  g.C = w.hS; g.ldc = bs;
  g.mode = GEMM_STORE;
  int rc = pt2q_launch_gemm(g, st);
  if (rc != PT2Q_OK) return rc;
  return pt2q_launch_aga_s1(1, w.hS, bs, nullptr, bs, w.S1, w.d, st);
}

// per-channel setup in one launch: perm = [0, m) (the block is every column in ascending order),
// the wide ATQ's counters (2 ints) and the iteration count zeroed -- instead of two memsets and a
// select_seq launch per linear
__global__ void pc_setup_kernel(int64_t* perm, int m, int* counters, int* iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) perm[i] = i;
  if (i < 2) counters[i] = 0;
  if (i == 0) *iters = 0;
}

// the grouped per-channel setup (pc_setup_kernel per linear z = blockIdx.y)
struct PcSetupGroup {
  int64_t* perm[PT2Q_PC_GROUP_MAX];
  int* counters[PT2Q_PC_GROUP_MAX];
  int* iters[PT2Q_PC_GROUP_MAX];
};
__global__ void pc_setup_group_kernel(PcSetupGroup g, int m) {
  const int z = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) g.perm[z][i] = i;
  if (i < 2) g.counters[z][i] = 0;
  if (i == 0) *g.iters[z] = 0;
}

__global__ void i64_to_i32_kernel(const int64_t* a, int n, int* b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (int)a[i];
}
__global__ void i32_to_i64_kernel(const int* a, int n, int64_t* b) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

int run_blocks(const void* W, int wdtype, long ldw_in, int n, int m, int b, int flags,
               const float* A, long lda, const float* Hinv, long ldhi, int max_iter, float* alpha,
               float* mu, void* T, int tdtype, int64_t* perm, int* iters_dev, BlockWs& w,
               hipStream_t st) {
  int rc;
  const int B = b < m ? ceil_div(m, b) : 1;
  const bool ssr = (flags & PT2Q_FLAG_SSR) != 0;
  const int aga = flags & PT2Q_AGA_MASK;
  int* iters = iters_dev ? iters_dev : w.iters;
  if (B == 1 && m > 512 && aga != PT2Q_AGA_HESS) {
    // Per-channel (block_size >= m, main.py:176-189 with one block): the block is every column in
    // ascending order -- SSR over the whole remaining set returns it in rem order, and rem is
    // [0, m) -- so the wide ATQ reads the caller's row-major W in place (no feature-major copy, no
    // code transpose) and writes T, alpha, mu (n x 1) straight into the outputs.
    {
      StageScope ts(PT2Q_TIMER_SETUP, st);
      hipLaunchKernelGGL(pc_setup_kernel, dim3(ceil_div(m, 256)), dim3(256), 0, st, perm, m, w.counters, iters);
      PT2Q_LAUNCH_CHECK();
    }
    StageScope ts_atq(PT2Q_TIMER_ATQ, st);
    const bool act = aga == PT2Q_AGA_ACT;
    // S1 / d given (PT2Q_FLAG_S1_GIVEN: A = S1 then d, formed once per Gram) or formed here
    const bool given = act && (flags & PT2Q_FLAG_S1_GIVEN) != 0;
    if (act && !given && (rc = pt2q_launch_aga_s1(1, A, lda, nullptr, m, w.S1, w.d, st)) != PT2Q_OK) return rc;
    const float* S1 = given ? A : w.S1;
    const float* dv = given ? A + m : w.d;
    return pt2q_launch_atq_wide_rm(W, wdtype, ldw_in, n, m, act ? S1 : nullptr, dv, max_iter, alpha, mu, T,
                                   tdtype, m, iters, w.counters, st);
  }
  {
    StageScope ts(PT2Q_TIMER_SETUP, st);
    // W (n x m) -> Wt (m x ldw, fp32)
    if ((rc = pt2q_launch_transpose_to_f32(W, wdtype, ldw_in, n, m, w.Wt, w.ldw, st)) != PT2Q_OK)
      return rc;
    if (hipMemsetAsync(w.counters, 0, sizeof(int) * (4 * B + pt2q_ssr_counter_ints(n)), st) != hipSuccess)
      return PT2Q_E_HIP;
    if (hipMemsetAsync(iters, 0, sizeof(int) * B, st) != hipSuccess) return PT2Q_E_HIP;
    // rem0 = [0, m)
    if ((rc = pt2q_launch_select_seq(0, 0, 0, m, nullptr, w.blk, w.rem[0], nullptr, st)) != PT2Q_OK)
      return rc;
  }
  float* part = w.ssr;
  float* wn = part + (size_t)ceil_div(m, 128) * n;
  float* sim = wn + n;
  int processed = 0, r = m, cur = 0;
  bool pre = false;  // part holds rem's w-bar partials (from the previous block's error feedback)
  for (int k = 0; k < B; ++k) {
    const int bs = r < b ? r : b;
    const int nr = r - bs;
    int* rem = w.rem[cur];
    int* nrem = w.rem[cur ^ 1];
    // variant M with blocks <= 128: the ATQ launch also forms S1/d (no separate launch; off
    // the critical path of the rows, which need it only for their AGA)
    const bool s1_in_atq = aga == PT2Q_AGA_ACT && bs <= 128 && pt2q_tuning().s1_in_atq;
    const bool s1_in_topk = !s1_in_atq && ssr && r > b && aga == PT2Q_AGA_ACT && bs <= 128;
    StageScope ts_ssr(PT2Q_TIMER_SSR, st);
    if (ssr) {
      if (r > b) {
        if ((rc = pt2q_launch_ssr_similarity(w.Wt, w.ldw, n, rem, r, part, wn, sim, st, w.counters + 4 * B,
                                             nullptr, pre)) != PT2Q_OK)
          return rc;
        if ((rc = pt2q_launch_ssr_topk(sim, rem, r, b, w.blk, nrem, perm + processed, st,
                                       s1_in_topk ? A : nullptr, lda, w.S1, w.d,
                                       w.counters + 2 * B + 2 * k, w.status)) != PT2Q_OK)
          return rc;
      } else {
        if ((rc = pt2q_launch_select_seq(1, 0, bs, m, rem, w.blk, nrem, perm + processed, st)) != PT2Q_OK)
          return rc;
      }
    } else {
      if ((rc = pt2q_launch_select_seq(0, processed, bs, m, nullptr, w.blk, nrem, perm + processed, st)) != PT2Q_OK)
        return rc;
    }
    ts_ssr.close();
    StageScope ts_atq(PT2Q_TIMER_ATQ, st);
    const float* S1 = nullptr;
    if (aga == PT2Q_AGA_ACT || aga == PT2Q_AGA_HESS) {
      if (hess_wide(flags, bs)) {
        if ((rc = hess_block_s1(A, lda, w.blk, bs, w, st)) != PT2Q_OK) return rc;
      } else if (!s1_in_topk && !s1_in_atq &&
                 (rc = pt2q_launch_aga_s1(aga == PT2Q_AGA_ACT ? 1 : 2, A, lda, w.blk, bs, w.S1, w.d, st)) != PT2Q_OK) {
        return rc;
      }
      S1 = w.S1;
    }
    if ((rc = pt2q_launch_atq_block(w.Wt, w.ldw, n, w.blk, bs, S1, w.d, max_iter,
                                    w.alpha_t + (size_t)k * n, w.mu_t + (size_t)k * n, w.Tt, w.ldw,
                                    nr > 0 ? w.Et : nullptr, w.ldw, iters + k, w.counters + 2 * k,
                                    st, Hinv, ldhi, nrem, nr, w.Ck, m, w.iters_part,
                                    s1_in_atq ? A : nullptr, lda,
                                    s1_in_atq ? w.counters + 2 * B + 2 * k : nullptr, w.status)) != PT2Q_OK)
      return rc;  // (also forms the EF coefficients C[k][e] when nr > 0)
    ts_atq.close();
    StageScope ts_ef(PT2Q_TIMER_EF, st);
    const bool want = ssr && nr > b && ef_wbar_ok(n, w.ldw, w.Wt);  // the next block runs SSR over nrem
    rc = (nr > 0 && pt2q_tuning().ef_kernel)
             ? pt2q_launch_ef(w.Ck, m, w.Et, w.Wt, w.ldw, m, nrem, nr, bs, st, nullptr, want ? part : nullptr, n)
             : PT2Q_E_UNSUPPORTED;
    if (rc != PT2Q_OK && rc != PT2Q_E_UNSUPPORTED) return rc;
    pre = want && rc == PT2Q_OK;
    if (nr > 0 && rc == PT2Q_E_UNSUPPORTED) {
      GemmDesc g{};
      g.M = nr; g.N = n; g.K = bs;
      g.A = w.Ck; g.lda = m; g.a_layout = LAY_KMAJOR;     // (e, k) = C[k][e]
      g.B = w.Et; g.ldb = w.ldw; g.b_layout = LAY_KMAJOR; // (k, i) = E[k][i]
      g.in_dtype = PT2Q_F32;
      g.C = w.Wt; g.ldc = w.ldw; g.crow = nrem;
      g.mode = GEMM_SUB;
      if ((rc = pt2q_launch_gemm(g, st)) != PT2Q_OK) return rc;
    }
    processed += bs;
    r = nr;
    cur ^= 1;
  }
  // outputs: T (n x m) from Tt (m x ldw); alpha/mu (n x B) from (B x n)
  StageScope ts(PT2Q_TIMER_OUT, st);
  if ((rc = pt2q_launch_transpose_i8(w.Tt, w.ldw, m, n, T, tdtype, m, st)) != PT2Q_OK) return rc;
  if ((rc = pt2q_launch_transpose_f32(w.alpha_t, n, B, n, alpha, B, st)) != PT2Q_OK) return rc;
  if ((rc = pt2q_launch_transpose_f32(w.mu_t, n, B, n, mu, B, st)) != PT2Q_OK) return rc;
  return PT2Q_OK;
}

// ---- grouped block loops (pt2q_quantize_blocks_group): per-linear workspace slices of one size

// A linear's slice: the block-loop buffers plus its permutation (int64, written by the
// selection launches and copied out at the end).
size_t group_slice_bytes(int n, int m, int b, int flags) {
  return blocks_bytes(n, m, b, flags) + (((size_t)m * 8 + 255) & ~(size_t)255);
}

// Every linear's counters and ITF iteration slots zeroed, its remaining set = [0, m).
__global__ void group_init_kernel(int* counters, int ncnt, int* iters, int B, int* rem0, int m, long zs) {
  counters = zws(counters, zs);
  iters = zws(iters, zs);
  rem0 = zws(rem0, zs);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ncnt) counters[t] = 0;
  if (t < B) iters[t] = 0;
  if (t < m) rem0[t] = t;
}

int run_blocks_group(int count, const void* const* W, int wdtype, long ldw_in, int n, int m, int b,
                     int flags, const float* const* A, long lda, const float* const* Hinv, long ldhi,
                     int max_iter, float* const* alpha, float* const* mu, void* const* T, int tdtype,
                     int64_t* const* perm, int* const* iters_dev, BlockWs& w, int64_t* perm64,
                     long zs, hipStream_t st) {
  int rc;
  const int B = ceil_div(m, b);
  const bool ssr = (flags & PT2Q_FLAG_SSR) != 0;
  const bool act = (flags & PT2Q_AGA_MASK) == PT2Q_AGA_ACT;
  Grp g{};
  g.ws = zs;
  g.count = count;
  StageScope ts0(PT2Q_TIMER_SETUP, st);
  for (int z = 0; z < count; ++z) {
    g.G[z] = act ? A[z] : nullptr;
    g.Hinv[z] = Hinv[z];
    // W (n x m) -> Wt (m x ldw, fp32) of every linear
    if ((rc = pt2q_launch_transpose_to_f32(W[z], wdtype, ldw_in, n, m, (float*)((char*)w.Wt + z * zs), w.ldw,
                                           st)) != PT2Q_OK)
      return rc;
  }
  const int ncnt = 4 * B + pt2q_ssr_counter_ints(n);
  hipLaunchKernelGGL(group_init_kernel, dim3(ceil_div(std::max(std::max(ncnt, B), m), 256), 1, count), dim3(256),
                     0, st, w.counters, ncnt, w.iters, B, w.rem[0], m, zs);
  PT2Q_LAUNCH_CHECK();
  ts0.close();
  float* part = w.ssr;
  float* wn = part + (size_t)ceil_div(m, 128) * n;
  float* sim = wn + n;
  int processed = 0, r = m, cur = 0;
  bool pre = false;  // part holds rem's w-bar partials (from the previous block's error feedback)
  for (int k = 0; k < B; ++k) {
    const int bs = r < b ? r : b;
    const int nr = r - bs;
    int* rem = w.rem[cur];
    int* nrem = w.rem[cur ^ 1];
    StageScope ts_ssr(PT2Q_TIMER_SSR, st);
    if (ssr && r > b) {
      if ((rc = pt2q_launch_ssr_similarity(w.Wt, w.ldw, n, rem, r, part, wn, sim, st, w.counters + 4 * B, &g,
                                           pre)) != PT2Q_OK)
        return rc;
      if ((rc = pt2q_launch_ssr_topk(sim, rem, r, b, w.blk, nrem, perm64 + processed, st, nullptr, 0, nullptr,
                                     nullptr, nullptr, w.status, &g)) != PT2Q_OK)
        return rc;
    } else if ((rc = pt2q_launch_select_seq(ssr ? 1 : 0, ssr ? 0 : processed, bs, m, ssr ? rem : nullptr, w.blk,
                                            nrem, perm64 + processed, st, &g)) != PT2Q_OK) {
      return rc;
    }
    ts_ssr.close();
    StageScope ts_atq(PT2Q_TIMER_ATQ, st);
    // variant M: S1/d of every linear's block formed inside its ATQ launch (table g.G)
    if ((rc = pt2q_launch_atq_block(w.Wt, w.ldw, n, w.blk, bs, act ? w.S1 : nullptr, w.d, max_iter,
                                    w.alpha_t + (size_t)k * n, w.mu_t + (size_t)k * n, w.Tt, w.ldw,
                                    nr > 0 ? w.Et : nullptr, w.ldw, w.iters + k, w.counters + 2 * k, st,
                                    Hinv[0], ldhi, nrem, nr, w.Ck, m, w.iters_part, act ? A[0] : nullptr, lda,
                                    act ? w.counters + 2 * B + 2 * k : nullptr, w.status, &g)) != PT2Q_OK)
      return rc;
    ts_atq.close();
    StageScope ts_ef(PT2Q_TIMER_EF, st);
    const bool want = ssr && nr > b && ef_wbar_ok(n, w.ldw, w.Wt);  // the next block runs SSR over nrem
    if (nr > 0 && (rc = pt2q_launch_ef(w.Ck, m, w.Et, w.Wt, w.ldw, m, nrem, nr, bs, st, &g,
                                       want ? part : nullptr, n)) != PT2Q_OK)
      return rc;
    pre = want && nr > 0;
    processed += bs;
    r = nr;
    cur ^= 1;
  }
  StageScope ts1(PT2Q_TIMER_OUT, st);
  for (int z = 0; z < count; ++z) {  // outputs: T (n x m), alpha / mu (n x B), perm, iters
    auto sl = [&](auto* p) { return (decltype(p))((char*)p + z * zs); };
    if ((rc = pt2q_launch_transpose_i8(sl(w.Tt), w.ldw, m, n, T[z], tdtype, m, st)) != PT2Q_OK) return rc;
    if ((rc = pt2q_launch_transpose_f32(sl(w.alpha_t), n, B, n, alpha[z], B, st)) != PT2Q_OK) return rc;
    if ((rc = pt2q_launch_transpose_f32(sl(w.mu_t), n, B, n, mu[z], B, st)) != PT2Q_OK) return rc;
    if (hipMemcpyAsync(perm[z], sl(perm64), sizeof(int64_t) * m, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return PT2Q_E_HIP;
    if (iters_dev && iters_dev[z] &&
        hipMemcpyAsync(iters_dev[z], sl(w.iters), sizeof(int) * B, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return PT2Q_E_HIP;
  }
  return PT2Q_OK;
}

bool dtype_ok(int dt) { return dt == PT2Q_F32 || dt == PT2Q_F16 || dt == PT2Q_BF16; }

// Every condition under which pt2q_quantize_blocks_group runs (else PT2Q_E_UNSUPPORTED): blocks
// of <= 128 columns with b < m, variant M or no AGA, the tuning defaults (S1 in the ATQ launch,
// the EF kernel, the fused w-bar), n <= 16384 with n % 4 == 0, and the error feedback's own
// limits (pt2q_launch_ef: coefficient rows 16-byte aligned, every Wt under 2 GiB of buffer range).
bool group_ok(int n, int m, int b, int flags) {
  const int aga = flags & PT2Q_AGA_MASK;
  const Pt2qTuning& tu = pt2q_tuning();
  return n > 0 && m > 0 && b > 0 && b <= 128 && b < m && m < 65536 &&
         (aga == PT2Q_AGA_ACT || aga == PT2Q_AGA_NONE) && tu.s1_in_atq && tu.ef_kernel && tu.wbar_fused &&
         n <= 16384 && n % 4 == 0 && m % 4 == 0 && (long)m * round_up(n, 64) * 4 < 0x80000000L;
}

// The status word every workspace-taking call reserves first (PT2Q_STATUS_BYTES), zeroed on the
// call's stream before any kernel that may report into it.
int* take_status(Carve& c, hipStream_t st, int& rc) {
  int* s = c.take<int>(PT2Q_STATUS_BYTES / sizeof(int));
  rc = PT2Q_OK;
  if (s && hipMemsetAsync(s, 0, sizeof(int), st) != hipSuccess) rc = PT2Q_E_HIP;
  return s;
}

}  // namespace

extern "C" const char* pt2q_version(void) { return "pt2q-mi355x 0.1.0 (gfx950)"; }

extern "C" const char* pt2q_strerror(int status) {
  switch (status) {
    case PT2Q_OK: return "ok";
    case PT2Q_E_ARG: return "invalid argument";
    case PT2Q_E_NOT_SPD: return "Hessian not positive definite (Cholesky breakdown)";
    case PT2Q_E_UNSUPPORTED: return "unsupported shape/configuration";
    case PT2Q_E_HIP: return "HIP runtime error";
    case PT2Q_E_WORKSPACE: return "workspace too small";
    case PT2Q_E_STALL: return "a cross-workgroup wait timed out (results invalid)";
  }
  return "unknown status";
}

extern "C" int pt2q_stage_timing(int enable) {
  StageLog& l = stage_log();
  if (enable) {
    l.recs.clear();
    l.next = 0;
  }
  l.on = enable != 0;
  return PT2Q_OK;
}

extern "C" int pt2q_stage_timing_read(double* ms, int nstages, int* records) {
  if (!ms || nstages <= 0) return PT2Q_E_ARG;
  StageLog& l = stage_log();
  for (int i = 0; i < nstages; ++i) ms[i] = 0.0;
  for (const StageRec& r : l.recs) {
    float t = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&t, r.a, r.b) != hipSuccess)
      return PT2Q_E_HIP;
    if (r.stage >= 0 && r.stage < nstages) ms[r.stage] += t;
  }
  if (records) *records = (int)l.recs.size();
  return PT2Q_OK;
}

extern "C" int pt2q_quantize_blocks_group_supported(int n, int m, int b, int flags) {
  return group_ok(n, m, b, flags) ? 1 : 0;
}

extern "C" size_t pt2q_blocks_workspace_bytes(int n, int m, int b, int flags) {
  if (n <= 0 || m <= 0 || b <= 0) return 0;
  return PT2Q_STATUS_BYTES + blocks_bytes(n, m, b, flags);
}

extern "C" size_t pt2q_cholesky_workspace_bytes(int m) {
  return 2 * (((size_t)m * m * 4 + 255) & ~(size_t)255);
}

extern "C" size_t pt2q_layer_workspace_bytes(int n, int m, int b, int flags) {
  if (n <= 0 || m <= 0 || b <= 0) return 0;
  size_t mm = ((size_t)m * m * 4 + 255) & ~(size_t)255;
  return PT2Q_STATUS_BYTES + blocks_bytes(n, m, b, flags) + 4 * mm + 2 * 256 + pt2q_gram_workspace_bytes(m);
}

extern "C" size_t pt2q_ssr_workspace_bytes(int n, int m) {
  return PT2Q_STATUS_BYTES + blocks_bytes(n, m, 128);
}

extern "C" size_t pt2q_gram_workspace_bytes(int m) {
  return m > 0 ? PT2Q_STATUS_BYTES + ((pt2q_gram_flags_ints(m) * sizeof(int) + 255) & ~(size_t)255) : 0;
}

extern "C" int pt2q_gram(const void* X, int xdtype, int64_t N, int m, int64_t ldx, float* G,
                         int64_t ldg, int accumulate, void* workspace, size_t workspace_bytes,
                         void* stream) {
  if ((!X && N > 0) || !G || N < 0 || N > INT_MAX || m <= 0 || !dtype_ok(xdtype) || ldx < m ||
      ldg < m)
    return PT2Q_E_ARG;
  GemmDesc g{};
  g.M = m; g.N = m; g.K = (int)N;
  g.A = X; g.lda = ldx; g.a_layout = LAY_KMAJOR;
  g.B = X; g.ldb = ldx; g.b_layout = LAY_KMAJOR;
  g.in_dtype = xdtype;
  g.C = G; g.ldc = ldg;
  if (accumulate < 0 || accumulate > 2) return PT2Q_E_ARG;
  g.mode = accumulate == 2 ? GEMM_CHAIN_POS : accumulate ? GEMM_ADD : GEMM_STORE;
  g.upper = 1; g.mirror = 1;
  // workspace: [status word][split flags]; without it every tile is one chain (nothing waits)
  int *status = nullptr, *flags = nullptr;
  if (workspace && workspace_bytes >= pt2q_gram_workspace_bytes(m)) {
    Carve c{(char*)workspace, workspace_bytes};
    int rc;
    status = take_status(c, (hipStream_t)stream, rc);
    if (rc != PT2Q_OK) return rc;
    flags = c.take<int>(pt2q_gram_flags_ints(m));
  }
  StageScope ts(PT2Q_TIMER_GRAM, (hipStream_t)stream);
  return pt2q_launch_gram(g, flags, (hipStream_t)stream, status);
}

extern "C" int pt2q_gram_batched(int batch, const void* const* X, int xdtype, int64_t N, int m, int64_t ldx,
                                 float* G, void* stream) {
  if (batch <= 0 || !X || !G || N < 0 || N > INT_MAX || m <= 0 || ldx < m) return PT2Q_E_ARG;
  StageScope ts(PT2Q_TIMER_GRAM, (hipStream_t)stream);
  if (xdtype == PT2Q_F32)
    return pt2q_launch_gram_f32_batched((const float* const*)X, N, m, ldx, G, (long)m * m, batch, (hipStream_t)stream);
  return pt2q_launch_gram16_batched(X, xdtype, N, m, ldx, G, (long)m * m, batch, (hipStream_t)stream);
}

extern "C" int pt2q_gram_batched_upper(int batch, const void* const* X, int xdtype, int64_t N, int m,
                                       int64_t ldx, float* G, void* stream) {
  if (batch <= 0 || !X || !G || N < 0 || N > INT_MAX || m <= 0 || ldx < m) return PT2Q_E_ARG;
  if (xdtype != PT2Q_F16 && xdtype != PT2Q_BF16) return PT2Q_E_UNSUPPORTED;
  StageScope ts(PT2Q_TIMER_GRAM, (hipStream_t)stream);
  return pt2q_launch_gram16_batched(X, xdtype, N, m, ldx, G, (long)m * m, batch, (hipStream_t)stream, true);
}

extern "C" int pt2q_prepare_hessian(const float* G, int64_t ldg, int m, int64_t nsamples,
                                    float percdamp, float* H, int64_t ldh, float* damp_dev,
                                    void* stream) {
  if (!G || !H || m <= 0 || nsamples <= 0) return PT2Q_E_ARG;
  return pt2q_launch_prepare_hessian(G, ldg, m, nsamples, percdamp, H, ldh, damp_dev,
                                     (hipStream_t)stream);
}

extern "C" int pt2q_cholesky_inverse(const float* H, int64_t ldh, int m, float* Hinv,
                                     int64_t ldhi, void* workspace, size_t workspace_bytes,
                                     int* info_dev, void* stream) {
  if (!H || !Hinv || !info_dev || m <= 0) return PT2Q_E_ARG;
  Carve c{(char*)workspace, workspace_bytes};
  float* U = c.take<float>((size_t)m * m);
  float* Ui = c.take<float>((size_t)m * m);
  if (!c.ok) return PT2Q_E_WORKSPACE;
  StageScope ts(PT2Q_TIMER_INVERSE, (hipStream_t)stream);
  return pt2q_launch_cholesky_inverse(H, ldh, m, Hinv, ldhi, U, Ui, info_dev, (hipStream_t)stream);
}

// ---- a batch of units' damped Hessian inverses (main.py:129-139 per unit, one launch sequence)
extern "C" size_t pt2q_hessian_inverse_batched_workspace_bytes(int m, int batch) {
  if (m <= 0 || batch <= 0) return 0;
  return (((size_t)m * m * batch * 4 + 255) & ~(size_t)255) + (((size_t)batch * 4 + 255) & ~(size_t)255);
}

extern "C" int pt2q_hessian_inverse_batched(const float* G, int m, int batch, int64_t nsamples,
                                            float percdamp, float* H, float* Hinv, void* workspace,
                                            size_t workspace_bytes, int* info_dev, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!G || !H || !Hinv || !info_dev || m <= 0 || batch <= 0 || nsamples <= 0 || G == H || H == Hinv)
    return PT2Q_E_ARG;
  Carve c{(char*)workspace, workspace_bytes};
  float* Ui = c.take<float>((size_t)m * m * batch);
  float* damp = c.take<float>((size_t)batch);
  if (!c.ok) return PT2Q_E_WORKSPACE;
  const long mm = (long)m * m;
  // H written as the Cholesky work matrix at once (strictly lower part zero) where the damping
  // pass can (m <= SUMN_LDS_MAX); else in full form, then made upper in place by the factor
  const bool upper = m <= SUMN_LDS_MAX;
  int rc;
  StageScope ts(PT2Q_TIMER_INVERSE, st);
  if (upper) {  // every item in one launch pair
    if ((rc = pt2q_launch_prepare_hessian(G, m, m, nsamples, percdamp, H, m, damp, st, true, batch, mm)) != PT2Q_OK)
      return rc;
  } else {
    for (int z = 0; z < batch; ++z)
      if ((rc = pt2q_launch_prepare_hessian(G + z * mm, m, m, nsamples, percdamp, H + z * mm, m, damp + z, st,
                                            false)) != PT2Q_OK)
        return rc;
  }
  return pt2q_launch_cholesky_inverse(H, m, m, Hinv, m, H, Ui, info_dev, st, upper, batch);
}

extern "C" int pt2q_quantize_blocks(const void* W, int wdtype, int64_t ldw, int n, int m, int b,
                                    int flags, const float* A, int64_t lda, const float* Hinv,
                                    int64_t ldhi, int max_iter, float* alpha, float* mu, void* T,
                                    int tdtype, int64_t* perm, int* iters_dev, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  // Hinv feeds only the error feedback: a single block (per-channel, b >= m) leaves no columns
  // behind and never reads it, so it may be NULL there
  if (!W || (!Hinv && b < m) || !alpha || !mu || !T || !perm || n <= 0 || m <= 0 || b <= 0 ||
      !dtype_ok(wdtype) || (tdtype != PT2Q_I8 && tdtype != PT2Q_F32) || max_iter < 0 || ldw < m ||
      (Hinv && ldhi < m))
    return PT2Q_E_ARG;
  int aga = flags & PT2Q_AGA_MASK;
  if (flags & PT2Q_FLAG_S1_GIVEN) {  // A = S1 (m) then d: only the per-channel path reads it so
    if (aga != PT2Q_AGA_ACT || b < m || m <= 512 || !A) return PT2Q_E_ARG;
  } else if (aga != PT2Q_AGA_NONE && (!A || lda < m)) {
    return PT2Q_E_ARG;
  }
  Carve c{(char*)workspace, workspace_bytes};
  BlockWs w;
  int rc;
  w.status = take_status(c, (hipStream_t)stream, rc);
  if (rc != PT2Q_OK) return rc;
  if (!carve_blocks(c, n, m, b, w, flags)) return PT2Q_E_WORKSPACE;
  return run_blocks(W, wdtype, ldw, n, m, b, flags, A, lda, Hinv, ldhi, max_iter, alpha, mu, T,
                    tdtype, perm, iters_dev, w, (hipStream_t)stream);
}

extern "C" size_t pt2q_quantize_perchannel_group_workspace_bytes(int count) {
  if (count <= 0) return 0;
  return PT2Q_STATUS_BYTES + (((size_t)count * 3 * sizeof(int) + 255) & ~(size_t)255);
}

extern "C" int pt2q_quantize_perchannel_group(int count, const void* const* W, int wdtype, int64_t ldw,
                                              const int* n, int m, const float* const* S1d, int max_iter,
                                              float* const* alpha, float* const* mu, void* const* T, int tdtype,
                                              int64_t* const* perm, int* const* iters_dev, void* workspace,
                                              size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (count <= 0 || count > PT2Q_PC_GROUP_MAX || !W || !n || !alpha || !mu || !T || !perm || m <= 512 ||
      !dtype_ok(wdtype) || (tdtype != PT2Q_I8 && tdtype != PT2Q_F32) || max_iter < 0 || ldw < m)
    return PT2Q_E_ARG;
  for (int z = 0; z < count; ++z)
    if (!W[z] || n[z] <= 0 || !alpha[z] || !mu[z] || !T[z] || !perm[z]) return PT2Q_E_ARG;
  Carve c{(char*)workspace, workspace_bytes};
  int rc;
  int* status = take_status(c, st, rc);
  (void)status;  // no cross-workgroup waits here: the word stays 0
  if (rc != PT2Q_OK) return rc;
  int* ints = c.take<int>((size_t)count * 3);
  if (!c.ok) return PT2Q_E_WORKSPACE;
  PcLinear lin[PT2Q_PC_GROUP_MAX];
  PcSetupGroup sg{};
  for (int z = 0; z < count; ++z) {
    const float* s1 = S1d ? S1d[z] : nullptr;
    int* it = (iters_dev && iters_dev[z]) ? iters_dev[z] : ints + 2 * count + z;
    lin[z] = PcLinear{W[z], (long)ldw, n[z], s1, s1 ? s1 + m : nullptr, alpha[z], mu[z], T[z], (long)m, it,
                      ints + 2 * z, perm[z]};
    sg.perm[z] = perm[z];
    sg.counters[z] = ints + 2 * z;
    sg.iters[z] = it;
  }
  {
    StageScope ts(PT2Q_TIMER_SETUP, st);
    hipLaunchKernelGGL(pc_setup_group_kernel, dim3(ceil_div(m, 256), count), dim3(256), 0, st, sg, m);
    PT2Q_LAUNCH_CHECK();
  }
  StageScope ts_atq(PT2Q_TIMER_ATQ, st);
  return pt2q_launch_atq_rm_group(count, lin, wdtype, m, max_iter, tdtype, st);
}

extern "C" size_t pt2q_quantize_blocks_group_workspace_bytes(int count, int n, int m, int b, int flags) {
  if (count <= 0 || n <= 0 || m <= 0 || b <= 0) return 0;
  return PT2Q_STATUS_BYTES + (size_t)count * group_slice_bytes(n, m, b, flags);
}

extern "C" int pt2q_quantize_blocks_group(int count, const void* const* W, int wdtype, int64_t ldw, int n,
                                          int m, int b, int flags, const float* const* A, int64_t lda,
                                          const float* const* Hinv, int64_t ldhi, int max_iter,
                                          float* const* alpha, float* const* mu, void* const* T, int tdtype,
                                          int64_t* const* perm, int* const* iters_dev, void* workspace,
                                          size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int aga = flags & PT2Q_AGA_MASK;
  if (flags & PT2Q_FLAG_S1_GIVEN) return PT2Q_E_ARG;  // per-channel blocks only (pt2q_quantize_blocks)
  if (count <= 0 || count > PT2Q_GROUP_MAX || !W || !Hinv || !alpha || !mu || !T || !perm || n <= 0 ||
      m <= 0 || b <= 0 || !dtype_ok(wdtype) || (tdtype != PT2Q_I8 && tdtype != PT2Q_F32) || max_iter < 0 ||
      ldw < m || ldhi < m)
    return PT2Q_E_ARG;
  if (aga == PT2Q_AGA_ACT && (!A || lda < m)) return PT2Q_E_ARG;
  for (int z = 0; z < count; ++z)
    if (!W[z] || !Hinv[z] || !alpha[z] || !mu[z] || !T[z] || !perm[z] || (aga == PT2Q_AGA_ACT && !A[z]))
      return PT2Q_E_ARG;
  // grouped launches: blocks of at most 128 columns, several blocks (the error feedback runs),
  // variant M (S1/d in the ATQ launch) or no AGA, the fused w-bar, the EF kernel (group_ok)
  if (!group_ok(n, m, b, flags)) return PT2Q_E_UNSUPPORTED;
  Carve c{(char*)workspace, workspace_bytes};
  BlockWs w;
  int rc;
  w.status = take_status(c, st, rc);
  if (rc != PT2Q_OK) return rc;
  const size_t slice = group_slice_bytes(n, m, b, flags);
  char* base = c.p;
  if (!c.ok || !base || c.left < slice * count) return PT2Q_E_WORKSPACE;
  Carve s0{base, slice};
  if (!carve_blocks(s0, n, m, b, w, flags)) return PT2Q_E_WORKSPACE;
  int64_t* perm64 = s0.take<int64_t>((size_t)m);
  if (!s0.ok) return PT2Q_E_WORKSPACE;
  return run_blocks_group(count, W, wdtype, ldw, n, m, b, flags, A, lda, Hinv, ldhi, max_iter, alpha, mu, T,
                          tdtype, perm, iters_dev, w, perm64, (long)slice, st);
}

extern "C" int pt2q_quantize_layer(const void* W, int wdtype, int64_t ldw, int n, int m,
                                   const void* X, int xdtype, int64_t N, int64_t ldx, int b,
                                   int flags, float percdamp, int max_iter, float* alpha,
                                   float* mu, void* T, int tdtype, int64_t* perm, int* iters_dev,
                                   int* info_dev, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!W || !X || !info_dev || N <= 0 || N > INT_MAX || m <= 0 || n <= 0 || b <= 0 ||
      !dtype_ok(xdtype) || !dtype_ok(wdtype) || ldx < m || ldw < m || (flags & PT2Q_FLAG_S1_GIVEN))
    return PT2Q_E_ARG;
  Carve c{(char*)workspace, workspace_bytes};
  int rc;
  int* status = take_status(c, st, rc);
  if (rc != PT2Q_OK) return rc;
  float* G = c.take<float>((size_t)m * m);
  float* H = c.take<float>((size_t)m * m);
  float* Ui = c.take<float>((size_t)m * m);
  float* Hinv = c.take<float>((size_t)m * m);
  float* damp = c.take<float>(1);
  int* gflags = c.take<int>(pt2q_gram_flags_ints(m));
  BlockWs w;
  if (!c.ok || !carve_blocks(c, n, m, b, w)) return PT2Q_E_WORKSPACE;
  w.status = status;
  {
    GemmDesc g{};
    g.M = m; g.N = m; g.K = (int)N;
    g.A = X; g.lda = ldx; g.a_layout = LAY_KMAJOR;
    g.B = X; g.ldb = ldx; g.b_layout = LAY_KMAJOR;
    g.in_dtype = xdtype;
    g.C = G; g.ldc = m;
    g.mode = GEMM_STORE;
    g.upper = 1; g.mirror = 1;
    StageScope ts(PT2Q_TIMER_GRAM, st);
    if ((rc = pt2q_launch_gram(g, gflags, st, status)) != PT2Q_OK) return rc;
  }
  StageScope ts_inv(PT2Q_TIMER_INVERSE, st);
  // H is consumed in place as the Cholesky work matrix (variant M's AGA uses the raw Gram G), so
  // it is written in that form at once (strictly lower part zero; no separate copy pass).
  // Hinv only feeds the error feedback; a single block (per-channel, b >= m) has none, so the
  // factorisation would be dead work: skip it and report success.
  const bool upper = b < m && m <= SUMN_LDS_MAX;
  if ((rc = pt2q_launch_prepare_hessian(G, m, m, N, percdamp, H, m, damp, st, upper)) != PT2Q_OK) return rc;
  if (b < m) {
    if ((rc = pt2q_launch_cholesky_inverse(H, m, m, Hinv, m, H, Ui, info_dev, st, upper)) != PT2Q_OK)
      return rc;
  } else if (hipMemsetAsync(info_dev, 0, sizeof(int), st) != hipSuccess) {
    return PT2Q_E_HIP;
  }
  ts_inv.close();
  int f = (flags & ~PT2Q_AGA_MASK) | PT2Q_AGA_ACT;
  return run_blocks(W, wdtype, ldw, n, m, b, f, G, m, Hinv, m, max_iter, alpha, mu, T, tdtype,
                    perm, iters_dev, w, st);
}

extern "C" int pt2q_s1_from_gram(const float* S, int64_t lds, int b, float* S1, float* d_dev,
                                 void* stream) {
  if (!S || !S1 || !d_dev || b <= 0) return PT2Q_E_ARG;
  return pt2q_launch_aga_s1(1, S, lds, nullptr, b, S1, d_dev, (hipStream_t)stream);
}

extern "C" int pt2q_s1_from_gram_batched(const float* S, int64_t lds, int m, int batch, int64_t item_stride,
                                         float* S1d, void* stream) {
  if (!S || !S1d || m <= 0 || batch < 0 || lds < m || (batch > 1 && item_stride < lds * m)) return PT2Q_E_ARG;
  if (batch == 0) return PT2Q_OK;
  StageScope ts(PT2Q_TIMER_ATQ, (hipStream_t)stream);  // the AGA's S1 / d (quantizer.py:215-218)
  return pt2q_launch_s1_batched(S, lds, m, batch, item_stride, S1d, (hipStream_t)stream);
}

extern "C" int pt2q_s1_from_upper_batched(const float* S, int64_t lds, int m, int batch, int64_t item_stride,
                                          float* S1d, void* stream) {
  if (!S || !S1d || m <= 0 || batch < 0 || lds < m || (batch > 1 && item_stride < lds * m)) return PT2Q_E_ARG;
  if (batch == 0) return PT2Q_OK;
  StageScope ts(PT2Q_TIMER_ATQ, (hipStream_t)stream);
  return pt2q_launch_s1_batched(S, lds, m, batch, item_stride, S1d, (hipStream_t)stream, true);
}

extern "C" int pt2q_ssr_select(const float* W, int64_t ldw, int n, int m, const int64_t* rem, int r,
                               int b, int64_t* blk, int64_t* newrem, float* sim, void* workspace,
                               size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!W || !rem || !blk || n <= 0 || m <= 0 || r <= 0 || r > m || b <= 0 || ldw < m) return PT2Q_E_ARG;
  if (r > b && !newrem) return PT2Q_E_ARG;
  Carve c{(char*)workspace, workspace_bytes};
  BlockWs w;
  int rc;
  w.status = take_status(c, st, rc);
  if (rc != PT2Q_OK) return rc;
  if (!carve_blocks(c, n, m, 128, w)) return PT2Q_E_WORKSPACE;
  if ((rc = pt2q_launch_transpose_to_f32(W, PT2Q_F32, ldw, n, m, w.Wt, w.ldw, st)) != PT2Q_OK) return rc;
  hipLaunchKernelGGL(i64_to_i32_kernel, dim3(ceil_div(r, 256)), dim3(256), 0, st, rem, r, w.rem[0]);
  PT2Q_LAUNCH_CHECK();
  const int bs = r < b ? r : b;
  // blk indices (int32) are staged in rem[1] (capacity m >= b); newrem in the Tt scratch
  int* blk32 = w.rem[1];
  int* nrem32 = (int*)w.Tt;  // m*ldw bytes >= 4m
  if (sim || r > b) {
    float* part = w.ssr;
    float* wn = part + (size_t)ceil_div(m, 128) * n;
    float* simb = sim ? sim : wn + n;
    int* cnt = w.counters + 4 * ceil_div(m, 128);
    if (hipMemsetAsync(cnt, 0, sizeof(int) * pt2q_ssr_counter_ints(n), st) != hipSuccess) return PT2Q_E_HIP;
    if ((rc = pt2q_launch_ssr_similarity(w.Wt, w.ldw, n, w.rem[0], r, part, wn, simb, st, cnt)) != PT2Q_OK)
      return rc;
    if (r > b) {
      if ((rc = pt2q_launch_ssr_topk(simb, w.rem[0], r, b, blk32, nrem32, nullptr, st)) != PT2Q_OK)
        return rc;
      hipLaunchKernelGGL(i32_to_i64_kernel, dim3(ceil_div(r - bs, 256)), dim3(256), 0, st, nrem32,
                         r - bs, newrem);
      PT2Q_LAUNCH_CHECK();
    }
  }
  if (r <= b) blk32 = w.rem[0];
  hipLaunchKernelGGL(i32_to_i64_kernel, dim3(ceil_div(bs, 256)), dim3(256), 0, st, blk32, bs, blk);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

// ---- standalone error feedback (main.py:187-214 / gptq.py:158-186 for one block)
extern "C" size_t pt2q_error_feedback_workspace_bytes(int n, int m, int bs) {
  if (n <= 0 || m <= 0 || bs <= 0) return 0;
  Carve c{nullptr, 0};
  c.dry = true;
  const long ldW = round_up(n, 64);
  c.take<int>(PT2Q_STATUS_BYTES / sizeof(int));
  c.take<float>((size_t)m * ldW);
  c.take<float>((size_t)bs * ldW);
  c.take<float>((size_t)bs * round_up(m, 4));
  c.take<int>((size_t)bs);
  c.take<int>((size_t)m);
  return c.used;
}

extern "C" int pt2q_error_feedback(float* W, int64_t ldw, int n, int m, const int64_t* blk, int bs,
                                   const int64_t* rem, int r, const float* E, int64_t lde,
                                   const float* Hinv, int64_t ldhi, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!W || !blk || !E || !Hinv || n <= 0 || m <= 0 || bs <= 0 || r < 0 || bs + r > m ||
      ldw < m || lde < bs || ldhi < m || (r > 0 && !rem))
    return PT2Q_E_ARG;
  if (r == 0) return PT2Q_OK;
  Carve c{(char*)workspace, workspace_bytes};
  int rc;
  take_status(c, st, rc);  // reserved (nothing in this call waits on another workgroup)
  if (rc != PT2Q_OK) return rc;
  const long ldW = round_up(n, 64), ldc = round_up(m, 4);
  float* Wt = c.take<float>((size_t)m * ldW);
  float* Et = c.take<float>((size_t)bs * ldW);
  float* Ck = c.take<float>((size_t)bs * ldc);
  int* blk32 = c.take<int>((size_t)bs);
  int* rem32 = c.take<int>((size_t)m);
  if (!c.ok) return PT2Q_E_WORKSPACE;
  // feature-major working copies: column gathers W[:, rem] become row gathers of Wt
  if ((rc = pt2q_launch_transpose_to_f32(W, PT2Q_F32, ldw, n, m, Wt, ldW, st)) != PT2Q_OK) return rc;
  if ((rc = pt2q_launch_transpose_to_f32(E, PT2Q_F32, lde, n, bs, Et, ldW, st)) != PT2Q_OK) return rc;
  hipLaunchKernelGGL(i64_to_i32_kernel, dim3(ceil_div(bs, 256)), dim3(256), 0, st, blk, bs, blk32);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(i64_to_i32_kernel, dim3(ceil_div(r, 256)), dim3(256), 0, st, rem, r, rem32);
  PT2Q_LAUNCH_CHECK();
  // C[k][e] = Hinv[blk_k][rem_e] / clamp(Hinv[blk_k][blk_k], 1e-8)   (main.py:201-209)
  if ((rc = pt2q_launch_ef_coeffs(Hinv, ldhi, blk32, bs, rem32, r, Ck, ldc, st)) != PT2Q_OK) return rc;
  // W[:, rem] -= E @ C   (main.py:214: product rounded, then one subtraction)
  rc = pt2q_tuning().ef_kernel ? pt2q_launch_ef(Ck, ldc, Et, Wt, ldW, m, rem32, r, bs, st)
                               : PT2Q_E_UNSUPPORTED;
  if (rc == PT2Q_E_UNSUPPORTED) {
    GemmDesc g{};
    g.M = r; g.N = n; g.K = bs;
    g.A = Ck; g.lda = ldc; g.a_layout = LAY_KMAJOR;
    g.B = Et; g.ldb = ldW; g.b_layout = LAY_KMAJOR;
    g.in_dtype = PT2Q_F32;
    g.C = Wt; g.ldc = ldW; g.crow = rem32;
    g.mode = GEMM_SUB;
    rc = pt2q_launch_gemm(g, st);
  }
  if (rc != PT2Q_OK) return rc;
  return pt2q_launch_transpose_f32(Wt, ldW, m, n, W, ldw, st);
}
