// Asymmetric Ternary Quantizer (ATQ) kernels: init + ITF + AGA + error term, one pass.
//
// Reference: quantizer.py:32-293 (AsymmetricTernaryQuantizer), main.py:176-189 (per-block use).
//
// Mapping: a wave64 holds 4 weight rows; the 16 lanes of a row own the block columns
// k = l + 16 s (l = lane & 15, s = 0..NS-1), keeping w and the ternary codes in registers.
// Every row reduction is the canonical SUM16 (lane-sequential over s, then an xor-8/4/2/1
// butterfly), the same order oracle/pt2q_oracle.c uses, so codes AND scales are bit-identical
// to the oracle.  The reference's whole-block ITF stop (torch.equal over the block,
// quantizer.py:164) is evaluated per wave: rows that have converged are fixed points of
// grid+round, so continuing them reproduces the block loop exactly; the one block-level case
// that differs (every row's T_init == 0 -> the block loop returns the init grid untouched) is
// detected with a per-block counter and repaired by the last workgroup to finish.
#include <algorithm>
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace {

constexpr int ROWS_PER_WAVE = 4;
constexpr int WAVES = 4;
constexpr int ROWS_PER_WG = ROWS_PER_WAVE * WAVES;
PT2Q_DEV int ceil_div_dev(int a, int b) { return (a + b - 1) / b; }

// FULL: b == 16 * NS (every lane holds NS elements; no per-element range checks)
template <int NS, bool FULL = false>
struct Row {
  float w[NS];
  float t[NS];
  int l, b;
  PT2Q_DEV bool has(int s) const { return FULL || l + 16 * s < b; }
};

template <int NS, bool F>
PT2Q_DEV float row_sum_w(const Row<NS, F>& R) {
  float p = 0.0f;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (R.has(s)) p = p + R.w[s];
  return bfly16(p);
}

// ternary_init, quantizer.py:32-69. Returns alpha0, mu0; sets R.t; returns whether all t == 0.
template <int NS, bool F>
PT2Q_DEV bool row_init(Row<NS, F>& R, float wsum, float* alpha0, float* mu0) {
  const float fb = (float)R.b;
  float mu = wsum / fb;
  float p = 0.0f;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (R.has(s)) p = p + fabsf(R.w[s] - mu);
  float delta = 0.75f * (bfly16(p) / fb);
  float pn = 0.0f, pd = 0.0f;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float t = 0.0f;
    if (R.has(s)) {
      float wc = R.w[s] - mu;
      t = (wc > delta) ? 1.0f : ((wc < -delta) ? -1.0f : 0.0f);
      pn = fmaf(t, wc, pn);  // t * wc exact
      pd = pd + fabsf(t);
    }
    R.t[s] = t;
  }
  float num = bfly16(pn);
  float cnt = bfly16(pd);
  *alpha0 = num / clampmin(cnt);
  *mu0 = mu;
  return cnt == 0.0f;
}

// build_optimal_grid, quantizer.py:71-108.  TERN (codes known to be in {-1, 0, 1}: every grid of
// the ITF loop): sum(w t) is the SUM16 of fmaf(w, t, p) (w * t is exact, so each step is the same
// rounding of p + w * t), and sum(t), sum(t^2) are integers with |sum t| <= sum t^2 <= b <= 512:
// one SUM16 of 1024 t^2 + t carries both exactly (every partial < 2^24; |sum t| / 1024 <= 0.5 and
// the tie at |sum t| = 512 -- all codes of one sign, sum t^2 = 512 -- rounds to the even 512).
// !TERN (the per-method GRID / ITF stages read the caller's T, any values): three separate
// SUM16 chains of the plain products, as the oracle (grid_row).
template <bool TERN, int NS, bool F>
PT2Q_DEV void row_grid(const Row<NS, F>& R, float wsum, float* a, float* m) {
  static_assert(16 * NS <= 512, "packed grid counts need b <= 512");
  float pwt = 0.0f, pt = 0.0f, pt2 = 0.0f;
  float swt, ts, t2;
  if constexpr (TERN) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (R.has(s)) {
        pwt = fmaf(R.w[s], R.t[s], pwt);
        pt = pt + R.t[s];
        pt2 = fmaf(R.t[s], R.t[s], pt2);
      }
    const float v = bfly16(fmaf(pt2, 1024.0f, pt));
    swt = bfly16(pwt);
    t2 = rintf(v * 0x1p-10f);
    ts = fmaf(-1024.0f, t2, v);
  } else {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (R.has(s)) {
        pwt = pwt + R.w[s] * R.t[s];
        pt = pt + R.t[s];
        pt2 = pt2 + R.t[s] * R.t[s];
      }
    swt = bfly16(pwt);
    ts = bfly16(pt);
    t2 = bfly16(pt2);
  }
  const float fb = (float)R.b;
  float den = clampmin(fb * t2 - ts * ts);
  *a = (fb * swt - ts * wsum) / den;
  *m = (t2 * wsum - ts * swt) / den;
}

// flexible_round, quantizer.py:110-134 (round_code). Returns true if this lane changed a code.
template <int NS, bool F>
PT2Q_DEV bool row_round(Row<NS, F>& R, float a, float m) {
  const RoundTh th = round_th(clampmin(a));
  bool changed = false;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (R.has(s)) {
      const float nt = round_code(R.w[s] - m, th);
      changed |= (nt != R.t[s]);
      R.t[s] = nt;
    }
  return changed;
}

// iterative_ternary_fitting, quantizer.py:136-175, wave-level stop (see file header).
// Assumes the block is not all-zero at init (iteration 0 never stops).  TERN: the codes on entry
// are ternary (from row_init); the stage entry passes the caller's T, so its first grid is the
// general one (every later grid sees round's codes).
template <bool TERN, int NS, bool F>
PT2Q_DEV int row_itf(Row<NS, F>& R, float wsum, int max_iter, float* a, float* m) {
  int it = 0;
  bool any = true;
  if (!TERN && max_iter > 0) {
    row_grid<false>(R, wsum, a, m);
    any = __any(row_round(R, *a, *m));
    it = 1;
  }
  for (; it < max_iter; ++it) {
    if (!any) break;
    row_grid<true>(R, wsum, a, m);
    bool ch = row_round(R, *a, *m);
    any = __any(ch);
  }
  return it;
}

// activation_aware_grid_alignment, quantizer.py:177-248, given S1 (per lane) and d.
template <int NS, bool F>
PT2Q_DEV void row_aga(const Row<NS, F>& R, const float (&S1)[NS], float d, float* a, float* m) {
  float pv = 0.0f, pws = 0.0f, pwts = 0.0f, pt2s = 0.0f;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (R.has(s)) {
      float t = R.t[s], w = R.w[s], c = S1[s];
      pv = fmaf(t, c, pv);
      pws = fmaf(w, c, pws);
      pwts = fmaf(w * t, c, pwts);
      pt2s = fmaf(t * t, c, pt2s);
    }
  float v = bfly16(pv), ws1 = bfly16(pws), wts1 = bfly16(pwts), t2s1 = bfly16(pt2s);
  float v2 = v * v;
  float den = clampmin(d * t2s1 - v2);
  *a = (d * wts1 - v * ws1) / den;
  *m = (t2s1 * ws1 - v * wts1) / den;
}

struct BlockArgs {
  const float* Wt;   // m x ldw feature-major working weights
  long ldw;
  int n, b;
  const int* blk;    // b column indices (selection order)
  const float* S1;   // b, or nullptr (no AGA)
  const float* d;    // device scalar
  int max_iter;
  float* alpha;      // n   (row kb of alpha_t)
  float* mu;         // n
  int8_t* Tt;        // m x ldt int8 codes (feature-major, original order)
  long ldt;
  float* Et;         // b x lde error term E[k][i] = w - (alpha*t + mu)
  long lde;
  int* iters;        // 1 int (atomicMax), nullable
  int* counters;     // [0] zero-init rows, [1] workgroups done
  int* iters_part;   // per-workgroup iteration maxima (reduced by the next launch), nullable
  // S1/d formed inside the launch (variant M, b <= 128): nS1 leading workgroups gather
  // S1 = G[blk][blk]·1 and d into S1w / dw and raise s1sync[0]; the row workgroups wait for it
  // only before their AGA.  nS1 = 0: S1 / d come ready from an earlier launch.
  const float* G;
  long ldg;
  int nS1;
  int* s1sync;       // [0] ready flag, [1] S1 workgroups done (zero before the launch)
  float* S1w;
  float* dw;
  int* status;       // stall reports (nullable)
  long cap;          // polls before a wait gives up
  int probe;         // development knock-outs (pt2q_tuning().atq_probe; 0 in release builds)
};

// Grouped launch: linear z's pointers -- its workspace slice, its raw Gram.
template <typename T>
PT2Q_DEV T* zslice(T* p, long ws, int z) {  // nullptr stays nullptr
  return p ? (T*)((char*)p + (long)z * ws) : p;
}
PT2Q_DEV BlockArgs at_linear(BlockArgs A, const Grp& g, int z) {
  if (g.count == 0) return A;
  const long zs = g.ws;
  A.Wt = zslice(A.Wt, zs, z);
  A.blk = zslice(A.blk, zs, z);
  A.S1 = zslice(A.S1, zs, z);
  A.d = zslice(A.d, zs, z);
  A.alpha = zslice(A.alpha, zs, z);
  A.mu = zslice(A.mu, zs, z);
  A.Tt = zslice(A.Tt, zs, z);
  A.Et = zslice(A.Et, zs, z);
  A.iters = zslice(A.iters, zs, z);
  A.counters = zslice(A.counters, zs, z);
  A.iters_part = zslice(A.iters_part, zs, z);
  A.s1sync = zslice(A.s1sync, zs, z);
  A.S1w = zslice(A.S1w, zs, z);
  A.dw = zslice(A.dw, zs, z);
  if (A.G) A.G = g.G[z];
  return A;  // status: one word for the whole call
}

// S1 / d of the block formed by one wave itself, in the order of atq_s1_part (S1[j]: l-ascending
// sum of G[blk_j][blk_l]; d: j-ascending sum of S1), so the values are the same bits.  The
// fallback of a row wave whose wait for the leading workgroups gives up: under heavy concurrency
// (several streams of launches with in-launch hand-offs) those workgroups can sit undispatched on
// a full XCD while this wave holds its CU, so the wave computes instead of waiting or failing.
// Lane (r, l) forms S1[l + 16 s]; d gathers S1[j] from lane (r, j & 15), slot j >> 4.
template <int NS>
PT2Q_DEV void s1_local(const BlockArgs& A, int l, float (&S1)[NS], float* dv) {
  const int b = A.b;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = l + 16 * s;
    float acc = 0.0f;
    if (k < b) {
      const long bj = (long)A.blk[k] * A.ldg;
      int q = 0;
      for (; q + 8 <= b; q += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = A.G[bj + A.blk[q + u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + t[u];
      }
      for (; q < b; ++q) acc = acc + A.G[bj + A.blk[q]];
    }
    S1[s] = acc;
  }
  const int base = (int)(threadIdx.x & 63) & 48;
  float d = 0.0f;
  for (int j = 0; j < b; ++j) {
    float x = 0.0f;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if ((j >> 4) == s) x = S1[s];
    d = d + __shfl(x, base | (j & 15));
  }
  *dv = d;
}

// Returns the wave's ITF iteration count (wave-uniform).
template <int NS, bool F = false>
PT2Q_DEV int block_rows(const BlockArgs& A, int row0, bool skip_itf, bool count_zero) {
  const int lane = threadIdx.x & 63;
  const int r = lane >> 4, l = lane & 15;
  const int i = row0 + r;
  const bool valid = i < A.n;
  Row<NS, F> R;
  R.l = l;
  R.b = A.b;
  // branch-free loads in two rounds (block indices, then the gathers), so that each round is
  // in flight at once instead of one dependent round trip per element; out-of-range lanes read
  // entry 0 / row 0 and discard it
  int colrow[NS];
  float S1[NS];
  const int ic = valid ? i : 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = l + 16 * s;
    colrow[s] = A.blk[k < A.b ? k : 0];
  }
  float v[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) v[s] = A.Wt[(long)colrow[s] * A.ldw + ic];
  const bool s1_now = A.S1 && A.nS1 == 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = l + 16 * s;
    S1[s] = s1_now ? A.S1[k < A.b ? k : 0] : 0.0f;
    S1[s] = k < A.b ? S1[s] : 0.0f;
    R.w[s] = (valid && k < A.b) ? v[s] : 0.0f;
  }
  float dv = s1_now ? *A.d : 0.0f;
  float wsum = row_sum_w(R);
  float a, m;
  bool zero = row_init(R, wsum, &a, &m);
  if (count_zero && valid && l == 0 && zero) atomicAdd(&A.counters[0], 1);
  int it = 0;
  if (!skip_itf && !(A.probe & 4)) it = row_itf<true>(R, wsum, A.max_iter, &a, &m);
  if (A.S1 && A.nS1 > 0 && !(A.probe & 1)) {  // S1 / d from this launch's leading workgroups (write-through)
    int ready = 1;
    if ((threadIdx.x & 63) == 0) ready = wait_flag_ge<2>(&A.s1sync[0], 1, A.cap, nullptr, 0);
    ready = __builtin_amdgcn_readfirstlane(ready);
    __builtin_amdgcn_wave_barrier();
    if (ready) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int k = l + 16 * s;
        const float x = __hip_atomic_load(&A.S1w[k < A.b ? k : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        S1[s] = k < A.b ? x : 0.0f;
      }
      dv = __hip_atomic_load(A.dw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      s1_local<NS>(A, l, S1, &dv);
    }
  }
  if (A.S1) row_aga(R, S1, dv, &a, &m);
  if (!valid) return it;
  if (l == 0) {
    A.alpha[i] = a;
    A.mu[i] = m;
  }
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (R.has(s)) {
      int k = l + 16 * s;
      A.Tt[(long)colrow[s] * A.ldt + i] = (int8_t)R.t[s];
      if (A.Et) A.Et[(long)k * A.lde + i] = R.w[s] - (a * R.t[s] + m);
    }
  return it;
}

// RG row groups per wave (rows base + 16 g + r, g < RG): every group's gathers are issued before
// the first group's arithmetic, the block indices and S1 / d are loaded once for all of them.  The
// block ATQ is bound by these load round trips, not by its ITF arithmetic (knock-outs,
// tools/atq_knock.sh: skipping ITF altogether moved a grouped 7B launch 100 -> 99 us), so one
// wave carrying several groups' loads at once is what shortens it.  Per row, the values and their
// order are block_rows' (same Row arithmetic), so the bits are the same.
template <int NS, bool F, int RG>
PT2Q_DEV int block_rows_rg(const BlockArgs& A, int base) {
  const int lane = threadIdx.x & 63;
  const int r = lane >> 4, l = lane & 15;
  int colrow[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = l + 16 * s;
    colrow[s] = A.blk[k < A.b ? k : 0];
  }
  float v[RG][NS];
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int i = base + 16 * g + r;
    const int ic = i < A.n ? i : 0;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      v[g][s] = (A.probe & 32) ? (float)(ic + s) : A.Wt[(long)colrow[s] * A.ldw + ic];
  }
  const bool s1_now = A.S1 && A.nS1 == 0;
  float S1[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = l + 16 * s;
    S1[s] = s1_now ? A.S1[k < A.b ? k : 0] : 0.0f;
    S1[s] = k < A.b ? S1[s] : 0.0f;
  }
  float dv = s1_now ? *A.d : 0.0f;
  int itmax = 0;
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int i = base + 16 * g + r;
    const bool valid = i < A.n;
    Row<NS, F> R;
    R.l = l;
    R.b = A.b;
#pragma unroll
    for (int s = 0; s < NS; ++s) R.w[s] = (valid && l + 16 * s < A.b) ? v[g][s] : 0.0f;
    const float wsum = row_sum_w(R);
    float a, m;
    const bool zero = row_init(R, wsum, &a, &m);
    if (valid && l == 0 && zero) atomicAdd(&A.counters[0], 1);
    int it = 0;
    if (!(A.probe & 4)) it = row_itf<true>(R, wsum, A.max_iter, &a, &m);
    itmax = max(itmax, it);
    if (g == 0 && A.S1 && A.nS1 > 0 && !(A.probe & 1)) {  // S1 / d from the leading workgroups, once
      int ready = 1;
      if (lane == 0) ready = wait_flag_ge<2>(&A.s1sync[0], 1, A.cap, nullptr, 0);
      ready = __builtin_amdgcn_readfirstlane(ready);
      __builtin_amdgcn_wave_barrier();
      if (ready) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int k = l + 16 * s;
          const float x = __hip_atomic_load(&A.S1w[k < A.b ? k : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          S1[s] = k < A.b ? x : 0.0f;
        }
        dv = __hip_atomic_load(A.dw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        s1_local<NS>(A, l, S1, &dv);
      }
    }
    if (A.S1) row_aga(R, S1, dv, &a, &m);
    if (valid) {
      if (l == 0 && !(A.probe & 256)) {
        A.alpha[i] = a;
        A.mu[i] = m;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
        if (R.has(s)) {
          const int k = l + 16 * s;
          if (!(A.probe & 8)) A.Tt[(long)colrow[s] * A.ldt + i] = (int8_t)R.t[s];
          if (A.Et && !(A.probe & 128)) A.Et[(long)k * A.lde + i] = R.w[s] - (a * R.t[s] + m);
        }
    }
  }
  return itmax;
}

// 128-column blocks through a per-wave LDS stage (VEC): a wave owns 16 consecutive rows (four
// groups of 4) and moves them as 16-byte pieces -- a block column's 16 rows of W are read, and its
// 16 codes and 16 error terms written, 16 bytes per lane.  The per-element form (block_rows_rg:
// 4- and 1-byte pieces, 16 cache lines per instruction) spent ~18 us of a grouped 7B launch on the
// code stores and ~18 us on the error-term stores (knock-outs, tools/atq_knock.sh masks 8 / 128).
// Per row, the arithmetic is block_rows_rg's, so the bits are the same.
constexpr int VEC_KC = 32;                  // block columns per staging chunk
constexpr int VEC_KS = 20;                  // floats per staged column: 16 rows + pad (16-B aligned,
                                            // the 64 lanes' writes on 64 distinct banks)
constexpr int VEC_STAGE = VEC_KC * VEC_KS;  // floats per wave (2560 B)

PT2Q_DEV uint32_t byte_of(uint32_t x, int j) { return (x >> (8 * j)) & 0xffu; }

template <int NS>
PT2Q_DEV int block_rows_vec(const BlockArgs& A, int base) {
  constexpr int RG = 4, NC = 16 * NS / VEC_KC;
  static_assert(16 * NS == 128, "VEC: 128-column blocks");
  __shared__ float stage_all[WAVES][VEC_STAGE];
  float* stg = stage_all[threadIdx.x >> 6];
  uint32_t* stg32 = (uint32_t*)stg;
  const int lane = threadIdx.x & 63;
  const int r = lane >> 4, l = lane & 15;
  const int q4 = lane >> 2, part = lane & 3;  // staging lanes: chunk columns q4 + 16 h, rows 4 part ..
  if (base >= A.n) return 0;                  // n % 16 == 0: a wave's rows are all valid or none
  // W: every chunk's 16-byte pieces in flight, then through the stage into the row layout
  float4 gv[NC][2];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long col = A.blk[VEC_KC * c + q4 + 16 * h];
      gv[c][h] = (A.probe & 32) ? make_float4(0.f, 1.f, 2.f, 3.f)
                                : *(const float4*)(A.Wt + col * A.ldw + base + 4 * part);
    }
  const bool s1_now = A.S1 && A.nS1 == 0;
  float S1[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) S1[s] = s1_now ? A.S1[l + 16 * s] : 0.0f;
  float dv = s1_now ? *A.d : 0.0f;
  float v[RG][NS];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int h = 0; h < 2; ++h) *(float4*)(stg + (q4 + 16 * h) * VEC_KS + 4 * part) = gv[c][h];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < RG; ++g) v[g][2 * c + j] = stg[(l + 16 * j) * VEC_KS + 4 * g + r];
  }
  uint32_t tc[NS];  // codes of the four groups, byte g = row base + 4 g + r
#pragma unroll
  for (int s = 0; s < NS; ++s) tc[s] = 0;
  int itmax = 0;
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int i = base + 4 * g + r;
    Row<NS, true> R;
    R.l = l;
    R.b = A.b;
#pragma unroll
    for (int s = 0; s < NS; ++s) R.w[s] = v[g][s];
    const float wsum = row_sum_w(R);
    float a, m;
    const bool zero = row_init(R, wsum, &a, &m);
    if (l == 0 && zero) atomicAdd(&A.counters[0], 1);
    int it = 0;
    if (!(A.probe & 4)) it = row_itf<true>(R, wsum, A.max_iter, &a, &m);
    itmax = max(itmax, it);
    if (g == 0 && A.S1 && A.nS1 > 0 && !(A.probe & 1)) {  // S1 / d from the leading workgroups, once
      int ready = 1;
      if (lane == 0) ready = wait_flag_ge<2>(&A.s1sync[0], 1, A.cap, nullptr, 0);
      ready = __builtin_amdgcn_readfirstlane(ready);
      __builtin_amdgcn_wave_barrier();
      if (ready) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
          S1[s] = __hip_atomic_load(&A.S1w[l + 16 * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dv = __hip_atomic_load(A.dw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        s1_local<NS>(A, l, S1, &dv);
      }
    }
    if (A.S1) row_aga(R, S1, dv, &a, &m);
    if (l == 0 && !(A.probe & 256)) {
      A.alpha[i] = a;
      A.mu[i] = m;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      tc[s] |= ((uint32_t)(uint8_t)(int8_t)R.t[s]) << (8 * g);
      v[g][s] = R.w[s] - (a * R.t[s] + m);  // the error term, in place of w
    }
  }
  // The stage is accessed as float (W, error terms) and as uint32 / uint4 (codes); the library
  // is built without -fno-strict-aliasing, so a compiler barrier keeps each typed phase's
  // accesses on its side (type-based alias analysis could otherwise move a uint32 store above
  // the float reads of W, or the error-term float stores above the code loads).
  asm volatile("" ::: "memory");
  // codes: lane (r, l) puts row r's four group bytes of column k at dword 4 k + r; lane q reads
  // column q + 64 h (16 bytes, row-group-major) and transposes it to row order
#pragma unroll
  for (int s = 0; s < NS; ++s) stg32[4 * (l + 16 * s) + r] = tc[s];
  if (!(A.probe & 8)) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = lane + 64 * h;
      const uint4 x = *(const uint4*)(stg32 + 4 * k);
      uint4 y;
      uint32_t* yy = (uint32_t*)&y;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        yy[g] = byte_of(x.x, g) | byte_of(x.y, g) << 8 | byte_of(x.z, g) << 16 | byte_of(x.w, g) << 24;
      *(uint4*)(A.Tt + (long)A.blk[k] * A.ldt + base) = y;
    }
  }
  asm volatile("" ::: "memory");  // code loads of the stage before its float reuse (see above)
  // error terms, a chunk of 32 columns at a time
  if (A.Et && !(A.probe & 128)) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < RG; ++g) stg[(l + 16 * j) * VEC_KS + 4 * g + r] = v[g][2 * c + j];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kk = q4 + 16 * h;
        *(float4*)(A.Et + (long)(VEC_KC * c + kk) * A.lde + base + 4 * part) =
            *(const float4*)(stg + kk * VEC_KS + 4 * part);
      }
    }
  }
  return itmax;
}

// row groups per wave of the fused block ATQ (registers: RG x NS gathered values in flight): 4 at
// 128-column blocks (122 VGPRs, four waves per SIMD), 2 in the six-wave variant (PT2Q_ATQ_OCC),
// one group for wider blocks
template <int NS, int OCC>
constexpr int atq_rg() { return NS == 8 ? (OCC > 0 ? 2 : 4) : 1; }

// Iteration count of a block: one store per wave (iters_part), reduced by the post / fixup
// launch -- not one atomic per wave on a single word (1024 atomics serialise at the memory side
// and hold the kernel's end for ~10 us).
// S1[j] = l-ascending sum of G[blk_j][blk_l], d = j-ascending sum of S1 (the s1_block order):
// 8 rows j per workgroup gathered into LDS, one lane sums each; the last S1 workgroup forms d
// and raises the flag.  Write-through stores drained before the counter / flag, sc1 loads.
// (Measured slower: rows forming d themselves with no last-workgroup stage; one workgroup for
// all of S1 -- its per-lane serial sums take longer than the hand-off they save.)
PT2Q_DEV float s1_serial_sum(const float* v, int b) {  // ((v0 + v1) + v2) ..., loads batched
  float s = 0.0f;
  int q = 0;
  for (; q + 8 <= b; q += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = v[q + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + t[u];
  }
  for (; q < b; ++q) s = s + v[q];
  return s;
}

PT2Q_DEV void atq_s1_part(const BlockArgs& A, int x) {
  __shared__ float gb[8][129];
  __shared__ int last;
  const int tid = threadIdx.x, jj = tid >> 5, ln = tid & 31;
  const int j = x * 8 + jj;
  if (j < A.b) {
    const long bj = (long)A.blk[j] * A.ldg;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int l = ln + 32 * u;
      if (l < A.b) gb[jj][l] = A.G[bj + A.blk[l]];
    }
  }
  __syncthreads();
  if (ln == 0 && j < A.b)
    __hip_atomic_store(&A.S1w[j], s1_serial_sum(gb[jj], A.b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) last = atomicAdd(&A.s1sync[1], 1) == A.nS1 - 1;
  __syncthreads();
  if (!last) return;
  if (tid < A.b) gb[0][tid] = __hip_atomic_load(&A.S1w[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(A.dw, s1_serial_sum(gb[0], A.b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&A.s1sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The error-feedback coefficients C[k][e] = Hinv[blk_k][rem_e] / clamp(Hinv[blk_k][blk_k])
// (main.py:201-209) of the block.  They depend only on the selection (blk, rem), not on the ATQ
// results, so they are formed by extra workgroups of the ATQ launch itself, placed AFTER the row
// workgroups: dispatched last, they fill the CUs the rows' ITF convergence tail leaves idle.
struct CoeffArgs {
  const float* Hinv;
  long ldh;
  const int* rem;
  int nr, bs;
  float* C;
  long ldc;
  int per_k;  // coefficient workgroups per k row (COEF_SPAN columns e each)
};
// columns e per coefficient workgroup: 16 per lane (4 x 16-byte index loads, 16 gathers in flight
// before the divisions); 1024 per workgroup (4 per lane) gave 4x the workgroups, each parked on
// two dependent load round trips for a few divisions
constexpr int COEF_SPAN = 4096;

PT2Q_DEV void coeff_part(const BlockArgs& A, const CoeffArgs& K, int cb) {
  const int k = cb / K.per_k;
  if (k >= K.bs) return;
  const int base = (cb - k * K.per_k) * COEF_SPAN + 4 * (int)threadIdx.x;  // + 1024 j + v
  const long rowb = (long)A.blk[k] * K.ldh;
  int re[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = base + 1024 * j;
    if (e + 3 < K.nr && (((uintptr_t)(K.rem + e)) & 15) == 0) {
      const int4 v = *(const int4*)(K.rem + e);
      re[4 * j] = v.x, re[4 * j + 1] = v.y, re[4 * j + 2] = v.z, re[4 * j + 3] = v.w;
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v) re[4 * j + v] = e + v < K.nr ? K.rem[e + v] : 0;
    }
  }
  const float dg = clampmin(K.Hinv[rowb + A.blk[k]]);
  float h[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) h[u] = K.Hinv[rowb + re[u]];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int e = base + 1024 * j + v;
      if (e < K.nr) K.C[(long)k * K.ldc + e] = h[4 * j + v] / dg;
    }
}

template <int NS, bool F, int RG, bool VEC>
PT2Q_DEV void atq_block_body(const BlockArgs& A0, const Grp& g, CoeffArgs K, int rowgrid, int cgrid);

// OCC: 0 = the compiler's register budget (four waves per SIMD at NS = 8); 6 = at least six waves
// per SIMD (80 VGPRs, two row groups per wave, no spills: PT2Q_ATQ_OCC).  VEC: block_rows_vec.
template <int NS, bool F, int OCC, bool VEC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC > 0 ? OCC : 1, 8))) void atq_block_kernel(
    BlockArgs A0, Grp g, CoeffArgs K, int rowgrid, int cgrid) {
  atq_block_body<NS, F, VEC ? 4 : atq_rg<NS, OCC>(), VEC>(A0, g, K, rowgrid, cgrid);
}

// One 1-D grid for every linear z of the launch, in three role ranges: the S1 / d workgroups of
// every linear (dispatched first, they wait on nobody), then the row workgroups of every linear,
// then the EF-coefficient workgroups of every linear (dispatched last, they fill the CUs the rows'
// ITF tail leaves idle).  Linear-major inside each range: every linear's S1 is under way before
// any row workgroup, where a grid.z launch dispatched linear z's S1 workgroups only after every
// workgroup of linears 0 .. z-1.
template <int NS, bool F, int RG, bool VEC>
PT2Q_DEV void atq_block_body(const BlockArgs& A0, const Grp& g, CoeffArgs K, int rowgrid, int cgrid) {
  const int nz = g.count > 0 ? g.count : 1;
  int b = (int)blockIdx.x;
  if (b < nz * A0.nS1) {
    const int z = b / A0.nS1;
    if (A0.probe & 16) return;
    atq_s1_part(at_linear(A0, g, z), b - z * A0.nS1);
    return;
  }
  b -= nz * A0.nS1;
  if (b >= nz * rowgrid) {
    b -= nz * rowgrid;
    const int z = b / cgrid;
    if (g.count > 0) {
      K.Hinv = g.Hinv[z];
      K.rem = zslice(K.rem, g.ws, z);
      K.C = zslice(K.C, g.ws, z);
    }
    coeff_part(at_linear(A0, g, z), K, b - z * cgrid);
    return;
  }
  if (A0.probe & 64) return;
  const int z = b / rowgrid;
  const BlockArgs A = at_linear(A0, g, z);
  const int wave = threadIdx.x >> 6;
  const int rb = b - z * rowgrid;
  int it;
  if constexpr (VEC && NS == 8)
    it = block_rows_vec<NS>(A, rb * ROWS_PER_WG * RG + wave * ROWS_PER_WAVE * RG);
  else
    it = block_rows_rg<NS, F, RG>(A, rb * ROWS_PER_WG * RG + wave * ROWS_PER_WAVE);
  if (!A.iters || (threadIdx.x & 63) != 0) return;
  // one store per wave, no barrier: a wave whose rows converged early leaves at once instead of
  // holding its slot until the workgroup's slowest wave (the block-ATQ waves were parked 59 % of
  // their cycles, profiles/r05j_atq7b_pmc.txt)
  if (A.iters_part) A.iters_part[rb * WAVES + wave] = it;
  else atomicMax(A.iters, it);
}

// *iters = max of the block kernel's per-workgroup maxima, or 0 for an all-zero block (ITF did
// not run: quantizer.py:164).  Workgroup 0, wave 0 of the launch after the block kernel.
PT2Q_DEV void finish_iters(const BlockArgs& A, int nparts) {
  if (!A.iters || !A.iters_part || blockIdx.x != 0 || threadIdx.x >= 64) return;
  int v = 0;
  for (int j = threadIdx.x; j < nparts; j += 64) v = max(v, A.iters_part[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  if (threadIdx.x == 0) *A.iters = (A.counters[0] == A.n) ? 0 : v;
}

// After the block's ATQ, one workgroup per linear: the block's ITF iteration count
// (finish_iters) and, only for an all-zero block, the repair of every row.  The whole-block
// T_init == 0 case (quantizer.py:164 breaks at iteration 0 and returns the init grid) is known
// only after every row workgroup: this launch reads the zero-row count after the kernel boundary
// and, only then, redoes every row without ITF (one workgroup: it costs nothing when it never
// runs; a last-arriving-workgroup repair inside atq_block_kernel cost an agent-scope release
// fence -- an L2 write-back -- per workgroup).
template <int NS>
__global__ __launch_bounds__(256) void atq_finish_kernel(BlockArgs A0, int rowgrid, Grp g) {
  const BlockArgs A = at_linear(A0, g, blockIdx.z);
  finish_iters(A, rowgrid * WAVES);
  if (A.counters[0] != A.n) return;
  const int wave = threadIdx.x >> 6;
  if (A.iters && !A.iters_part && threadIdx.x == 0) *A.iters = 0;
  for (int rb = 0; rb < ceil_div_dev(A.n, ROWS_PER_WG); ++rb)
    block_rows<NS>(A, rb * ROWS_PER_WG + wave * ROWS_PER_WAVE, true, false);
}

// ----------------------------------------------------------------- per-stage kernel (row-major)

struct StageArgs {
  int mode;
  const float* W;
  long ldw;
  int n, b;
  float* alpha;
  float* mu;
  float* T;
  long ldt;
  const float* S1;
  const float* d;
  int max_iter;
  int* iters;
  int* zero_rows;  // FULL / ITF: block all-zero detection (two-pass)
  int pass;        // FULL: 0 = init + count, 1 = finish
};

template <int NS>
__global__ __launch_bounds__(256) void atq_stage_kernel(StageArgs A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane >> 4, l = lane & 15;
  const int i = blockIdx.x * ROWS_PER_WG + wave * ROWS_PER_WAVE + r;
  const bool valid = i < A.n;
  Row<NS> R;
  R.l = l;
  R.b = A.b;
  float S1[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int k = l + 16 * s;
    R.w[s] = (valid && k < A.b) ? A.W[(long)i * A.ldw + k] : 0.0f;
    R.t[s] = (valid && k < A.b && A.mode != PT2Q_STAGE_INIT && A.mode != PT2Q_STAGE_ROUND &&
              A.mode != PT2Q_STAGE_FULL)
                 ? A.T[(long)i * A.ldt + k]
                 : 0.0f;
    S1[s] = (A.S1 && k < A.b) ? A.S1[k] : 0.0f;
  }
  float wsum = row_sum_w(R);
  float a = valid ? A.alpha[i] : 0.0f, m = valid ? A.mu[i] : 0.0f;
  int it = 0;
  bool write_t = true;
  switch (A.mode) {
    case PT2Q_STAGE_INIT:
      row_init(R, wsum, &a, &m);
      break;
    case PT2Q_STAGE_GRID:
      row_grid<false>(R, wsum, &a, &m);
      write_t = false;
      break;
    case PT2Q_STAGE_ROUND:
      row_round(R, a, m);
      break;
    case PT2Q_STAGE_ITF: {
      // Caller passes init (alpha, mu, T); zero_rows[0] holds the count of all-zero T rows.
      bool block_zero = (*A.zero_rows == A.n);
      if (!block_zero) it = row_itf<false>(R, wsum, A.max_iter, &a, &m);
      break;
    }
    case PT2Q_STAGE_AGA:
      row_aga(R, S1, *A.d, &a, &m);
      write_t = false;
      break;
    case PT2Q_STAGE_FULL: {
      bool zero = row_init(R, wsum, &a, &m);
      if (A.pass == 0) {
        if (valid && l == 0 && zero) atomicAdd(A.zero_rows, 1);
        return;
      }
      bool block_zero = (*A.zero_rows == A.n);
      if (!block_zero) it = row_itf<true>(R, wsum, A.max_iter, &a, &m);
      if (A.S1) row_aga(R, S1, *A.d, &a, &m);
      break;
    }
  }
  if (A.iters && lane == 0) atomicMax(A.iters, it);
  if (!valid) return;
  if (l == 0 && A.mode != PT2Q_STAGE_ROUND) {
    A.alpha[i] = a;
    A.mu[i] = m;
  }
  if (write_t) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (R.has(s)) A.T[(long)i * A.ldt + l + 16 * s] = R.t[s];
  }
}

// count of all-zero T rows (for the ITF stage's iteration-0 block check)
__global__ void count_zero_rows_kernel(const float* T, long ldt, int n, int b, int* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool z = true;
  for (int k = 0; k < b; ++k) z &= (T[(long)i * ldt + k] == 0.0f);
  if (z) atomicAdd(out, 1);
}

// ----------------------------------------------------------------- wide blocks (b > 512)
//
// Per-channel quantisation (block_size = m, BASELINE config 5) makes a block as wide as the
// layer (5120 .. 13824 columns): a row no longer fits in registers.  The lane mapping stays the
// narrow kernels' -- 4 rows per wave, the 16 lanes of a row own the columns k = l + 16 s -- so the
// SUM16 partials are one register per lane and bfly16 folds them: every value is bit-identical
// to the register-resident kernels and to the oracle.  Instead of holding the row, each pass
// STREAMS it: batches of 16 columns per lane (16 index loads, then 16 weight and 16 code loads
// in flight, then the 16 sequential updates).  Lane groups of a wave read 4 adjacent rows of one
// column (feature-major: 16 B of a line per row group, the rest of the line by the neighbouring
// waves of the workgroup through L1) or 64 B of one row (row-major).  The codes live in the
// output array T between passes.  Passes: sum(w); sum|w - mu|; init (writes T, also the first
// grid's partials); one pass per ITF iteration (round + the next grid's partials); AGA; E.
// waves per workgroup (4 rows each): pt2q_tuning().wide_waves (4 or 8), up to WIDE_WAVES_MAX
constexpr int WIDE_WAVES_MAX = 8;
inline int wide_waves() { return pt2q_tuning().wide_waves; }

struct WideArgs {
  int mode;          // PT2Q_STAGE_* ; BLOCK = fused init+ITF+AGA+E of the block loop
  const float* W;    // FM: Wt[col * ldw + i] (feature-major); RM: W[i * ldw + k]
  long ldw;
  int n, b;
  const int* blk;    // FM: b column indices (selection order); RM: unused
  const float* S1;
  const float* d;
  int max_iter;
  float* alpha;
  float* mu;
  void* T;           // FM: int8 Tt[col * ldt + i]; RM: float T[i * ldt + k]
  long ldt;
  float* Et;         // FM: b x lde error term, nullable
  long lde;
  int* iters;
  int* counters;     // [0] all-zero init rows, [1] workgroups done
  int pass;          // STAGE_FULL: 0 = init + count, 1 = finish
};
constexpr int MODE_BLOCK = 100;

// Storage layouts of a wide row (the policy of WideRow): where column c of row i lives in W and
// T, and their element types.  FM: the block loop's feature-major fp32 Wt / int8 Tt; RM<TI, TO>:
// row-major W of type TI (float / _Float16 / uint16_t bf16 bits, read as exact fp32) and T of type TO (fp32 codes for
// the per-method stage surface, int8 or fp32 for the per-channel block loop, which reads the
// caller's weights in place).
struct LayFM {
  static constexpr bool FM = true;
  PT2Q_DEV static float w(const WideArgs& A, long i, long c) { return A.W[c * A.ldw + i]; }
  PT2Q_DEV static float t(const WideArgs& A, long i, long c) { return (float)((const int8_t*)A.T)[c * A.ldt + i]; }
  PT2Q_DEV static void set_t(const WideArgs& A, long i, long c, float v) { ((int8_t*)A.T)[c * A.ldt + i] = (int8_t)v; }
};
PT2Q_DEV float to_f32(float x) { return x; }
PT2Q_DEV float to_f32(_Float16 x) { return (float)x; }
PT2Q_DEV float to_f32(uint16_t x) { return __uint_as_float(((uint32_t)x) << 16); }  // bf16 bits
template <class TI, class TO>
struct LayRM {
  static constexpr bool FM = false;
  PT2Q_DEV static float w(const WideArgs& A, long i, long c) {
    return to_f32(((const TI*)(const void*)A.W)[i * A.ldw + c]);
  }
  PT2Q_DEV static float t(const WideArgs& A, long i, long c) { return (float)((const TO*)A.T)[i * A.ldt + c]; }
  PT2Q_DEV static void set_t(const WideArgs& A, long i, long c, float v) { ((TO*)A.T)[i * A.ldt + c] = (TO)v; }
};
typedef LayRM<float, float> LayStage;

template <class L>
struct WideRow {
  const WideArgs& A;
  int i, l;  // row (clamped to 0 when invalid: reads stay in range), residue class
  bool valid;
  PT2Q_DEV float t(long c) const { return L::t(A, i, c); }
  PT2Q_DEV void set_t(long c, float v) const {
    if (valid) L::set_t(A, i, c, v);
  }

  // One streamed pass: f(k, c, w, t) for this lane's columns k = l + 16 s in s order (c = the
  // storage column of k, w / t = 0 on an invalid row; t only with TC).
  template <bool TC, typename F>
  PT2Q_DEV void pass(F&& f) const {
    const int b = A.b;
    for (int k0 = 0; k0 < b; k0 += 256) {
      long c[16];
      float w[16], tv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + 16 * u + l;
        const int kc = k < b ? k : 0;
        c[u] = (L::FM && A.blk) ? (long)A.blk[kc] : (long)kc;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) w[u] = L::w(A, i, c[u]);
      if constexpr (TC) {
#pragma unroll
        for (int u = 0; u < 16; ++u) tv[u] = t(c[u]);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + 16 * u + l;
        if (k < b) f(k, c[u], valid ? w[u] : 0.0f, TC && valid ? tv[u] : 0.0f);
      }
    }
  }
};

template <class L>
PT2Q_DEV float wide_sum_w(const WideRow<L>& R) {
  float p = 0.0f;
  R.template pass<false>([&](int, long, float w, float) { p = p + w; });
  return bfly16(p);
}

// ternary_init (quantizer.py:32-69): writes T; also returns the first grid's sums (row_grid's
// partials over the codes just written -- same values, same order).  Returns all-zero.
template <class L>
PT2Q_DEV bool wide_init(const WideRow<L>& R, float wsum, float* a, float* m, float* g) {
  const float fb = (float)R.A.b;
  const float mu = wsum / fb;
  float p = 0.0f;
  R.template pass<false>([&](int, long, float w, float) { p = p + fabsf(w - mu); });
  const float delta = 0.75f * (bfly16(p) / fb);
  float pn = 0.0f, pd = 0.0f, pwt = 0.0f, pt = 0.0f, pt2 = 0.0f;
  R.template pass<false>([&](int, long c, float w, float) {
    const float wc = w - mu;
    const float t = (wc > delta) ? 1.0f : ((wc < -delta) ? -1.0f : 0.0f);
    R.set_t(c, t);
    pn = fmaf(t, wc, pn);  // t * wc exact
    pd = pd + fabsf(t);
    pwt = fmaf(w, t, pwt);
    pt = pt + t;
    pt2 = fmaf(t, t, pt2);
  });
  const float num = bfly16(pn), cnt = bfly16(pd);
  g[0] = bfly16(pwt);
  g[1] = bfly16(pt);
  g[2] = bfly16(pt2);
  *a = num / clampmin(cnt);
  *m = mu;
  return cnt == 0.0f;
}

// build_optimal_grid (quantizer.py:71-108) from the folded sums
PT2Q_DEV void wide_grid(const float* g, float fb, float wsum, float* a, float* m) {
  const float den = clampmin(fb * g[2] - g[1] * g[1]);
  *a = (fb * g[0] - g[1] * wsum) / den;
  *m = (g[2] * wsum - g[1] * g[0]) / den;
}

// grid partials over the caller's T (the GRID / ITF stage entries, no preceding init pass): any
// values, so the plain rounded products of the oracle's grid_row (the fmaf form of the passes
// below is the same only for ternary codes)
template <class L>
PT2Q_DEV void wide_grid_pass(const WideRow<L>& R, float* g) {
  float pwt = 0.0f, pt = 0.0f, pt2 = 0.0f;
  R.template pass<true>([&](int, long, float w, float t) {
    pwt = pwt + w * t;
    pt = pt + t;
    pt2 = pt2 + t * t;
  });
  g[0] = bfly16(pwt);
  g[1] = bfly16(pt);
  g[2] = bfly16(pt2);
}

// flexible_round (quantizer.py:110-134) over the row, writing changed codes; accumulates the
// next grid's sums into g.  Returns whether this lane changed a code.
template <class L>
PT2Q_DEV bool wide_round_pass(const WideRow<L>& R, float a, float m, float* g) {
  const RoundTh th = round_th(clampmin(a));
  bool changed = false;
  float pwt = 0.0f, pt = 0.0f, pt2 = 0.0f;
  R.template pass<true>([&](int, long c, float w, float old) {
    const float nt = round_code(w - m, th);
    if (nt != old) {
      changed = true;
      R.set_t(c, nt);
    }
    pwt = fmaf(w, nt, pwt);  // exact product (row_grid)
    pt = pt + nt;
    pt2 = fmaf(nt, nt, pt2);
  });
  g[0] = bfly16(pwt);
  g[1] = bfly16(pt);
  g[2] = bfly16(pt2);
  return changed;
}

// iterative_ternary_fitting (quantizer.py:136-175), wave-level stop as row_itf; g holds the
// grid sums of the codes in T on entry.
template <class L>
PT2Q_DEV int wide_itf(const WideRow<L>& R, float wsum, int max_iter, float* a, float* m, float* g) {
  int it = 0;
  bool any = true;
  for (; it < max_iter; ++it) {
    if (!any) break;
    wide_grid(g, (float)R.A.b, wsum, a, m);
    const bool ch = wide_round_pass(R, *a, *m, g);
    any = __any(ch);
  }
  return it;
}

// activation_aware_grid_alignment (quantizer.py:177-248) given S1 and d
template <class L>
PT2Q_DEV void wide_aga(const WideRow<L>& R, const float* S1, float d, float* a, float* m) {
  float pv = 0.0f, pws = 0.0f, pwts = 0.0f, pt2s = 0.0f;
  R.template pass<true>([&](int k, long, float w, float t) {
    const float c = S1[k];
    pv = fmaf(t, c, pv);
    pws = fmaf(w, c, pws);
    pwts = fmaf(w * t, c, pwts);
    pt2s = fmaf(t * t, c, pt2s);
  });
  const float v = bfly16(pv), ws1 = bfly16(pws), wts1 = bfly16(pwts), t2s1 = bfly16(pt2s);
  const float v2 = v * v;
  const float den = clampmin(d * t2s1 - v2);
  *a = (d * wts1 - v * ws1) / den;
  *m = (t2s1 * ws1 - v * wts1) / den;
}

template <class L>
PT2Q_DEV WideRow<L> wide_row(const WideArgs& A) {
  const int lane = threadIdx.x & 63;
  const int i = ((int)blockIdx.x * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6)) * 4 + (lane >> 4);
  const bool valid = i < A.n;
  return WideRow<L>{A, valid ? i : 0, lane & 15, valid};
}

// Block-loop mode for this wave's 4 rows: init -> ITF -> AGA -> E.
template <class L>
PT2Q_DEV void wide_block_rows(const WideArgs& A, bool skip_itf, bool count_zero) {
  const WideRow<L> R = wide_row<L>(A);
  const float wsum = wide_sum_w(R);
  float a, m, g[3];
  const bool zero = wide_init(R, wsum, &a, &m, g);
  if (count_zero && R.valid && R.l == 0 && zero) atomicAdd(&A.counters[0], 1);
  int it = 0;
  if (!skip_itf) it = wide_itf(R, wsum, A.max_iter, &a, &m, g);
  if (A.S1) wide_aga(R, A.S1, *A.d, &a, &m);
  if (A.iters && (threadIdx.x & 63) == 0 && !skip_itf) atomicMax(A.iters, it);
  if (!R.valid) return;
  if (R.l == 0) {
    A.alpha[R.i] = a;
    A.mu[R.i] = m;
  }
  if (A.Et)
    R.template pass<true>([&](int k, long, float w, float t) { A.Et[(long)k * A.lde + R.i] = w - (a * t + m); });
}

template <class L>
__global__ __launch_bounds__(64 * WIDE_WAVES_MAX) void atq_wide_block_kernel(WideArgs A) {
  wide_block_rows<L>(A, false, true);
}

// whole-block T_init == 0 repair after the kernel boundary (see atq_finish_kernel)
template <class L>
__global__ __launch_bounds__(64 * WIDE_WAVES_MAX) void atq_wide_zero_fixup_kernel(WideArgs A) {
  if (A.counters[0] != A.n) return;
  if (A.iters && blockIdx.x == 0 && threadIdx.x == 0) *A.iters = 0;
  wide_block_rows<L>(A, true, false);
}

// the repair of a grouped per-channel launch: linear blockIdx.y (its rows past blockIdx.x's skip)
struct WideGroup {
  int count;
  WideArgs a[PT2Q_PC_GROUP_MAX];
};
template <class L>
__global__ __launch_bounds__(64 * WIDE_WAVES_MAX) void atq_wide_zero_fixup_group_kernel(WideGroup G) {
  const WideArgs& A = G.a[blockIdx.y];
  if (A.counters[0] != A.n) return;
  if ((int)blockIdx.x * (int)(blockDim.x >> 6) * 4 >= A.n) return;
  if (A.iters && blockIdx.x == 0 && threadIdx.x == 0) *A.iters = 0;
  wide_block_rows<L>(A, true, false);
}

// Per-method stages on row-major W / float T (quantizer.py surface) for b > 512.
__global__ __launch_bounds__(64 * WIDE_WAVES_MAX) void atq_wide_stage_kernel(WideArgs A) {
  const WideRow<LayStage> R = wide_row<LayStage>(A);
  const float wsum = wide_sum_w(R);
  float a = R.valid ? A.alpha[R.i] : 0.0f, m = R.valid ? A.mu[R.i] : 0.0f, g[3];
  int it = 0;
  bool write_am = true;
  switch (A.mode) {
    case PT2Q_STAGE_INIT:
      wide_init(R, wsum, &a, &m, g);
      break;
    case PT2Q_STAGE_GRID:
      wide_grid_pass(R, g);
      wide_grid(g, (float)A.b, wsum, &a, &m);
      break;
    case PT2Q_STAGE_ROUND:
      wide_round_pass(R, a, m, g);
      write_am = false;
      break;
    case PT2Q_STAGE_ITF:
      if (*A.counters != A.n) {
        wide_grid_pass(R, g);
        it = wide_itf(R, wsum, A.max_iter, &a, &m, g);
      }
      break;
    case PT2Q_STAGE_AGA:
      wide_aga(R, A.S1, *A.d, &a, &m);
      break;
    case PT2Q_STAGE_FULL: {
      const bool zero = wide_init(R, wsum, &a, &m, g);
      if (A.pass == 0) {
        if (R.valid && R.l == 0 && zero) atomicAdd(A.counters, 1);
        return;
      }
      if (*A.counters != A.n) it = wide_itf(R, wsum, A.max_iter, &a, &m, g);
      if (A.S1) wide_aga(R, A.S1, *A.d, &a, &m);
      break;
    }
  }
  if (A.iters && (threadIdx.x & 63) == 0) atomicMax(A.iters, it);
  if (R.valid && R.l == 0 && write_am) {
    A.alpha[R.i] = a;
    A.mu[R.i] = m;
  }
}

template <typename F>
int dispatch_ns(int b, F&& f) {
  if (b <= 128) return f(std::integral_constant<int, 8>{});
  if (b <= 256) return f(std::integral_constant<int, 16>{});
  if (b <= 512) return f(std::integral_constant<int, 32>{});
  return PT2Q_E_UNSUPPORTED;
}

}  // namespace

// ------------------------------------------------------------------- internal launchers

int pt2q_launch_atq_block(const float* Wt, long ldw, int n, const int* blk, int b,
                          const float* S1, const float* d, int max_iter, float* alpha, float* mu,
                          int8_t* Tt, long ldt, float* Et, long lde, int* iters, int* counters,
                          hipStream_t st, const float* Hinv, long ldh, const int* rem, int nr,
                          float* C, long ldc, int* iters_part, const float* G, long ldg,
                          int* s1sync, int* status, const Grp* grp) {
  const unsigned nz = grp_z(grp);
  const Grp g = grp_or_none(grp);
  if (nz > 1 && b > 512) return PT2Q_E_UNSUPPORTED;  // grouped launches: blocks <= 512 columns
  if (b > 512) {
    WideArgs WA{MODE_BLOCK, Wt, ldw, n, b, blk, S1, d, max_iter, alpha, mu, Tt, ldt, Et, lde,
                iters, counters, 0};
    const int wgrid = ceil_div(n, 4 * wide_waves());
    hipLaunchKernelGGL(atq_wide_block_kernel<LayFM>, dim3(wgrid), dim3(64 * wide_waves()), 0, st, WA);
    PT2Q_LAUNCH_CHECK();
    hipLaunchKernelGGL(atq_wide_zero_fixup_kernel<LayFM>, dim3(wgrid), dim3(64 * wide_waves()), 0, st, WA);
    PT2Q_LAUNCH_CHECK();
    if (Hinv && nr > 0) return pt2q_launch_ef_coeffs(Hinv, ldh, blk, b, rem, nr, C, ldc, st);
    return PT2Q_OK;
  }
  const int nS1 = (G && S1 && s1sync && b <= 128) ? ceil_div(b, 8) : 0;
  BlockArgs A{Wt, ldw, n, b, blk, S1, d, max_iter, alpha, mu, Tt, ldt, Et, lde, iters, counters, iters_part,
              G, ldg, nS1, s1sync, (float*)S1, (float*)d, status, pt2q_tuning().spin_cap_fallback,
              pt2q_tuning().atq_probe};
  // the EF coefficient workgroups (Hinv given, columns left): COEF_SPAN columns e of one k row each
  const int per_k = (Hinv && nr > 0) ? ceil_div(nr, COEF_SPAN) : 0;
  const CoeffArgs K{Hinv, ldh, rem, nr, b, C, ldc, per_k > 0 ? per_k : 1};
  const int cgrid = (pt2q_tuning().atq_probe & 2) ? 0 : per_k * b;
  return dispatch_ns(b, [&](auto ns) {
    constexpr int NS = decltype(ns)::value;
    // the six-wave variant only where it costs no spills: full 128-column blocks
    constexpr int OCC = NS == 8 ? 6 : 0;
    // 16-byte staged rows (block_rows_vec): full 128-column blocks, 16-byte aligned pieces
    const auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool vec = NS == 8 && b == 128 && pt2q_tuning().atq_vec && n % 16 == 0 && al16(Wt) && ldw % 4 == 0 &&
                     al16(Tt) && ldt % 16 == 0 && (!Et || (al16(Et) && lde % 4 == 0)) && g.ws % 16 == 0;
    const bool occ = !vec && OCC && b == 16 * NS && pt2q_tuning().atq_occ == 6;
    // row workgroups: RG groups of 4 rows per wave (atq_rg; 4 in the staged form)
    const int rg = vec ? 4 : occ ? atq_rg<NS, OCC>() : atq_rg<NS, 0>();
    const int grid = ceil_div(n, ROWS_PER_WG * rg);
    const dim3 gd(nz * (nS1 + grid + cgrid));
    if (b == 16 * NS) {
      if (vec)
        hipLaunchKernelGGL((atq_block_kernel<NS, true, 0, NS == 8>), gd, dim3(256), 0, st, A, g, K, grid, cgrid);
      else if (occ)
        hipLaunchKernelGGL((atq_block_kernel<NS, true, OCC>), gd, dim3(256), 0, st, A, g, K, grid, cgrid);
      else
        hipLaunchKernelGGL((atq_block_kernel<NS, true, 0>), gd, dim3(256), 0, st, A, g, K, grid, cgrid);
    } else {
      hipLaunchKernelGGL((atq_block_kernel<NS, false, 0>), gd, dim3(256), 0, st, A, g, K, grid, cgrid);
    }
    PT2Q_LAUNCH_CHECK();
    hipLaunchKernelGGL(atq_finish_kernel<NS>, dim3(1, 1, nz), dim3(256), 0, st, A, grid, g);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  });
}

// Per-channel block of the block loop (b = m > 512, one block of every column in ascending
// order): the wide ATQ on the caller's row-major W (wdtype f32 / f16 / bf16, read as exact fp32)
// writing T (tdtype int8 / f32, ld ldt) and alpha / mu (n) in place -- the same values, in the
// same order, as the feature-major wide path on the transposed copy (LayRM vs LayFM: only the
// addresses differ).  counters[0] (zero rows) and *iters are zeroed by the caller.
int pt2q_launch_atq_wide_rm(const void* W, int wdtype, long ldw, int n, int b, const float* S1, const float* d,
                            int max_iter, float* alpha, float* mu, void* T, int tdtype, long ldt, int* iters,
                            int* counters, hipStream_t st) {
  WideArgs WA{MODE_BLOCK, (const float*)W, ldw, n, b, nullptr, S1, d, max_iter, alpha, mu, T, ldt, nullptr, 0,
              iters, counters, 0};
  const int wgrid = ceil_div(n, 4 * wide_waves());
  const bool pc = pt2q_atq_pc_supported(W, wdtype, ldw, b);  // codes held on-chip (atq_pc.hip)
  auto go = [&](auto lay) {
    typedef decltype(lay) L;
    if (pc) {
      const int rc = pt2q_launch_atq_pc(W, wdtype, ldw, n, b, S1, d, max_iter, alpha, mu, T, tdtype, ldt, iters,
                                        counters, st);
      if (rc != PT2Q_OK) return rc;
    } else {
      hipLaunchKernelGGL(atq_wide_block_kernel<L>, dim3(wgrid), dim3(64 * wide_waves()), 0, st, WA);
      PT2Q_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(atq_wide_zero_fixup_kernel<L>, dim3(wgrid), dim3(64 * wide_waves()), 0, st, WA);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  };
  const bool i8 = tdtype == PT2Q_I8;
  switch (wdtype) {
    case PT2Q_F32: return i8 ? go(LayRM<float, int8_t>{}) : go(LayRM<float, float>{});
    case PT2Q_F16: return i8 ? go(LayRM<_Float16, int8_t>{}) : go(LayRM<_Float16, float>{});
    case PT2Q_BF16: return i8 ? go(LayRM<uint16_t, int8_t>{}) : go(LayRM<uint16_t, float>{});
  }
  return PT2Q_E_ARG;
}

// Grouped per-channel blocks (pt2q_quantize_perchannel_group): the rows of every linear in one
// atq_pc launch when the streamed / register kernels take them all (else each linear on the wide
// kernel), then one repair launch for the group (grid.y = linear).  The same per-row programs as
// pt2q_launch_atq_wide_rm: the same bits.
int pt2q_launch_atq_rm_group(int count, const PcLinear* lin, int wdtype, int m, int max_iter, int tdtype,
                             hipStream_t st) {
  if (count <= 0 || count > PT2Q_PC_GROUP_MAX) return PT2Q_E_ARG;
  bool pc = true;
  int nmax = 0;
  for (int z = 0; z < count; ++z) {
    pc = pc && pt2q_atq_pc_supported(lin[z].W, wdtype, lin[z].ldw, m);
    nmax = std::max(nmax, lin[z].n);
  }
  WideGroup G{};
  G.count = count;
  for (int z = 0; z < count; ++z) {
    const PcLinear& L = lin[z];
    G.a[z] = WideArgs{MODE_BLOCK, (const float*)L.W, L.ldw, L.n, m, nullptr, L.S1, L.d, max_iter, L.alpha, L.mu,
                      L.T, L.ldt, nullptr, 0, L.iters, L.counters, 0};
  }
  const int wgrid = ceil_div(nmax, 4 * wide_waves());
  auto go = [&](auto lay) {
    typedef decltype(lay) L;
    if (pc) {
      const int rc = pt2q_launch_atq_pc_group(count, lin, wdtype, m, max_iter, tdtype, st);
      if (rc != PT2Q_OK) return rc;
    } else {
      for (int z = 0; z < count; ++z) {
        hipLaunchKernelGGL(atq_wide_block_kernel<L>, dim3(ceil_div(lin[z].n, 4 * wide_waves())),
                           dim3(64 * wide_waves()), 0, st, G.a[z]);
        PT2Q_LAUNCH_CHECK();
      }
    }
    hipLaunchKernelGGL(atq_wide_zero_fixup_group_kernel<L>, dim3(wgrid, count), dim3(64 * wide_waves()), 0, st, G);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  };
  const bool i8 = tdtype == PT2Q_I8;
  switch (wdtype) {
    case PT2Q_F32: return i8 ? go(LayRM<float, int8_t>{}) : go(LayRM<float, float>{});
    case PT2Q_F16: return i8 ? go(LayRM<_Float16, int8_t>{}) : go(LayRM<_Float16, float>{});
    case PT2Q_BF16: return i8 ? go(LayRM<uint16_t, int8_t>{}) : go(LayRM<uint16_t, float>{});
  }
  return PT2Q_E_ARG;
}

extern "C" int pt2q_atq_stage(int mode, const float* W, int64_t ldw, int n, int b, float* alpha,
                              float* mu, float* T, int64_t ldt, const float* S1,
                              const float* d_dev, int max_iter, int* iters_dev, void* workspace,
                              size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0 || b <= 0 || !W || !alpha || !mu || !T) return PT2Q_E_ARG;
  if ((mode == PT2Q_STAGE_AGA) && (!S1 || !d_dev)) return PT2Q_E_ARG;
  if ((mode == PT2Q_STAGE_ITF || mode == PT2Q_STAGE_FULL) &&
      (!workspace || workspace_bytes < sizeof(int)))
    return PT2Q_E_WORKSPACE;
  int* zero_rows = (int*)workspace;
  const float* Wp = W;
  int grid = ceil_div(n, ROWS_PER_WG);
  StageArgs A{mode, W, ldw, n, b, alpha, mu, T, ldt, S1, d_dev, max_iter, iters_dev, zero_rows, 0};
  if (iters_dev && (mode == PT2Q_STAGE_ITF || mode == PT2Q_STAGE_FULL))
    if (hipMemsetAsync(iters_dev, 0, sizeof(int), st) != hipSuccess) return PT2Q_E_HIP;
  if (mode == PT2Q_STAGE_ITF) {
    if (hipMemsetAsync(zero_rows, 0, sizeof(int), st) != hipSuccess) return PT2Q_E_HIP;
    hipLaunchKernelGGL(count_zero_rows_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, T, ldt,
                       n, b, zero_rows);
    PT2Q_LAUNCH_CHECK();
  }
  if (b > 512) {
    WideArgs WA{mode, Wp, ldw, n, b, nullptr, S1, d_dev, max_iter, alpha, mu, T,
                ldt, nullptr, 0, iters_dev, zero_rows, 0};
    const int wgrid = ceil_div(n, 4 * wide_waves());
    if (mode == PT2Q_STAGE_FULL) {
      if (hipMemsetAsync(zero_rows, 0, sizeof(int), st) != hipSuccess) return PT2Q_E_HIP;
      hipLaunchKernelGGL(atq_wide_stage_kernel, dim3(wgrid), dim3(64 * wide_waves()), 0, st, WA);
      PT2Q_LAUNCH_CHECK();
      WA.pass = 1;
    }
    hipLaunchKernelGGL(atq_wide_stage_kernel, dim3(wgrid), dim3(64 * wide_waves()), 0, st, WA);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  return dispatch_ns(b, [&](auto ns) {
    constexpr int NS = decltype(ns)::value;
    if (mode == PT2Q_STAGE_FULL) {
      if (hipMemsetAsync(zero_rows, 0, sizeof(int), st) != hipSuccess) return PT2Q_E_HIP;
      StageArgs A0 = A;
      A0.pass = 0;
      hipLaunchKernelGGL(atq_stage_kernel<NS>, dim3(grid), dim3(256), 0, st, A0);
      PT2Q_LAUNCH_CHECK();
      A.pass = 1;
    }
    hipLaunchKernelGGL(atq_stage_kernel<NS>, dim3(grid), dim3(256), 0, st, A);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  });
}
