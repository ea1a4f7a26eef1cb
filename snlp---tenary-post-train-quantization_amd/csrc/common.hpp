// Shared device helpers for libpt2q (gfx950 / CDNA4, wave64).
//
// PT2Q arithmetic contract: this whole library is compiled with
// -ffp-contract=off, so `a * b + c` is always two roundings; fused multiply-adds appear only
// where the contract says so, written as fmaf() or as an f32 MFMA (which is a k-ordered fmaf
// chain on gfx950, tools/probe_numerics.hip).  The reductions below define the canonical
// orders that oracle/pt2q_oracle.c restates on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt2q.h"

#define PT2Q_DEV __device__ __forceinline__

// clamp(min=1e-8) with torch semantics (NaN propagates): quantizer.py:66,100,125,240.
PT2Q_DEV float clampmin(float x) { return (x < 1e-8f) ? 1e-8f : x; }

// flexible_round's code of RN(d / as) at the ±0.5 thresholds (quantizer.py:127-131), decided
// exactly with no division.  RN(x) > 0.5 iff x > 0.5 + 2^-25 (that midpoint to the next float
// rounds to even, i.e. to 0.5), so the code is sign(d) iff |d| - as/2 > as * 2^-25 in exact
// arithmetic.  as/2 and as * 2^-25 are exact (as >= 1e-8 by the clamp); the float |d| - as/2 is
// exact whenever as/4 <= |d| <= as (Sterbenz), and outside that range its rounding cannot cross
// as * 2^-25.  NaN / inf operands give the division's codes (0 for a NaN quotient).  Checked
// against the correctly rounded division on 1.2e8 pairs within 40 ulp of the thresholds
// (tests/test_oracle.py::test_round_threshold_rule).
struct RoundTh {
  float hs, eps;
};
PT2Q_DEV RoundTh round_th(float as) { return {as * 0.5f, as * 0x1p-25f}; }
PT2Q_DEV float round_code(float d, RoundTh th) {
  return (fabsf(d) - th.hs > th.eps) ? copysignf(1.0f, d) : 0.0f;
}

// The value of lane (this lane ^ K), K in {1, 2, 4, 8}, by DPP inside a row of 16 lanes (no
// trip through the LDS crossbar as ds_bpermute takes): xor 1 / 2 are quad permutations, xor 8 a
// row rotation by 8, xor 4 two row shifts by 4 into alternate banks of 4 lanes.  All lanes active.
template <int K>
PT2Q_DEV float xor_lane(float p) {
  const int v = __float_as_int(p);
  int r;
  if constexpr (K == 1) {
    r = __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  } else if constexpr (K == 2) {
    r = __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  } else if constexpr (K == 8) {
    r = __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, true);  // row_ror:8
  } else {
    static_assert(K == 4, "xor_lane: K in {1, 2, 4, 8}");
    r = __builtin_amdgcn_update_dpp(0, v, 0x104, 0xF, 0x5, false);  // banks 0, 2: row_shl:4
    r = __builtin_amdgcn_update_dpp(r, v, 0x114, 0xF, 0xA, false);  // banks 1, 3: row_shr:4
  }
  return __int_as_float(r);
}

// xor_lane<4> for a value already symmetric under xor 8 (p[l] == p[l ^ 8], as after a butterfly's
// xor-8 step): the row rotation by 4 (lane (l + 4) mod 16) then delivers the value of lane l ^ 4,
// one DPP move instead of two bank-masked shifts.
PT2Q_DEV float xor4_sym8(float p) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(p), 0x124, 0xF, 0xF, true));  // row_ror:4
}

// Butterfly over the 16 lanes of a lane group (xor 8,4,2,1): every lane ends with the same sum.
PT2Q_DEV float bfly16(float p) {
  p = p + xor_lane<8>(p);
  p = p + xor4_sym8(p);
  p = p + xor_lane<2>(p);
  p = p + xor_lane<1>(p);
  return p;
}

// Butterfly over a whole wave64 (xor 32..1).
PT2Q_DEV float bfly64(float p) {
  p = p + __shfl_xor(p, 32);
  p = p + __shfl_xor(p, 16);
  return bfly16(p);
}

// SUMN partial for one lane t over a logical vector v[0..n): elements {256u + 4t + q} in
// ascending order (float4-per-lane pattern).  `fma_sq` selects p = fmaf(x, x, p).
template <bool FMA_SQ>
PT2Q_DEV float sumn_lane(const float* v, long n, long stride, int t) {
  float p = 0.0f;
  for (long base = 4 * t; base < n; base += 256) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      long i = base + q;
      if (i < n) {
        float x = v[i * stride];
        p = FMA_SQ ? fmaf(x, x, p) : p + x;
      }
    }
  }
  return p;
}

// SUMN of v[0..n) (stride) for a whole workgroup: the vector is first staged in LDS with every
// lane's loads in flight at once (lds >= n floats), then lanes 0..63 reduce it in the canonical
// order.  The result is returned to every thread.  Call from all threads of the block.
template <bool FMA_SQ>
PT2Q_DEV float block_sumn_lds(const float* v, long n, long stride, float* lds, float* out_slot) {
  for (long i = threadIdx.x; i < n; i += blockDim.x) lds[i] = v[i * stride];
  __syncthreads();
  if (threadIdx.x < 64) {
    float p = sumn_lane<FMA_SQ>(lds, n, 1, threadIdx.x);
    p = bfly64(p);
    if (threadIdx.x == 0) *out_slot = p;
  }
  __syncthreads();
  return *out_slot;
}

constexpr int SUMN_LDS_MAX = 12288;  // floats staged in LDS by block_sumn_lds users (48 KiB)

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// ---- Launch configuration fixed at library load.
// The production path has no tunables; these development overrides (PT2Q_* environment
// variables, used only by the tools/ probes) are read ONCE when libpt2q.so is loaded, never in a
// launch path.  Defaults are the measured best configuration.
struct Pt2qTuning {
  int gram_super = 0;          // PT2Q_GRAM_SUPER: 16-bit Gram super-block side (0: by m)
  int gram_groups = 8;         // PT2Q_GRAM_GROUPS: XCD groups of the 16-bit Gram split
  int gram_cus = 0;            // PT2Q_GRAM_CUS: CUs the batched Gram may hold (0: all)
  bool gram_split = true;      // PT2Q_GRAM_STREAMK=0: one chain per tile, no split
  bool gram_pair = true;       // PT2Q_GRAM_PAIR=0: no tile-pair teams
  bool gram_dp = true;         // PT2Q_GRAM_DP=0: no data-parallel waves
  bool gram_wide = true;       // PT2Q_GRAM_WIDE=0: no 256 x 256 tiles
  int gram_seglen = 0;         // PT2Q_GRAM_SEGLEN: f32 stream-K segment override
  int gemm_tile = 0;           // PT2Q_GEMM_TILE: 1 = 128x128, 6 = 64x64
  bool rank_update = true;     // PT2Q_RANK_UPDATE=0: generic grouped GEMM for Cholesky updates
  bool chol_lookahead = true;  // PT2Q_CHOL_LOOKAHEAD=0: the trailing updates on the main stream only
  int chol_panel = 0;          // PT2Q_CHOL_PANEL: rows per rank-P Cholesky update (0: by m)
  int chol_subpanel = 256;     // PT2Q_CHOL_SUBPANEL: rank-64 strip updates only inside sub-panels of
                               // this many rows, rank-SP updates (gemmx) to the rest of the panel (0: off)
  bool wbar_fused = true;      // PT2Q_WBAR_FUSED=0: three SSR-mean launches
  bool ef_wbar = true;         // PT2Q_EF_WBAR=0: the SSR mean pass reads W again (no EF partials)
  bool sim_split = true;       // PT2Q_SIM_SPLIT=0: one wave per column for n > 4096 (256 VGPRs)
  int gemmx_stages = 2;        // PT2Q_GEMMX_STAGES: LDS stages of the f32 chain GEMM (2: 64 KiB, 2 WGs per CU;
                               // batched inverse 596 -> 534 ms per 7B step vs 3)
  bool chol_lane = true;       // PT2Q_CHOL_LANE=0: the four-lanes-per-column panel / in-block inverse
  bool gemmx_gram = true;      // PT2Q_GEMMX_GRAM=0: batched f32 Grams on the generic GEMM
  bool s1_in_atq = true;       // PT2Q_S1_IN_ATQ=0: S1/d in the top-k launch
  bool ef_kernel = true;       // PT2Q_EF_GEMM=0: error feedback through the generic GEMM
  int ef_v2 = 1;               // PT2Q_EF_V2: 1 = ef2_gemm_kernel (two workgroups per CU, default), 0 = ef_gemm_kernel
  bool ef2_g1lds = true;       // PT2Q_EF2_G1LDS=0: column group 1's old values loaded in the epilogue
  int ef2_per_cu = 2;          // PT2Q_EF2_PER_CU: ef2 workgroups per CU (1 or 2)
  int ef2_teams = 1;           // PT2Q_EF2_TEAMS: 2 = one 8-wave workgroup of two barrier-coupled teams per CU
  int ef2_team_offset = 5;     // PT2Q_EF2_TEAM_OFFSET: barriers team 1 starts behind team 0
  int ef2_stagger = 0;         // PT2Q_EF2_STAGGER: ef2 start de-phasing (0: off)
  int ef2_probe = 0;           // PT2Q_EF2_PROBE: ef2 knock-out mask (tools only; results garbage)
  int atq_probe = 0;           // PT2Q_ATQ_PROBE (DEV_PROBES builds only; results garbage): block-ATQ
                               // knock-outs, 1 = rows skip the S1 wait, 2 = no coefficient workgroups,
                               // 4 = rows skip ITF, 8 / 128 / 256 = no code / error-term / scale
                               // stores, 16 = no S1 workgroups, 32 = no row gathers, 64 = idle rows
  bool gram_order = true;      // PT2Q_GRAM_ORDER=0: batched Gram in the super-block tile order
  bool atq_vec = true;         // PT2Q_ATQ_VEC=0: 128-column block ATQ with per-element row stores
  int wide_waves = 4;          // PT2Q_WIDE_WAVES: waves (4 rows each) per wide-ATQ workgroup (4 or 8)
  int atq_occ = 6;             // PT2Q_ATQ_OCC: block-ATQ waves per SIMD floor (6, or 0: compiler's)
  bool atq_pc = true;          // PT2Q_ATQ_PC=0: per-channel rows on the old streaming wide kernel
  bool atq_pc_regs = true;     // PT2Q_ATQ_PC_REGS=0: m = 5120 rows streamed like the others
  // Cross-workgroup waits poll at most this many times (each poll sleeps ~64-128 cycles), i.e.
  // seconds, before they give up and report PT2Q_E_STALL.  PT2Q_DEBUG_SPIN_CAP overrides both
  // (0: every hand-off reports a stall -- tests force the reporting path with it).
  long spin_cap_long = 1l << 28;   // Gram partial-tile hand-offs (a long chain may be in flight)
  long spin_cap_short = 1l << 26;  // in-launch hand-offs (S1 / d, top-k picks)
  long spin_cap_fallback = 1l << 13;  // ATQ S1 / d wait: polls before the wave forms S1 / d itself
};
const Pt2qTuning& pt2q_tuning();  // api.hip

// ---- Stall reporting.
// Every call that takes a workspace reserves its first PT2Q_STATUS_BYTES (pt2q.h) for a status
// word (int, zeroed by the call).  A wait on another workgroup that gives up ORs its bit into that
// word instead of carrying on silently; the host reads it after the stream completes and raises
// PT2Q_E_STALL (_lib.check_status).
enum : int { STALL_GRAM = 0x1, STALL_ATQ_S1 = 0x2, STALL_TOPK = 0x4 };

// Poll *flag until it is >= v.  Returns false (and marks *status) if the wait gave up after `cap`
// polls.  Call from one thread; the caller orders the data it then reads (fence / sc1 loads).
// cap == 0 is the test setting: every hand-off reports a stall, ready or not, so the reporting
// path is exercised deterministically.
template <int SLEEP>
PT2Q_DEV bool wait_flag_ge(const int* flag, int v, long cap, int* status, int bit) {
  if (cap == 0) {
    if (status) atomicOr(status, bit);
    return false;
  }
  long spins = 0;
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
    if (++spins > cap) {
      if (status) atomicOr(status, bit);
      return false;
    }
    __builtin_amdgcn_s_sleep(SLEEP);
  }
  return true;
}

#define PT2Q_LAUNCH_CHECK()                                      \
  do {                                                           \
    if (hipGetLastError() != hipSuccess) return PT2Q_E_HIP;      \
  } while (0)
