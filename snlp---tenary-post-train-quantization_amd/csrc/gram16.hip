// 16-bit-input Gram G = XᵀX on the 16-bit MFMA (gfx950 v_mfma_f32_32x32x16_{f16,bf16}).
//
// main.py:128 (H = X.T @ X over the calibration activations) and gptq.py:75 (add_batch) for
// fp16/bf16 activations.  The arithmetic is the instruction's own: per output element, each
// MFMA consumes k in two groups of 8 with one rounding per group (the model restated by
// oracle/pt2q_oracle.c orc_gram16 and checked against the hardware by
// tests/golden/mfma16_probe.npz).  The chain runs over X's rows in ascending groups of 8, so
// splitting K at multiples of 64 (stream-K pieces, batches continued with accumulate=2) does
// not change a bit.
//
// Work: 128 x 256 output tiles (4 waves, 2 x 2, each 64 x 128 = 2 x 4 MFMA tiles of 32 x 32)
// over the upper triangle, column-block major.  Operands: the k-rows of X's column panels go
// global -> LDS by LDS-DMA (16 B per lane, 3-stage ring of 64 rows) into a row-major image
// whose 16-byte chunks are XOR-swizzled by (row & 3) << 2; each lane then gathers its MFMA
// operand (8 k-consecutive elements of one column) with two ds_read_b64_tr_b16 — conflict-free
// under that swizzle.  Static balanced split of the tile-major work line over one workgroup
// per CU (each tile split at most once; the continuing piece waits on the previous workgroup).
#include "common.hpp"
#include "internal.hpp"
#include "probe.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int GX_BM = 128, GX_BN = 256, GX_BK = 64, GX_NS = 3;
constexpr int GX_AROW = 2 * GX_BM;          // 256 B per k-row of the A panel
constexpr int GX_BROW = 2 * GX_BN;          // 512 B per k-row of the B panel
constexpr int GX_ASTG = GX_BK * GX_AROW;    // 16 KiB
constexpr int GX_BSTG = GX_BK * GX_BROW;    // 32 KiB
constexpr int GX_STG = GX_ASTG + GX_BSTG;   // 48 KiB per stage
constexpr int GX_LDS = GX_NS * GX_STG;      // 144 KiB
constexpr int GX_DMA_PER_STAGE = 12;        // LDS-DMA wave-instructions per wave per stage

__device__ uint4 gx_zero16;  // the source of out-of-range chunks (zero-initialised)

// Upper tiles of the BM x BN grid (BN = RATIO * BM; tile (ti, tj) exists iff ti < RATIO (tj + 1))
// ordered by super-blocks of (RATIO SJ) x SJ tiles (column-block major over super-blocks, column
// major inside one), so that a contiguous run of the order -- one XCD's share -- covers a
// compact square of G and its workgroups read few distinct panels of X through their common L2.
template <int RATIO>
PT2Q_DEV int gx_col_count(int tj, int lo, int hi) {  // tiles ti in [lo, hi) of column tj
  return max(0, min(hi, RATIO * (tj + 1)) - lo);
}

template <int RATIO>
PT2Q_DEV void gx_tile(int a, int TI, int TJ, int SJ, int& ti, int& tj) {
  const int SI = RATIO * SJ;
  for (int J = 0; J * SJ < TJ; ++J) {
    const int tj1 = min(TJ, (J + 1) * SJ);
    for (int I = 0; I * SI < TI; ++I) {
      const int lo = I * SI, hi = min(TI, lo + SI);
      int c = 0;
      for (int t = J * SJ; t < tj1; ++t) c += gx_col_count<RATIO>(t, lo, hi);
      if (a >= c) {
        a -= c;
        continue;
      }
      for (int t = J * SJ; t < tj1; ++t) {
        const int ct = gx_col_count<RATIO>(t, lo, hi);
        if (a < ct) {
          ti = lo + a;
          tj = t;
          return;
        }
        a -= ct;
      }
    }
  }
  ti = tj = 0;  // unreachable for a < gx_ntile
}

long gx_ntile(int TI, int TJ, int ratio) {
  long s = 0;
  for (int t = 0; t < TJ; ++t) s += std::min(ratio * (t + 1), TI);
  return s;
}
long gx_ntile(int m) { return gx_ntile(ceil_div(m, GX_BM), ceil_div(m, GX_BN), GX_BN / GX_BM); }

// The work split of both 16-bit Gram kernels over one workgroup per CU.
// D data-parallel waves first: in wave v workgroup w = x + NG*r takes whole tile
// v*grid + x*R + r, so the R workgroups of one XCD run 32 neighbouring tiles of the order at the
// same k and share their X panels through that XCD's L2.  The rest of the tile line (stream-K)
// is cut into NG contiguous groups; group x is worked by workgroups w = x, x + NG, x + 2NG, ...
// (R of them), which on the round-robin dispatch share an XCD and so its L2 (speed only).
// Inside a group, team r/P takes rows [team*L, (team+1)*L) of the group's line of cnt * Kp rows
// (units of P tiles): tail piece first (chains from the start of its last unit), full units,
// then the head piece of its first unit, continuing the partial that the same member of the
// previous team (w - P*NG, dispatched earlier) published.  L >= Kp.  NG = 1 and L = Kp: no split.
// Forward progress of that wait: a workgroup only ever waits on a LOWER blockIdx (w - P*NG),
// the dispatcher hands workgroups out in blockIdx order (round-robin over the XCDs, in order
// within each XCD), and P*NG is a multiple of the 8 XCDs, so the producer sits on the waiter's
// own XCD, earlier in that XCD's queue: it was resident before the waiter took a slot and it
// waits, in turn, only on still lower indices -- induction from w < P*NG, which waits on nobody.
// The argument needs no co-residency of the grid.  Should the order ever be violated, the wait
// gives up after the spin cap, sets STALL_GRAM in the status word and the host raises
// Pt2qError (no hang, no silent result); a consumer-side recompute is not possible since the
// producer's partial lives only in C.  The batched Gram of a step (gram16b_kernel, the bench
// and GramsFirst default) is purely data parallel and has no such wait at all.
// P = 2: the line is cut into tile pairs (2j, 2j+1), which share their column block tj, and
// workgroups r = 2i, 2i+1 (a team) walk the same stretch of pairs in step, one tile of each
// pair apiece, so the X panel of tj is fetched into L2 once for both.
struct GxSched {
  long base, t0;
  int D, R, P, x, r, mem, Kp, a0, a1, k0, k1, f0, npieces;
  bool head, tail;

  PT2Q_DEV GxSched(long ntile, int Kp_, int NG, int R_, int P_, int D_) : D(D_), R(R_), P(P_), Kp(Kp_) {
    const int w = blockIdx.x;
    x = w % NG;
    r = w / NG;
    base = (long)D * gridDim.x;  // first stream-K tile
    mem = r % P;
    const int team = r / P, nteam = R / P;
    const long npair = max(0l, (ntile - base) / P);
    t0 = P * (npair * x / NG);
    const long cnt = npair * (x + 1) / NG - npair * x / NG;
    const long W = cnt * Kp;
    const long L = (R == 0) ? Kp : ((W + nteam - 1) / nteam + GX_BK - 1) / GX_BK * GX_BK;
    const long s = (long)team * L, e = min(s + L, W);
    a0 = (int)(s / Kp);
    k0 = (int)(s % Kp);
    a1 = (int)((e - 1) / Kp);
    k1 = (int)(e - (long)a1 * Kp);
    head = k0 > 0;
    tail = k1 < Kp && !(head && a1 == a0);
    f0 = head ? a0 + 1 : a0;
    const int f1 = tail ? a1 - 1 : a1;
    const int nfull = f1 >= f0 ? f1 - f0 + 1 : 0;
    npieces = (s >= e || npair == 0) ? 0 : (tail ? 1 : 0) + nfull + (head ? 1 : 0);
  }

  // piece pc in [-D, npieces): global tile a (flags are per tile), rows [kb, ke), and whether it
  // continues a partial that another workgroup publishes
  PT2Q_DEV void piece(int pc, int& a, int& kb, int& ke, bool& from_partial) const {
    from_partial = false;
    if (pc < 0) {
      a = (pc + D) * (int)gridDim.x + x * R + r;
      kb = 0;
      ke = Kp;
      return;
    }
    if (tail && pc == 0) {
      a = a1; kb = 0; ke = k1;
    } else if (head && pc == npieces - 1) {
      a = a0; kb = k0; ke = (a0 == a1) ? k1 : Kp; from_partial = true;
    } else {
      a = f0 + pc - (tail ? 1 : 0); kb = 0; ke = Kp;
    }
    a = (int)(base + t0) + P * a + mem;
  }
};

template <bool DMA>
PT2Q_DEV void gx_copy16(const uint16_t* X, long ld, int gk, int kend, int gd, int M, uint8_t* blk,
                        int lane) {
  if constexpr (DMA) {
    const void* src = (gk < kend && gd < M) ? (const void*)(X + (long)gk * ld + gd) : (const void*)&gx_zero16;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)blk, 16, 0, 0);
  } else {
    uint16_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (gk < kend && gd + e < M) ? X[(long)gk * ld + gd + e] : (uint16_t)0;
    uint4 u;
    __builtin_memcpy(&u, v, 16);
    *(uint4*)(blk + lane * 16) = u;
  }
}

// One stage: k-rows [k0, k0+64) of the A panel (features i0..i0+127) and of the B panel
// (features j0..j0+255).  Physical chunk p of row r holds logical chunk p ^ ((r & 3) << 2).
template <bool DMA>
PT2Q_DEV void gx_stage(const uint16_t* X, long ld, int i0, int j0, int k0, int kend, int M,
                       uint8_t* stg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // A: 16 wave-instructions of 4 rows
    const int q = wave * 4 + j;
    const int row = q * 4 + (lane >> 4), c = (lane & 15) ^ ((row & 3) << 2);
    gx_copy16<DMA>(X, ld, k0 + row, kend, i0 + 8 * c, M, stg + q * 1024, lane);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // B: 32 wave-instructions of 2 rows
    const int q = wave * 8 + j;
    const int row = q * 2 + (lane >> 5), c = (lane & 31) ^ ((row & 3) << 2);
    gx_copy16<DMA>(X, ld, k0 + row, kend, j0 + 8 * c, M, stg + GX_ASTG + q * 1024, lane);
  }
}

// Fast staging (DMA path, whole stage in range): this lane's 12 chunk sources as byte offsets
// from the stage's first k-row (fixed for a piece), so each DMA is one global_load_lds with a
// scalar base and a 32-bit vector offset, and the LDS destination is wave-uniform (M0).
PT2Q_DEV void gx_voff(long ld, int i0, int j0, uint32_t (&vo)[12]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (wave * 4 + j) * 4 + (lane >> 4), c = (lane & 15) ^ ((row & 3) << 2);
    vo[j] = (uint32_t)(((long)row * ld + i0 + 8 * c) * 2);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = (wave * 8 + j) * 2 + (lane >> 5), c = (lane & 31) ^ ((row & 3) << 2);
    vo[4 + j] = (uint32_t)(((long)row * ld + j0 + 8 * c) * 2);
  }
}

// Quarter qq of a fast stage: A chunk j = qq, B chunks j = 2qq, 2qq + 1.
PT2Q_DEV void gx_stage_q(const uint16_t* Xk0, const uint32_t (&vo)[12], uint8_t* stg, int qq) {
  if constexpr (probe::gram_no_dma) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* sb = (const char*)Xk0;
  typedef __attribute__((address_space(3))) void* lptr;
  __builtin_amdgcn_global_load_lds((const void*)(sb + vo[qq]), (lptr)(stg + (wave * 4 + qq) * 1024), 16, 0, 0);
#pragma unroll
  for (int e = 0; e < 2; ++e)
    __builtin_amdgcn_global_load_lds((const void*)(sb + vo[4 + 2 * qq + e]),
                                     (lptr)(stg + GX_ASTG + (wave * 8 + 2 * qq + e) * 1024), 16, 0, 0);
}

// LDS reads are inline asm: hipcc cannot tell them apart from the LDS-DMA writes still in
// flight and would wait vmcnt(0) before the first read of every stage (cdna_hip_programming.md
// §5 trap 4a).  Ordering is by hand: counted vmcnt + raw barrier for the DMA, lgkmcnt(0) tied
// to the fragment registers before the MFMAs that use them.
template <int OFF>
PT2Q_DEV s16x4 gx_tr(uint32_t addr) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// The 12 transposed reads of one k16 step (rows 16S .. 16S+15 of the stage): per fragment 8
// k-consecutive elements of one column = two 4-row reads.
struct GxFrags {
  s16x4 lo[6], hi[6];  // 0, 1: A tiles mt; 2..5: B tiles nt
};

template <int S>
PT2Q_DEV void gx_read(GxFrags& f, const uint32_t (&addr)[6]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    f.lo[q] = gx_tr<S * 16 * GX_AROW>(addr[q]);
    f.hi[q] = gx_tr<S * 16 * GX_AROW + 4 * GX_AROW>(addr[q]);
  }
#pragma unroll
  for (int q = 2; q < 6; ++q) {
    f.lo[q] = gx_tr<S * 16 * GX_BROW>(addr[q]);
    f.hi[q] = gx_tr<S * 16 * GX_BROW + 4 * GX_BROW>(addr[q]);
  }
}

PT2Q_DEV void gx_wait(GxFrags& f) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(f.lo[0]), "+v"(f.lo[1]), "+v"(f.lo[2]), "+v"(f.lo[3]), "+v"(f.lo[4]),
                 "+v"(f.lo[5]), "+v"(f.hi[0]), "+v"(f.hi[1]), "+v"(f.hi[2]), "+v"(f.hi[3]),
                 "+v"(f.hi[4]), "+v"(f.hi[5]));
}

PT2Q_DEV s16x8 gx_cat(s16x4 lo, s16x4 hi) {
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <bool BF16>
PT2Q_DEV f32x16 gx_mfma(s16x8 a, s16x8 b, f32x16 c) {
  if constexpr (BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

struct GxTile {
  f32x16 acc[2][4];

  PT2Q_DEV static int row(int i0, int mt, int r) {
    const int lane = threadIdx.x & 63, wr = (threadIdx.x >> 6) >> 1;
    return i0 + wr * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
  }
  PT2Q_DEV static int col(int j0, int nt) {
    const int lane = threadIdx.x & 63, wc = (threadIdx.x >> 6) & 1;
    return j0 + wc * 128 + nt * 32 + (lane & 31);
  }

  template <bool BF16>
  PT2Q_DEV void mma(const GxFrags& f) {
    if constexpr (probe::gram_no_mfma) return;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = gx_mfma<BF16>(gx_cat(f.lo[mt], f.hi[mt]), gx_cat(f.lo[2 + nt], f.hi[2 + nt]),
                                    acc[mt][nt]);
    __builtin_amdgcn_s_setprio(0);
  }

  // continue the chains over X rows [kbeg, kend) (kbeg a multiple of 64)
  template <bool BF16, bool DMA>
  PT2Q_DEV void chain(const uint16_t* X, long ld, int M, int i0, int j0, int kbeg, int kend,
                      uint8_t* smem) {
    const int nk = (kend - kbeg + GX_BK - 1) / GX_BK;
    if (nk <= 0) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3, gh = (lane >> 4) & 1, h = lane >> 5;
    // byte offsets of this lane's first transposed read inside a stage, per MFMA tile
    int offA[2], offB[4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int cf = wr * 8 + mt * 4 + 2 * gh + (p >> 1);
      offA[mt] = (8 * h + q) * GX_AROW + ((cf ^ (q << 2)) << 4) + 8 * (p & 1);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int cf = wc * 16 + nt * 4 + 2 * gh + (p >> 1);
      offB[nt] = GX_ASTG + (8 * h + q) * GX_BROW + ((cf ^ (q << 2)) << 4) + 8 * (p & 1);
    }
    const bool fastcols = DMA && i0 + GX_BM <= M && j0 + GX_BN <= M;
    uint32_t vo[12];
    if (fastcols) gx_voff(ld, i0, j0, vo);
    gx_stage<DMA>(X, ld, i0, j0, kbeg, kend, M, smem);
    if (nk > 1) gx_stage<DMA>(X, ld, i0, j0, kbeg + GX_BK, kend, M, smem + GX_STG);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
    for (int t = 0; t < nk; ++t) {
      // stage t landed (this wave's DMAs; stage t+1 may stay in flight), then a raw barrier:
      // __syncthreads()'s fence would wait vmcnt(0) and drain the prefetch every step.  The
      // barrier also retires every wave's reads of stage t-1, whose slot stage t+2 reuses.
      if (t + 1 < nk)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GX_DMA_PER_STAGE) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
      // stage t+2 goes into the slot stage t-1 used, issued in quarters between the k16 steps
      const bool pre = t + 2 < nk;
      const int kn = kbeg + (t + 2) * GX_BK;
      uint8_t* stn = smem + ((t + 2) % GX_NS) * GX_STG;
      const bool fast = pre && fastcols && kn + GX_BK <= kend;
      const uint16_t* Xn = X + (long)kn * ld;
      if (pre && !fast) gx_stage<DMA>(X, ld, i0, j0, kn, kend, M, stn);
      const uint32_t base = lds0 + (uint32_t)((t % GX_NS) * GX_STG);
      uint32_t addr[6];
#pragma unroll
      for (int q = 0; q < 2; ++q) addr[q] = base + offA[q];
#pragma unroll
      for (int q = 0; q < 4; ++q) addr[2 + q] = base + offB[q];
      GxFrags f0, f1;
      gx_read<0>(f0, addr);
      gx_wait(f0);
      gx_read<1>(f1, addr);
      if (fast) gx_stage_q(Xn, vo, stn, 0);
      mma<BF16>(f0);
      gx_wait(f1);
      gx_read<2>(f0, addr);
      if (fast) gx_stage_q(Xn, vo, stn, 1);
      mma<BF16>(f1);
      gx_wait(f0);
      gx_read<3>(f1, addr);
      if (fast) gx_stage_q(Xn, vo, stn, 2);
      mma<BF16>(f0);
      gx_wait(f1);
      if (fast) gx_stage_q(Xn, vo, stn, 3);
      mma<BF16>(f1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the ring is reused by the next piece
  }
};

// ---- the hand-scheduled chain (LDS-DMA path of both tile shapes) -----------------------------
// BM x 256 output tiles, BM = 128 (gram16x_kernel) or 256 (gram16w_kernel: m % 256 == 0, at
// least two tile waves).  Per k-row a 128 x 256 tile reads 768 B of X for 65 536 MACs, a
// 256 x 256 tile 1 KiB for 131 072: a third fewer L2 -> LDS bytes per MFMA.  4 waves, 2 x 2,
// each (BM/2) x 128 = MT x 4 MFMA tiles (BM = 256: 256 accumulator registers, one wave per
// SIMD).  Stages of 32 k-rows in an NS-slot ring that fills the LDS (5 x 32 KiB / 6 x 24 KiB:
// 128 / 120 KiB in flight per CU, which L2-miss latency needs); panel rows carry the swizzle of
// gx_stage.  Stage t+NS-1 is issued during stage t.  Fragment reads and LDS-DMA issues are
// inline asm and every MFMA is followed by a full scheduling barrier, so each k16 step keeps
// exactly this interleaving: its MFMAs are spaced by the reads of the next step's fragment
// halves (two per MFMA gap, absorbed in the MFMA's shadow) and by the DMAs of half a future
// stage; the barrier that publishes the next stage sits after the step's first MFMA, so the
// MFMA pipe is busy while the waves meet.  (Compiler-scheduled, the same loop left the MFMA
// pipe idle half the time at m = 11008: 34.7 vs 30.0 ms.)
constexpr int GW_B = 256, GW_BK = 32;
constexpr int GW_ROW = 2 * GW_B;          // 512 B per k-row of a 256-feature panel (B, wide A)
constexpr int GW_PNL = GW_BK * GW_ROW;    // 16 KiB: a 256-feature panel of one stage

template <int BM>
struct GwGeo {
  static constexpr int MT = BM / 64;              // MFMA row tiles per wave
  static constexpr int AROW = 2 * BM;             // bytes per k-row of the A panel
  static constexpr int APNL = GW_BK * AROW;       // the A panel of one stage
  static constexpr int STG = APNL + GW_PNL;       // A panel, then B panel
  static constexpr int NS = BM == 256 ? 5 : 6;    // ring slots
  static constexpr int LDS = NS * STG;            // 160 / 144 KiB
  static constexpr int ADMA = APNL / 1024 / 4;    // A wave-instructions per wave per stage
  static constexpr int DMA = ADMA + 4;            // + B: LDS-DMA wave-instructions per wave per stage
  static constexpr int NF = MT + 4;               // fragments per k16 step
};

// lane's DMA chunk of wave-instruction q of a panel with `row` bytes per k-row: k-row, column
template <int ROWB>
PT2Q_DEV void gw_chunk(int q, int& row, int& c) {
  constexpr int LPR = ROWB / 16;  // lanes per k-row
  const int lane = threadIdx.x & 63;
  row = (64 / LPR) * q + lane / LPR;
  c = (lane % LPR) ^ ((row & 3) << 2);
}

// whole stage with per-lane sources: rows past kend and columns past M read the zero chunk
template <int BM>
PT2Q_DEV void gw_stage(const uint16_t* X, long ld, int M, int i0, int j0, int k0, int kend, uint8_t* stg) {
  if constexpr (probe::gram_no_dma) return;
  using G = GwGeo<BM>;
  const int wave = threadIdx.x >> 6;
  typedef __attribute__((address_space(3))) void* lptr;
#pragma unroll
  for (int j = 0; j < G::ADMA; ++j) {
    const int q = wave * G::ADMA + j;
    int row, c;
    gw_chunk<G::AROW>(q, row, c);
    const bool in = k0 + row < kend && i0 + 8 * c < M;
    __builtin_amdgcn_global_load_lds(in ? (const void*)(X + (long)(k0 + row) * ld + i0 + 8 * c) : (const void*)&gx_zero16,
                                     (lptr)(stg + q * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = wave * 4 + j;
    int row, c;
    gw_chunk<GW_ROW>(q, row, c);
    const bool in = k0 + row < kend && j0 + 8 * c < M;
    __builtin_amdgcn_global_load_lds(in ? (const void*)(X + (long)(k0 + row) * ld + j0 + 8 * c) : (const void*)&gx_zero16,
                                     (lptr)(stg + G::APNL + q * 1024), 16, 0, 0);
  }
}

// byte offsets of this lane's chunk sources from a stage's first k-row: A chunks, then B chunks
template <int BM>
PT2Q_DEV void gw_voff(long ld, int i0, int j0, uint32_t (&vo)[GwGeo<BM>::DMA]) {
  using G = GwGeo<BM>;
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < G::ADMA; ++j) {
    int row, c;
    gw_chunk<G::AROW>(wave * G::ADMA + j, row, c);
    vo[j] = (uint32_t)(((long)row * ld + i0 + 8 * c) * 2);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int row, c;
    gw_chunk<GW_ROW>(wave * 4 + j, row, c);
    vo[G::ADMA + j] = (uint32_t)(((long)row * ld + j0 + 8 * c) * 2);
  }
}

template <int NF>
struct GwFrags {
  s16x4 lo[NF], hi[NF];  // 0 .. NF-5: A tiles mt; NF-4 .. NF-1: B tiles nt
};

// wait until at most N LDS reads are outstanding (N <= 15: the counter's range), tying f
template <int N, int NF>
PT2Q_DEV void gw_wait(GwFrags<NF>& f) {
  if constexpr (NF == 8)
    asm volatile("s_waitcnt lgkmcnt(%16)"
                 : "+v"(f.lo[0]), "+v"(f.lo[1]), "+v"(f.lo[2]), "+v"(f.lo[3]), "+v"(f.lo[4]), "+v"(f.lo[5]),
                   "+v"(f.lo[6]), "+v"(f.lo[7]), "+v"(f.hi[0]), "+v"(f.hi[1]), "+v"(f.hi[2]), "+v"(f.hi[3]),
                   "+v"(f.hi[4]), "+v"(f.hi[5]), "+v"(f.hi[6]), "+v"(f.hi[7])
                 : "n"(N));
  else
    asm volatile("s_waitcnt lgkmcnt(%12)"
                 : "+v"(f.lo[0]), "+v"(f.lo[1]), "+v"(f.lo[2]), "+v"(f.lo[3]), "+v"(f.lo[4]), "+v"(f.lo[5]),
                   "+v"(f.hi[0]), "+v"(f.hi[1]), "+v"(f.hi[2]), "+v"(f.hi[3]), "+v"(f.hi[4]), "+v"(f.hi[5])
                 : "n"(N));
}

template <int N>
PT2Q_DEV void gw_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait for a stage while the y younger stages (0 <= y <= NS - 2) stay in flight
template <int D>
PT2Q_DEV void gw_vmwait_y(int y) {
  switch (y) {
    case 0: gw_vmwait<0>(); break;
    case 1: gw_vmwait<D>(); break;
    case 2: gw_vmwait<2 * D>(); break;
    case 3: gw_vmwait<3 * D>(); break;
    default: gw_vmwait<4 * D>(); break;
  }
}

template <bool BF16>
PT2Q_DEV void gw_mfma1(f32x16& acc, const s16x4& alo, const s16x4& ahi, const s16x4& blo, const s16x4& bhi) {
  if constexpr (!probe::gram_no_mfma) acc = gx_mfma<BF16>(gx_cat(alo, ahi), gx_cat(blo, bhi), acc);
  __builtin_amdgcn_sched_barrier(0);  // nothing moves across: the step's interleaving stays
}

// one 16-B LDS-DMA: global (sbase + voff) -> LDS m0 + 16 lane
PT2Q_DEV void gw_dma_asm(const char* sbase, uint32_t voff, uint32_t m0) {
  if constexpr (probe::gram_no_dma) return;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(m0)
               : "memory");  // (m0 is reserved: the compiler sets it afresh before its own DMAs)
}

struct GwDma {          // a future stage's LDS-DMAs
  const char* src;      // the stage's first k-row
  uint32_t mA, mB;      // LDS: this wave's first A chunk, first B chunk
};

// one k16 step: MFMAs on cur, the reads of nxt (byte offsets ROFFA / ROFFB from ra) in the gaps.
// SYNC: after the first MFMA wait for the stage the reads need (VM younger DMAs stay in flight;
// VM < 0: y younger whole stages, y at run time) and meet the other waves.  HALF >= 0: issue that half of a stage's
// DMAs.  No run-time branch between the MFMAs of a steady step (VM >= 0): a branch there makes
// the register allocator shuffle the accumulator registers.
template <int BM, bool BF16, int ROFFA, int ROFFB, bool SYNC, int VM, int HALF>
PT2Q_DEV void gw_step(f32x16 (&acc)[GwGeo<BM>::MT][4], const GwFrags<GwGeo<BM>::NF>& cur,
                      GwFrags<GwGeo<BM>::NF>& nxt, const uint32_t (&ra)[GwGeo<BM>::NF], int y, const GwDma& d,
                      const uint32_t (&vo)[GwGeo<BM>::DMA]) {
  using G = GwGeo<BM>;
  constexpr int NM = G::MT * 4, HD = G::DMA / 2;
  gw_mfma1<BF16>(acc[0][0], cur.lo[0], cur.hi[0], cur.lo[G::MT], cur.hi[G::MT]);
  if constexpr (SYNC) {
    if constexpr (VM >= 0)
      gw_vmwait<VM>();
    else
      gw_vmwait_y<G::DMA>(y);
    asm volatile("s_barrier" ::: "memory");
  }
#pragma unroll
  for (int i = 1; i < NM; ++i) {
    const int mt = i >> 2, nt = i & 3;
    gw_mfma1<BF16>(acc[mt][nt], cur.lo[mt], cur.hi[mt], cur.lo[G::MT + nt], cur.hi[G::MT + nt]);
    if (i <= G::NF) {
      const int q = i - 1;
      if (q < G::MT) {
        nxt.lo[q] = gx_tr<ROFFA>(ra[q]);
        nxt.hi[q] = gx_tr<ROFFA + 4 * G::AROW>(ra[q]);
      } else {
        nxt.lo[q] = gx_tr<ROFFB>(ra[q]);
        nxt.hi[q] = gx_tr<ROFFB + 4 * GW_ROW>(ra[q]);
      }
    }
    if constexpr (HALF >= 0) {
      if (i >= NM - HD) {
        const int e = HALF * HD + i - (NM - HD);  // chunk e of the stage: A chunks, then B
        if (e < G::ADMA)
          gw_dma_asm(d.src, vo[e], d.mA + e * 1024);
        else
          gw_dma_asm(d.src, vo[e], d.mB + (e - G::ADMA) * 1024);
      }
    }
  }
  gw_wait<0>(nxt);
}

// continue the chains of tile (i0, j0) over X rows [kbeg, kend) (kbeg a multiple of 32); a tile
// that crosses the matrix edge (full = false) takes every stage with per-lane sources
template <int BM, bool BF16>
PT2Q_DEV void gw_chain(f32x16 (&acc)[GwGeo<BM>::MT][4], const uint16_t* X, long ld, int M, int i0, int j0,
                       int kbeg, int kend, bool full, uint8_t* smem) {
  using G = GwGeo<BM>;
  constexpr int NS = G::NS;
  const int nk = (kend - kbeg + GW_BK - 1) / GW_BK;
  if (nk <= 0) return;
  const int nkf = (kend - kbeg) / GW_BK;  // whole stages
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3, gh = (lane >> 4) & 1, h = lane >> 5;
  uint32_t off[G::NF];
#pragma unroll
  for (int t = 0; t < G::MT; ++t) {
    const int ca = wr * 4 * G::MT + t * 4 + 2 * gh + (p >> 1);  // 16-B chunk of the A panel row
    off[t] = (8 * h + q) * G::AROW + ((ca ^ (q << 2)) << 4) + 8 * (p & 1);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int cb = wc * 16 + t * 4 + 2 * gh + (p >> 1);
    off[G::MT + t] = G::APNL + (8 * h + q) * GW_ROW + ((cb ^ (q << 2)) << 4) + 8 * (p & 1);
  }
  uint32_t vo[G::DMA];
  gw_voff<BM>(ld, i0, j0, vo);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) gw_stage<BM>(X, ld, M, i0, j0, kbeg + s * GW_BK, kend, smem + s * G::STG);
  gw_vmwait_y<G::DMA>(min(NS - 2, nk - 1));
  asm volatile("s_barrier" ::: "memory");
  uint32_t ra[G::NF];
#pragma unroll
  for (int u = 0; u < G::NF; ++u) ra[u] = lds0 + off[u];
  GwFrags<G::NF> P, Q;
#pragma unroll
  for (int u = 0; u < G::MT; ++u) {
    P.lo[u] = gx_tr<0>(ra[u]);
    P.hi[u] = gx_tr<4 * G::AROW>(ra[u]);
  }
#pragma unroll
  for (int u = G::MT; u < G::NF; ++u) {
    P.lo[u] = gx_tr<0>(ra[u]);
    P.hi[u] = gx_tr<4 * GW_ROW>(ra[u]);
  }
  gw_wait<0>(P);
  const uint32_t mwA = lds0 + (uint32_t)(wave * G::ADMA * 1024), mwB = lds0 + (uint32_t)(G::APNL + wave * 4 * 1024);
  constexpr int RA1 = 16 * G::AROW, RB1 = 16 * GW_ROW;  // rows 16..31 of a stage
  // steady state: stage t+NS-1 is a whole in-range stage, issued by the fast DMAs of both steps
  const int t1 = full ? max(0, nkf - (NS - 1)) : 0;
  int t = 0;
  for (; t < t1; ++t) {
    GwDma d;
    d.src = (const char*)(X + (long)(kbeg + (t + NS - 1) * GW_BK) * ld);
    const uint32_t so = (uint32_t)(((t + NS - 1) % NS) * G::STG);
    d.mA = mwA + so;
    d.mB = mwB + so;
    gw_step<BM, BF16, RA1, RB1, false, 0, 0>(acc, P, Q, ra, 0, d, vo);
    const uint32_t base = lds0 + (uint32_t)(((t + 1) % NS) * G::STG);
#pragma unroll
    for (int u = 0; u < G::NF; ++u) ra[u] = base + off[u];
    // in flight past stage t+1: stages t+2 .. t+NS-2 and the first half of t+NS-1 (step A's DMAs)
    gw_step<BM, BF16, 0, 0, true, (NS - 3) * G::DMA + G::DMA / 2, 1>(acc, Q, P, ra, 0, d, vo);
  }
  // the rest: per-lane sources (a ragged last stage, an edge tile) and a draining ring
  for (; t < nk; ++t) {
    if (t + NS - 1 < nk)
      gw_stage<BM>(X, ld, M, i0, j0, kbeg + (t + NS - 1) * GW_BK, kend, smem + ((t + NS - 1) % NS) * G::STG);
    GwDma d{};
    gw_step<BM, BF16, RA1, RB1, false, 0, -1>(acc, P, Q, ra, 0, d, vo);
    const uint32_t base = lds0 + (uint32_t)(((t + 1) % NS) * G::STG);
#pragma unroll
    for (int u = 0; u < G::NF; ++u) ra[u] = base + off[u];
    // (past the last stage: vmcnt(0), a barrier and reads of a stale slot, never used)
    gw_step<BM, BF16, 0, 0, true, -1, -1>(acc, Q, P, ra, max(0, min(t + NS - 1, nk - 1) - (t + 1)), d, vo);
  }
  asm volatile("s_barrier" ::: "memory");  // the ring is reused by the next piece
}

// g: M = N = m, K = rows, A = X (ld lda), C = G (ldc), mode STORE / ADD / CHAIN_POS; the split:
// GxSched.  DMA: the hand-scheduled chain (gw_chain); else register-staged operands (GxTile).
template <bool BF16, bool DMA>
__global__ __launch_bounds__(256) void gram16x_kernel(GemmDesc g, int TI, int TJ, int SJ, int Kp, long ntile, int NG,
                                                      int R, int P, int D, int* flags, int* status,
                                                      long cap) {
  static_assert(GwGeo<GX_BM>::LDS == GX_LDS, "one LDS image for both chains");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[GX_LDS];
  const uint16_t* X = (const uint16_t*)g.A;
  const GxSched S(ntile, Kp, NG, R, P, D);
  const bool vec4 = ((uintptr_t)g.C % 16 == 0) && (g.ldc % 4 == 0);
  for (int pc = -D; pc < S.npieces; ++pc) {
    int a, kb, ke;
    bool from_partial;
    S.piece(pc, a, kb, ke, from_partial);
    int ti, tj;
    gx_tile<GX_BN / GX_BM>(a, TI, TJ, SJ, ti, tj);
    const int i0 = ti * GX_BM, j0 = tj * GX_BN;
    GxTile F;
    if (from_partial && threadIdx.x == 0) {
      wait_flag_ge<2>(&flags[a], 1, cap, status, STALL_GRAM);  // gives up loudly (status word)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (from_partial) __syncthreads();
    const bool load = from_partial || g.mode == GEMM_CHAIN_POS;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int c = GxTile::col(j0, nt);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rw = GxTile::row(i0, mt, r);
          F.acc[mt][nt][r] = (load && rw < g.M && c < g.N && c >= rw) ? g.C[(long)rw * g.ldc + c] : 0.0f;
        }
      }
    if constexpr (DMA)
      gw_chain<GX_BM, BF16>(F.acc, X, g.lda, g.M, i0, j0, kb, min(ke, g.K), i0 + GX_BM <= g.M && j0 + GX_BN <= g.M,
                            smem);
    else
      F.chain<BF16, DMA>(X, g.lda, g.M, i0, j0, kb, min(ke, g.K), smem);
    const bool final = (ke >= Kp);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int c = GxTile::col(j0, nt);
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int rb = GxTile::row(i0, mt, 4 * g4);  // rows rb .. rb+3
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v[u] = F.acc[mt][nt][4 * g4 + u];
            const int rw = rb + u;
            if (rw < g.M && c < g.N && c >= rw) {
              float* dst = g.C + (long)rw * g.ldc + c;
              if (final && g.mode == GEMM_ADD) v[u] = *dst + v[u];
              *dst = v[u];
            }
          }
          if (!final || c >= g.N) continue;
          if (vec4 && c > rb + 3 && rb + 3 < g.M) {
            *(float4*)(g.C + (long)c * g.ldc + rb) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (rb + u < g.M && c > rb + u) g.C[(long)c * g.ldc + rb + u] = v[u];
          }
        }
      }
    if (!final) {  // publish the partial for workgroup w+1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&flags[a], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Same split and output contract as gram16x_kernel (STORE / CHAIN_POS, upper + mirror), on
// 256 x 256 tiles of the T x T grid.  A published partial is the whole tile, unpredicated.
template <bool BF16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gram16w_kernel(
    GemmDesc g, int T, int SJ, int Kp, long ntile, int NG, int R, int D, int* flags, int* status, long cap) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[GwGeo<GW_B>::LDS];
  const uint16_t* X = (const uint16_t*)g.A;
  const GxSched S(ntile, Kp, NG, R, 1, D);
  const int lane = threadIdx.x & 63;
  const long ldc = g.ldc;
  for (int pc = -D; pc < S.npieces; ++pc) {
    int a, kb, ke;
    bool from_partial;
    S.piece(pc, a, kb, ke, from_partial);
    int ti, tj;
    gx_tile<1>(a, T, T, SJ, ti, tj);
    const int i0 = ti * GW_B, j0 = tj * GW_B;
    if (from_partial && threadIdx.x == 0) {
      wait_flag_ge<2>(&flags[a], 1, cap, status, STALL_GRAM);  // gives up loudly (status word)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (from_partial) __syncthreads();
    // this lane's element (mt, nt, r) sits at row R(mt, r) + 4(lane>>5), column C(nt) + (lane&31)
    // with R, C wave-uniform: addresses are a uniform row pointer plus a 32-bit lane offset
    const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wu >> 1, wc = wu & 1;
    const int iw = i0 + wr * 128, jw = j0 + wc * 128;  // the wave's 128 x 128 block
    const uint32_t lo = (uint32_t)(4 * (lane >> 5)) * (uint32_t)ldc + (lane & 31);
    f32x16 acc[4][4];
    if (from_partial || g.mode == GEMM_CHAIN_POS) {
      // (a diagonal tile's lower half continues whatever is there; it is never stored as final)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float* rp = g.C + (long)(iw + mt * 32 + (r & 3) + 8 * (r >> 2)) * ldc + jw;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[mt][nt][r] = rp[lo + nt * 32];
        }
        // into the accumulator registers per row group, so the loads do not all stay live
        asm volatile("" : "+a"(acc[mt][0]), "+a"(acc[mt][1]), "+a"(acc[mt][2]), "+a"(acc[mt][3]));
      }
    } else {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the chain counts its own DMAs
    gw_chain<GW_B, BF16>(acc, X, g.lda, g.M, i0, j0, kb, min(ke, g.K), true, smem);
    if (ke < Kp) {  // publish the partial (whole tile) for the workgroup that continues it
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* rp = g.C + (long)(iw + mt * 32 + (r & 3) + 8 * (r >> 2)) * ldc + jw;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) rp[lo + nt * 32] = acc[mt][nt][r];
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&flags[a], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
    const bool diag = ti == tj;
    // column minus row of this lane's element (mt, nt, 4 g4 + u), minus (tile-local) u
    const int dl = (wc * 128 + (lane & 31)) - (wr * 128 + 4 * (lane >> 5));
    // mirror: column c of the tile is row c of G; the 4 rows (r&3) of a register group are 4
    // consecutive elements of it
    const uint32_t lm = (uint32_t)(lane & 31) * (uint32_t)ldc + 4 * (lane >> 5);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int rl = mt * 32 + 8 * g4;
          const f32x16& A = acc[mt][nt];
          const int dc = dl + nt * 32 - rl;  // element (u) exists iff dc >= u (diagonal tiles)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float* rp = g.C + (long)(iw + rl + u) * ldc + jw;
            if (!diag || dc >= u) rp[lo + nt * 32] = A[4 * g4 + u];
          }
          float* mp = g.C + (long)(jw + nt * 32) * ldc + iw + rl;
          if (!diag || dc > 3) {
            *(float4*)(mp + lm) = make_float4(A[4 * g4], A[4 * g4 + 1], A[4 * g4 + 2], A[4 * g4 + 3]);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (dc > u) mp[lm + u] = A[4 * g4 + u];
          }
        }
  }
}

// ---- a batch of Grams in one data-parallel launch (pt2q_gram_batched) ------------------------
// `batch` Grams of the same shape (N x m, m % 256 == 0), item z from X[z] into G + z*gstride.
// The work line is every item's 256 x 256 upper tiles, item-major, in the super-block order of
// gram16w_kernel; one workgroup per CU walks it in waves, workgroup w = x + NG r taking tile
// v*grid + x*R + r (the R workgroups of an XCD run R neighbouring tiles of one item at the same
// k, as the data-parallel waves of gram16w_kernel).  Every tile is ONE chain over all rows: no
// stream-K pieces, no hand-offs, and the bits of pt2q_gram on each item alone.
constexpr int GB_MAX = 128;
struct GbArgs {
  const uint16_t* X[GB_MAX];
  float* G;
  long gstride, ldx, ldc;
  int T, SJ, K, M, batch, NG, R;
  long ntile, total;
  // searched tile order (gram_order.inc; ord < 0: the super-block order): go_tab[ord + a] is tile a
  // of an item's order, whose first fr tiles are whole runs of R = 32 and the last lo a partial
  // one.  The line holds every item's fr run tiles first, then every item's lo tiles.
  int ord, fr, lo;
  int upper;     // 1: only the upper triangle (c >= r) of each G is written (no mirror stores)
};

// Batched-Gram tile orders searched offline (tools/gram_order_search.c): an XCD's 32 concurrent
// tiles (a run) read 10.3 distinct X panels per k-row at m = 11008 instead of 15.2 (super-block
// order); tables for m = 8192 / 11008 / 13824 (at m = 4096 a searched order measured no faster).
#include "gram_order.inc"

template <bool BF16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gram16b_kernel(GbArgs b) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[GwGeo<GW_B>::LDS];
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x, x = w % b.NG, r = w / b.NG;
  const long ldc = b.ldc;
  for (long L = (long)x * b.R + r; L < b.total; L += gridDim.x) {
    int z, ti, tj;
    if (b.ord >= 0) {
      const long full = (long)b.batch * b.fr;
      int a;
      if (L < full) {
        z = (int)(L / b.fr);
        a = (int)(L - (long)z * b.fr);
      } else {
        const long L2 = L - full;
        z = (int)(L2 / b.lo);
        a = b.fr + (int)(L2 - (long)z * b.lo);
      }
      const uint32_t e = go_tab[b.ord + a];
      ti = (int)(e & 0xffu);
      tj = (int)(e >> 8);
    } else {
      z = (int)(L / b.ntile);
      const int a = (int)(L - (long)z * b.ntile);
      gx_tile<1>(a, b.T, b.T, b.SJ, ti, tj);
    }
    // upper-only, off the diagonal: the TRANSPOSED tile (rows tj, columns ti), whose mirror
    // stores -- 16 bytes per lane instead of 4 -- land in the upper triangle.  Its elements have
    // the bits of the direct tile's: every MFMA group sums exact 16-bit products of the same k
    // before one rounding, so G[j][i] == G[i][j] bit for bit (test_gram_batched_upper).  C5's
    // per-channel Grams: 23.7 -> 21.7 ms per width launch (the dword stores' 256 instructions
    // per wave, against a 63-deep vmcnt, held the next tile's first stage).
    const bool diag = ti == tj, swap = b.upper && !diag;
    const int i0 = (swap ? tj : ti) * GW_B, j0 = (swap ? ti : tj) * GW_B;
    float* const C = b.G + (long)z * b.gstride;
    const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wu >> 1, wc = wu & 1;
    const int iw = i0 + wr * 128, jw = j0 + wc * 128;
    const uint32_t lo = (uint32_t)(4 * (lane >> 5)) * (uint32_t)ldc + (lane & 31);
    f32x16 acc[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[mt][nt][q] = 0.0f;
    // No wait for the previous tile's stores: they overlap this tile's first DMAs.  The chain's
    // hand-counted waits stay exact bounds -- a wait for at most K outstanding operations with the
    // stores older than every DMA still means the oldest DMAs (loads complete in order) landed; it
    // may only wait longer.  (A vmcnt(0) here held every tile's ramp behind its predecessor's 256-512
    // KiB of stores: most of the ~40-54 us fixed cost per tile that dominates at N = 4096.)
    gw_chain<GW_B, BF16>(acc, b.X[z], b.ldx, b.M, i0, j0, 0, b.K, true, smem);
    // upper tile and its mirror, as gram16w_kernel's final store (swap: the mirror only)
    const int dl = (wc * 128 + (lane & 31)) - (wr * 128 + 4 * (lane >> 5));
    const uint32_t lm = (uint32_t)(lane & 31) * (uint32_t)ldc + 4 * (lane >> 5);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int rl = mt * 32 + 8 * g4;
          const f32x16& A = acc[mt][nt];
          const int dc = dl + nt * 32 - rl;
          float* mp = C + (long)(jw + nt * 32) * ldc + iw + rl;
          if (swap) {
            *(float4*)(mp + lm) = make_float4(A[4 * g4], A[4 * g4 + 1], A[4 * g4 + 2], A[4 * g4 + 3]);
            continue;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float* rp = C + (long)(iw + rl + u) * ldc + jw;
            if (!diag || dc >= u) rp[lo + nt * 32] = A[4 * g4 + u];
          }
          if (b.upper) continue;
          if (!diag || dc > 3) {
            *(float4*)(mp + lm) = make_float4(A[4 * g4], A[4 * g4 + 1], A[4 * g4 + 2], A[4 * g4 + 3]);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (dc > u) mp[lm + u] = A[4 * g4 + u];
          }
        }
  }
}

}  // namespace

// batch Grams G[z] = X[z]ᵀX[z] (STORE), X[z] N x m 16-bit (ld ldx), G packed (gstride floats apart,
// ld m).  E_UNSUPPORTED unless m % 256 == 0 and the LDS-DMA staging conditions hold.  upper: only
// the upper triangle is stored (a per-channel unit's Gram feeds nothing but S1 / d, which
// s1_upper_ring_kernel forms from it): half the epilogue's stores, C5's Grams 55.4 -> 46.6 ms;
// off-diagonal tiles then computed transposed and stored by 16-byte mirror stores, -> ~43 ms.
int pt2q_launch_gram16_batched(const void* const* X, int dtype, long N, int m, long ldx, float* G, long gstride,
                               int batch, hipStream_t st, bool upper) {
  if ((dtype != PT2Q_F16 && dtype != PT2Q_BF16) || batch <= 0 || m <= 0 || N < 0 || !G) return PT2Q_E_ARG;
  if (batch > GB_MAX || m % GW_B || ldx % 8 || ldx >= (1l << 25) || (uintptr_t)G % 16 || gstride % 4)
    return PT2Q_E_UNSUPPORTED;
  GbArgs b{};
  for (int z = 0; z < batch; ++z) {
    if (!X[z] && N > 0) return PT2Q_E_ARG;
    if ((uintptr_t)X[z] % 16) return PT2Q_E_UNSUPPORTED;
    b.X[z] = (const uint16_t*)X[z];
  }
  const Pt2qTuning& tu = pt2q_tuning();
  b.G = G; b.gstride = gstride; b.ldx = ldx; b.ldc = m;
  b.T = m / GW_B;
  b.SJ = tu.gram_super > 0 ? tu.gram_super : 8;
  b.K = (int)N;
  b.M = m;
  b.batch = batch;
  b.ntile = (long)b.T * (b.T + 1) / 2;
  b.total = b.ntile * batch;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  b.NG = std::max(1, tu.gram_groups);
  // PT2Q_GRAM_CUS (development knob): CUs the batched Gram may hold (one workgroup each)
  const int use = tu.gram_cus > 0 ? std::min(tu.gram_cus, cus) : cus;
  b.R = std::max(1, use / b.NG);
  const long grid = std::min<long>(b.total, (long)b.NG * b.R);
  if (grid < (long)b.NG * b.R) {  // fewer tiles than workgroups: one tile each, no team order
    b.NG = 1;
    b.R = (int)grid;
  }
  b.ord = -1;
  b.upper = upper ? 1 : 0;
  if (tu.gram_order && b.R == 32 && b.NG * b.R == cus && b.ntile >= 32)
    for (int q = 0; q < GO_COUNT; ++q)
      if (go_T[q] == b.T) {
        b.ord = go_off[q];
        b.fr = (int)(b.ntile / 32) * 32;
        b.lo = (int)(b.ntile - b.fr);
      }
  hipLaunchKernelGGL(dtype == PT2Q_BF16 ? gram16b_kernel<true> : gram16b_kernel<false>, dim3((unsigned)grid),
                     dim3(256), 0, st, b);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

size_t pt2q_gram16_flags_ints(int m) { return (size_t)gx_ntile(m) + 2; }

// 16-bit Gram, every shape and mode.  flags (nullable, >= pt2q_gram16_flags_ints(m) ints):
// scratch for the split; without it (or in ADD mode, whose C holds the old values) every tile
// is one chain on one workgroup.
int pt2q_launch_gram16(const GemmDesc& g, int* flags, hipStream_t st, int* status) {
  if (g.in_dtype != PT2Q_F16 && g.in_dtype != PT2Q_BF16) return PT2Q_E_ARG;
  if (g.M != g.N || g.A != g.B || g.lda != g.ldb) return PT2Q_E_ARG;
  const Pt2qTuning& tu = pt2q_tuning();
  const int m = g.M;
  const int TI = ceil_div(m, GX_BM), TJ = ceil_div(m, GX_BN);
  // super-block side ~ the square one XCD's share of the triangle covers
  const int SJ = tu.gram_super > 0 ? tu.gram_super : (m <= 6144 ? 4 : 8);
  const long ntile = gx_ntile(m);
  const int Kp = std::max(1, ceil_div(g.K, GX_BK)) * GX_BK;  // K = 0: one all-zero stage
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // split when there are more tiles than CUs: NG XCD groups of R workgroups (one per CU)
  int NG = std::max(1, tu.gram_groups);
  int R = cus / NG;
  const bool split = flags && g.mode != GEMM_ADD && tu.gram_split && R > 0 && ntile >= (long)NG * R;
  // tile pairs need every column run of the tile order to be even (TI even) and teams of two
  int P = (split && TI % 2 == 0 && R % 2 == 0 && tu.gram_pair) ? 2 : 1;
  // whole data-parallel waves while at least one tile per workgroup is left for stream-K
  const int D = (split && tu.gram_dp) ? (int)std::max(0l, ntile / (NG * R) - 1) : 0;
  unsigned grid;
  if (split) {
    grid = (unsigned)(NG * R);
    if (hipMemsetAsync(flags, 0, sizeof(int) * pt2q_gram16_flags_ints(m), st) != hipSuccess) return PT2Q_E_HIP;
  } else {
    NG = 1;
    R = 0;
    P = 1;
    grid = (unsigned)ntile;
  }
  // the status word: the caller's, else a word of the flag area (zeroed above)
  if (!status && split) status = flags + ntile;
  // (fast staging keeps a stage's byte offsets in 32 bits: 64 rows * lda * 2 < 2^32)
  const bool dma = ((uintptr_t)g.A % 16 == 0) && (g.lda % 8 == 0) && (m % 8 == 0) && g.lda < (1l << 25);
  const bool bf = g.in_dtype == PT2Q_BF16;
  // 256 x 256 tiles when m is a multiple of 256 and they make at least two waves (so the
  // data-parallel part keeps every CU busy); mirror stores are float4
  const int TW = m / GW_B;
  const long ntw = (long)TW * (TW + 1) / 2;
  if (split && dma && tu.gram_wide && m % GW_B == 0 && ntw >= 2l * NG * R && (uintptr_t)g.C % 16 == 0 &&
      g.ldc % 4 == 0) {
    const int SW = tu.gram_super > 0 ? tu.gram_super : 8;
    const int Dw = tu.gram_dp ? (int)std::max(0l, ntw / (NG * R) - 1) : 0;
    hipLaunchKernelGGL(bf ? gram16w_kernel<true> : gram16w_kernel<false>, dim3(grid), dim3(256), 0, st, g, TW, SW,
                       Kp, ntw, NG, R, Dw, flags, status, tu.spin_cap_long);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  void (*k)(GemmDesc, int, int, int, int, long, int, int, int, int, int*, int*, long) =
      bf ? (dma ? gram16x_kernel<true, true> : gram16x_kernel<true, false>)
         : (dma ? gram16x_kernel<false, true> : gram16x_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, g, TI, TJ, SJ, Kp, ntile, NG, R, P, D, flags, status,
                     tu.spin_cap_long);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}
