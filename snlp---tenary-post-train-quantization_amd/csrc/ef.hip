// GPTQ error feedback of one block (main.py:214, gptq.py:181-186):
//   W[:, rem] -= E · C,   E = W_b − (α T + μ) (n × bs),  C = Hinv[blk][:, rem] / diag (bs × nr)
// in the feature-major layout: Wt[rem_e][i] -= Σ_k C[k][e] · E[k][i], the product a k-ascending
// f32 chain (v_mfma_f32_32x32x2_f32 issues k in ascending pairs: D = fma(a1,b1, fma(a0,b0, C)),
// the oracle's order), rounded once, then one subtraction -- the contract of DESIGN.md §3.
//
// A K <= 128 GEMM is too short for the generic tile loop (load, sync, compute, reload C): here a
// persistent workgroup walks 128 × 128 output tiles and keeps the operand stream running across
// them.  The two 64-deep K halves of a tile live in two LDS stages (A: C[k][e0..], B: E[k][i0..],
// 64 KiB per stage) filled by LDS-DMA; while one half is multiplied the other half of the next
// tile is fetched, and the old Wt rows of a tile are loaded into registers while its MFMAs run.
// Every wave issues the same number of memory instructions per tile (out-of-range rows and
// columns go through buffer ops with offsets past the end, which the hardware drops), so the
// hand-counted s_waitcnt vmcnt values below are exact.
//
// With a partial buffer the epilogue also forms the NEXT block's SSR mean partials (the w-bar of
// ssr.hip over the rows just written, crow = the next block's rem): a tile's 128 rows e are
// exactly one w-bar chunk, so per column i its new values are folded in registers -- rows e and
// e + 32 of a lane added, a butterfly over the 32 lanes (xor 16 by ds_swizzle, then bfly16), the
// two waves of a column half combined through LDS -- the CHUNK128 order of DESIGN.md §3.  That
// removes the separate w-bar pass over W[:, rem] (one full read per block).
#include "common.hpp"
#include "internal.hpp"
#include "probe.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int EF_T = 128;                    // output tile (e and i)
constexpr int EF_KH = 64;                    // k rows per LDS stage
constexpr int EF_ROWB = EF_T * 4;            // 512 B per k row of a panel
constexpr int EF_PANEL = EF_KH * EF_ROWB;    // 32 KiB
[[maybe_unused]] constexpr int EF_STAGE = 2 * EF_PANEL;  // A + B (ef_gemm_kernel: development builds)
constexpr int EF_DMA = 16;                   // DMA instructions per wave per stage
constexpr int EF_CV = 16;                    // C float4 loads (= stores) per lane per tile
constexpr unsigned EF_DROP = 0x80000000u;    // buffer offset past any Wt (dropped access)

__device__ uint4 ef_zero16;  // DMA source of the k rows past bs (zero-initialised)

// wave index inside a team of 4 waves (a workgroup is one team, or two: ef2_gemm_kernel TEAMS)
PT2Q_DEV int ef_wave() { return (int)(threadIdx.x >> 6) & 3; }

struct EfArgs {
  const float* Ck;  // C[k][e], ld m
  long ldk;
  const float* Et;  // E[k][i], ld ldw
  float* Wt;        // Wt[j][i], ld ldw
  long ldw;
  const int* crow;  // rem (nr entries)
  int nr, bs, te, ti, ntile, nh;
  long zs;          // grouped: bytes between the linears' workspace slices (Ck, Et, Wt, crow, part)
  int nz;           // linears; the work line is nz * ntile tiles, linear-major
  float* part;      // nullable: w-bar chunk partials part[c][i] of the updated rows, i < n
  int n;
  int stagger;      // ef2: the grid's second half first sleeps stagger x 4K cycles (PT2Q_EF2_STAGGER)
  int probe;        // ef2 development knock-outs (PT2Q_EF2_PROBE, tools only; results garbage):
                    // 1 = Wt traffic dropped, 2 = operand DMAs from one hot chunk, 4 = no MFMAs
  int toff;         // ef2 TEAMS = 2: barriers team 1 starts behind team 0
};

// The arguments of linear z (its workspace slice).
PT2Q_DEV EfArgs ef_linear(const EfArgs& a0, int z) {
  EfArgs a = a0;
  const long o = (long)z * a0.zs;
  a.Ck = (const float*)((const char*)a0.Ck + o);
  a.Et = (const float*)((const char*)a0.Et + o);
  a.Wt = (float*)((char*)a0.Wt + o);
  a.crow = (const int*)((const char*)a0.crow + o);
  if (a0.part) a.part = (float*)((char*)a0.part + o);
  return a;
}

// One stage (K half h) of tile (e0, i0) into LDS: 8 DMA of A (2 k-rows of 512 B each), 8 of B.
// k rows past bs come from a zero chunk (their MFMA steps are then exact no-ops); columns past
// the data come from row 0 (garbage in rows / columns whose results are dropped), so every wave
// issues exactly EF_DMA instructions.
PT2Q_DEV void ef_stage_q(const EfArgs& a, int e0, int i0, int h, uint8_t* stg, int q, bool withB) {
  const int lane = threadIdx.x & 63, wave = ef_wave();
  typedef __attribute__((address_space(3))) void* lptr;
  const int kr = (wave * 8 + q) * 2 + (lane >> 5);  // k row inside the stage
  const int k = h * EF_KH + kr;
  const int d = 4 * (lane & 31);
  const bool kin = k < a.bs;
  const int e = e0 + d, i = i0 + d;
  const void* sa = kin && !probe::ef_zero_dma ? (const void*)(a.Ck + (e < a.nr ? (long)k * a.ldk + e : 0)) : (const void*)&ef_zero16;
  const void* sb = kin && !probe::ef_zero_dma ? (const void*)(a.Et + (i < a.ldw ? (long)k * a.ldw + i : 0)) : (const void*)&ef_zero16;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  if constexpr (probe::ef_no_dma) return;
  __builtin_amdgcn_global_load_lds(sa, (lptr)(stg + (wv * 8 + q) * 1024), 16, 0, 0);
  if (withB) __builtin_amdgcn_global_load_lds(sb, (lptr)(stg + EF_PANEL + (wv * 8 + q) * 1024), 16, 0, 0);
}

// withB = false: the B panel (E columns i0) already holds this K half -- the previous tile of the
// workgroup had the same linear and i0 -- so only the A panel is fetched (8 DMAs instead of 16)
PT2Q_DEV int ef_stage(const EfArgs& a, int e0, int i0, int h, uint8_t* stg, bool withB = true) {
#pragma unroll
  for (int q = 0; q < 8; ++q) ef_stage_q(a, e0, i0, h, stg, q, withB);
  return withB ? EF_DMA : EF_DMA / 2;
}

// Fast staging (every k row and column of the stage in range: all tiles but ragged edges): this
// lane's byte offsets of its 8 A and 8 B chunks from the stage's panel bases, fixed for the launch
// (ldk and ldw are common to a group's linears), so a DMA is s_mov m0 + one global_load_lds with a
// scalar base -- three instructions instead of the ~35 of ef_stage_q's per-lane address math,
// which held every stage issue to ~1 us (tools/ef_probe.hip stamps).
struct EfVo {
  uint32_t a[8], b[8];
};

PT2Q_DEV void ef_voff(const EfArgs& a, EfVo& v) {
  const int lane = threadIdx.x & 63, wave = ef_wave();
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int kr = (wave * 8 + q) * 2 + (lane >> 5), d = 4 * (lane & 31);
    v.a[q] = (uint32_t)(((long)kr * a.ldk + d) * 4);
    v.b[q] = (uint32_t)(((long)kr * a.ldw + d) * 4);
  }
}

// one 16-B LDS-DMA: global (sbase + voff) -> LDS m0 + 16 lane (m0 is set afresh by every DMA)
PT2Q_DEV void ef_dma_asm(const char* sbase, uint32_t voff, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(m0)
               : "memory");
}

// a stage by the fast path when it is whole, else by ef_stage; returns the DMAs issued per wave
PT2Q_DEV int ef_stage_any(const EfArgs& a, int e0, int i0, int h, uint8_t* stg, uint32_t stg_lds, const EfVo& v,
                          bool withB) {
  const bool fast = (h + 1) * EF_KH <= a.bs && e0 + EF_T <= a.nr && i0 + EF_T <= a.ldw &&
                    !probe::ef_zero_dma && !probe::ef_no_dma;
  if (!fast) return ef_stage(a, e0, i0, h, stg, withB);
  const int wv = __builtin_amdgcn_readfirstlane(ef_wave());
  const char* ba = (const char*)(a.Ck + (long)h * EF_KH * a.ldk + e0);
  const char* bb = (const char*)(a.Et + (long)h * EF_KH * a.ldw + i0);
  const uint32_t mA = stg_lds + (uint32_t)(wv * 8 * 1024), mB = mA + EF_PANEL;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ef_dma_asm(ba, v.a[q], mA + q * 1024);
    if (withB) ef_dma_asm(bb, v.b[q], mB + q * 1024);
  }
  return withB ? EF_DMA : EF_DMA / 2;
}

template <int OFF>
PT2Q_DEV float ef_ld(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// wait until at most N LDS operations are outstanding, tying the operand registers a, b
template <int N>
PT2Q_DEV void ef_wait(float (&a)[2], float (&b)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]) : "n"(N));
}

// k-pair S of a stage: lane reads A rows e (2 MFMA row blocks) and B columns i (2 blocks).
template <int S>
PT2Q_DEV void ef_read(uint32_t baseA, uint32_t baseB, float (&a)[2], float (&b)[2]) {
  a[0] = ef_ld<S * 2 * EF_ROWB>(baseA);
  a[1] = ef_ld<S * 2 * EF_ROWB + 128>(baseA);
  b[0] = ef_ld<S * 2 * EF_ROWB>(baseB);
  b[1] = ef_ld<S * 2 * EF_ROWB + 128>(baseB);
}

// KS k rows per LDS stage (EF_KH for ef_gemm_kernel's two K halves, E2_KS for ef2_gemm_kernel)
template <int KS>
struct EfAccT {
  f32x16 acc[2][2];  // [rm][rn], transposed MFMA: lane <-> e row, registers <-> i columns

  // k-pair S: its operands are in set S % 4; the reads of pair S+2 go to set (S+2) % 4, whose
  // registers the MFMAs of pair S-2 read long ago (no overwrite of an operand in flight), so an
  // LDS read has two pairs (~500 cycles) to land instead of one.  The IO work of the pair sits in
  // the shadows of its four MFMAs (io.g0 .. g3, one piece after each): a VMEM issue or a dependent
  // VALU chain longer than the 64-cycle shadow would leave the MFMA pipe idle.  The LDS writes
  // of the IO (IO::lds_writes) are counted in the lgkmcnt waits.  The order reads -> MFMAs ->
  // wait is pinned.
  template <int S, class IO>
  PT2Q_DEV void run(uint32_t bA, uint32_t bB, float (&a)[4][2], float (&b)[4][2], IO& io) {
    constexpr int NP = KS / 2;
    if constexpr (S < NP) {
      constexpr int c = S % 4;
      if constexpr (S + 2 < NP) ef_read<S + 2>(bA, bB, a[(S + 2) % 4], b[(S + 2) % 4]);
      if constexpr (S > 0) {  // pair S-1's operands stay allocated until these reads are out
        constexpr int p = (S + 3) % 4;
        asm volatile("" ::"v"(a[p][0]), "v"(a[p][1]), "v"(b[p][0]), "v"(b[p][1]));
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[c][0], a[c][0], acc[0][0], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      io.template g0<S>();
      __builtin_amdgcn_sched_barrier(0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[c][1], a[c][0], acc[0][1], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      io.template g1<S>();
      __builtin_amdgcn_sched_barrier(0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[c][0], a[c][1], acc[1][0], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      io.template g2<S>();
      __builtin_amdgcn_sched_barrier(0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[c][1], a[c][1], acc[1][1], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      io.template g3<S>();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (S + 1 < NP) {  // pair S+1's reads (issued at pair S-1) landed; younger LDS
        // operations: pair S-1's IO writes, pair S+2's reads, pair S's IO writes
        constexpr int n = (S >= 1 ? IO::template lds_writes<S - 1>() : 0) + (S + 2 < NP ? 4 : 0) +
                          IO::template lds_writes<S>();
        ef_wait<n>(a[(S + 1) % 4], b[(S + 1) % 4]);
      }
      run<S + 1>(bA, bB, a, b, io);
    }
  }

  // the KS / 2 k-pairs of one stage (k rows past bs are zero in LDS: exact no-op steps)
  template <class IO>
  PT2Q_DEV void half(uint32_t stg, IO& io) {
    const int lane = threadIdx.x & 63, wave = ef_wave();
    const int wr = wave >> 1, wc = wave & 1, li = lane & 31, lk = lane >> 5;
    const uint32_t bA = stg + lk * EF_ROWB + (wr * 64 + li) * 4;
    const uint32_t bB = stg + KS * EF_ROWB + lk * EF_ROWB + (wc * 64 + li) * 4;
    float a[4][2], b[4][2];
    ef_read<0>(bA, bB, a[0], b[0]);
    ef_read<1>(bA, bB, a[1], b[1]);
    ef_wait<4>(a[0], b[0]);
    run<0>(bA, bB, a, b, io);
  }
};
using EfAcc = EfAccT<EF_KH>;

PT2Q_DEV int ef_row(int e0, int rm) {
  const int lane = threadIdx.x & 63, wr = ef_wave() >> 1;
  return e0 + wr * 64 + rm * 32 + (lane & 31);
}
PT2Q_DEV int ef_col(int i0, int rn, int q) {
  const int lane = threadIdx.x & 63, wc = ef_wave() & 1;
  return i0 + wc * 64 + rn * 32 + 8 * q + 4 * (lane >> 5);
}

// byte offset of the old/new Wt values of group (rm, rn, q), or EF_DROP; wrow[rm] = the Wt row
// of this lane's output row in row block rm (-1 past nr)
PT2Q_DEV unsigned ef_coff(const EfArgs& a, const int (&wrow)[2], int i0, int rm, int rn, int q) {
  const int i = ef_col(i0, rn, q);
  if (wrow[rm] < 0 || i >= a.ldw || probe::ef_drop_wt) return EF_DROP;
  return (unsigned)(((long)wrow[rm] * a.ldw + i) * 4);
}

// ef_coff as a per-tile row base: group (rm, rn, q) of this lane sits at rb[rm] + 4 (32 rn + 8 q)
// bytes (the constant folds into the buffer instruction's offset field), rb[rm] = EF_DROP for a row
// past nr or a column half past ldw (ldw % 64 == 0, so a wave's 64 columns are in or out together)
PT2Q_DEV void ef_rowbase(const EfArgs& a, const int (&wrow)[2], int i0, uint32_t (&rb)[2]) {
  const int lane = threadIdx.x & 63, wc = ef_wave() & 1;
  const int i = i0 + wc * 64 + 4 * (lane >> 5);
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
    rb[rm] = (wrow[rm] < 0 || i0 + wc * 64 >= a.ldw || probe::ef_drop_wt)
                 ? EF_DROP
                 : (uint32_t)(((long)wrow[rm] * a.ldw + i) * 4);
}

// the Wt rows of this lane's two output rows (crow from L2: two loads per lane, issued uniformly
// by every wave and older than every operation a later hand-counted vmcnt wait covers)
PT2Q_DEV void ef_rows(const EfArgs& a, int e0, int (&wrow)[2]) {
  int v[2];
#pragma unroll
  for (int rm = 0; rm < 2; ++rm) {
    const int e = ef_row(e0, rm);
    v[rm] = a.crow[e < a.nr ? e : 0];
  }
#pragma unroll
  for (int rm = 0; rm < 2; ++rm) wrow[rm] = ef_row(e0, rm) < a.nr ? v[rm] : -1;
}

struct EfNoIO {
  template <int S>
  PT2Q_DEV void g0() {}
  template <int S>
  PT2Q_DEV void g1() {}
  template <int S>
  PT2Q_DEV void g2() {}
  template <int S>
  PT2Q_DEV void g3() {}
  template <int S>
  static constexpr int lds_writes() { return 0; }
};

// ---- the next block's w-bar partials (see the file header), one column j per k-pair of the
// next tile's first K half.  Column j = (rn, q, u) of the tile's results pend; the lane sum over
// rows e and e + 32 (its two row blocks rm), bfly16 inside each 16-lane row, then row_bcast:15
// adds row 0's sum into row 1 (row 2's into row 3): lanes 16 and 48 hold the wave's 64-row sum
// for column halves h = 0, 1 and store it to LDS (the other lanes to a per-lane spare slot).
constexpr int EF_PS = 8;    // w-bar partial stores per wave per tile (float4; dropped where unused)
constexpr int EF_RED = 512; // LDS floats: [wave][64] sums + [wave][64] spare slots

template <int J>
PT2Q_DEV void ef_wbar_step(const int (&prow)[2], const u32x4 (&pend)[EF_CV], float* red) {
  constexpr int rn = J >> 4, q = (J >> 2) & 3, u = J & 3;
  const int lane = threadIdx.x & 63, wave = ef_wave();
  const float v0 = prow[0] >= 0 ? __uint_as_float(pend[rn * 4 + q][u]) : 0.0f;
  const float v1 = prow[1] >= 0 ? __uint_as_float(pend[(2 + rn) * 4 + q][u]) : 0.0f;
  float x = bfly16(v0 + v1);
  x = x + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xA, 0xF, false));  // row_bcast:15
  const bool sel = (lane & 31) == 16;
  red[sel ? wave * 64 + (lane >> 5) * 32 + J : 256 + wave * 64 + lane] = x;
}

// ef_wbar_step for columns J and J+1 in four pieces, one per MFMA shadow of a k-pair: the two
// columns' dependent DPP chains interleaved (each column's operations and order are
// ef_wbar_step's, so the sums are the same bits).
struct EfWb2 {
  float x0, x1;
};

template <int J>
PT2Q_DEV void ef_wb_a(EfWb2& w, const int (&prow)[2], const u32x4 (&pend)[EF_CV]) {
  constexpr int rn = J >> 4, q = (J >> 2) & 3, u = J & 3;
  constexpr int rn1 = (J + 1) >> 4, q1 = ((J + 1) >> 2) & 3, u1 = (J + 1) & 3;
  const float a0 = prow[0] >= 0 ? __uint_as_float(pend[rn * 4 + q][u]) : 0.0f;
  const float a1 = prow[0] >= 0 ? __uint_as_float(pend[rn1 * 4 + q1][u1]) : 0.0f;
  const float b0 = prow[1] >= 0 ? __uint_as_float(pend[(2 + rn) * 4 + q][u]) : 0.0f;
  const float b1 = prow[1] >= 0 ? __uint_as_float(pend[(2 + rn1) * 4 + q1][u1]) : 0.0f;
  w.x0 = a0 + b0;
  w.x1 = a1 + b1;
}

PT2Q_DEV void ef_wb_b(EfWb2& w) {
  const float s0 = xor_lane<8>(w.x0), s1 = xor_lane<8>(w.x1);
  w.x0 = w.x0 + s0;
  w.x1 = w.x1 + s1;
  const float t0 = xor4_sym8(w.x0), t1 = xor4_sym8(w.x1);  // after the xor-8 step
  w.x0 = w.x0 + t0;
  w.x1 = w.x1 + t1;
}

PT2Q_DEV void ef_wb_c(EfWb2& w) {
  const float s0 = xor_lane<2>(w.x0), s1 = xor_lane<2>(w.x1);
  w.x0 = w.x0 + s0;
  w.x1 = w.x1 + s1;
  const float t0 = xor_lane<1>(w.x0), t1 = xor_lane<1>(w.x1);
  w.x0 = w.x0 + t0;
  w.x1 = w.x1 + t1;
}

template <int J>
PT2Q_DEV void ef_wb_d(EfWb2& w, float* red) {
  const int lane = threadIdx.x & 63, wave = ef_wave();
  const float r0 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(w.x0), 0x142, 0xA, 0xF, false));
  const float r1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(w.x1), 0x142, 0xA, 0xF, false));
  const float y0 = w.x0 + r0, y1 = w.x1 + r1;  // row_bcast:15
  const bool sel = (lane & 31) == 16;
  red[sel ? wave * 64 + (lane >> 5) * 32 + J : 256 + wave * 64 + lane] = y0;
  red[sel ? wave * 64 + (lane >> 5) * 32 + J + 1 : 256 + wave * 64 + lane] = y1;
}

// The Wt traffic of a tile, spread over the first K half of the next one instead of bursting
// at tile ends (every CU would burst at once): at every even k-pair one store of the previous
// tile's results and one load of this tile's old values.  Rows of the previous tile are -1
// before the first tile (stores dropped, counts unchanged).
struct EfIO {
  const EfArgs& a;
  __amdgpu_buffer_rsrc_t rc;   // this tile's Wt (old values)
  __amdgpu_buffer_rsrc_t prc;  // the previous tile's Wt (its results), possibly another linear's
  const int (&prow)[2];          // the previous tile's Wt rows (-1 past nr): its w-bar pieces
  const uint32_t (&rb)[2];       // ef_rowbase of this tile (old values)
  const uint32_t (&prb)[2];      // ef_rowbase of the previous tile (its results)
  const u32x4 (&pend)[EF_CV];
  u32x4 (&c)[EF_CV];
  float* red;  // the previous tile's w-bar wave sums (ef_wbar_step)

  EfWb2 w;     // the w-bar pieces' state between the gaps of an odd k-pair

  // even k-pairs: one store of the previous tile's results, one load of this tile's old values;
  // odd k-pairs S: the w-bar of columns S-1 and S of the previous tile's results
  template <int S>
  PT2Q_DEV void g0() {
    if constexpr (S % 2 == 0 && S / 2 < EF_CV) {
      constexpr int j = S / 2, rm = j >> 3, rn = (j >> 2) & 1, q = j & 3;
      __builtin_amdgcn_raw_buffer_store_b128(pend[j], prc, prb[rm] + 4 * (32 * rn + 8 * q), 0, 0);
    }
    if constexpr (S % 2 == 1) ef_wb_a<S - 1>(w, prow, pend);
  }
  template <int S>
  PT2Q_DEV void g1() {
    if constexpr (S % 2 == 0 && S / 2 < EF_CV) {
      constexpr int j = S / 2, rm = j >> 3, rn = (j >> 2) & 1, q = j & 3;
      c[j] = __builtin_amdgcn_raw_buffer_load_b128(rc, rb[rm] + 4 * (32 * rn + 8 * q), 0, 0);
    }
    if constexpr (S % 2 == 1) ef_wb_b(w);
  }
  template <int S>
  PT2Q_DEV void g2() {
    if constexpr (S % 2 == 1) ef_wb_c(w);
  }
  // (always issued; without a partial buffer the sums land in `red` and nothing reads them)
  template <int S>
  PT2Q_DEV void g3() {
    if constexpr (S % 2 == 1) ef_wb_d<S - 1>(w, red);
  }
  template <int S>
  static constexpr int lds_writes() { return S % 2 == 1 ? 2 : 0; }
};

// s_waitcnt vmcnt(N) for the small set of counts the schedule needs (immediate operand)
PT2Q_DEV void ef_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
  }
}

// The w-bar partials of a finished tile (e0, i0) from the wave sums in LDS: part[c][i] = X + Y,
// X from the row-half-0 wave of the column half, Y from the row-half-1 wave.  Branch-free: every
// lane reads (b128, all in flight) and every wave issues exactly EF_PS buffer stores (real ones:
// lanes 0 and 32 of the row-half-0 waves, i < n; the rest dropped).
PT2Q_DEV void ef_wbar_store(int n, __amdgpu_buffer_rsrc_t rp, bool valid, int e0, int i0, const float* red) {
  const int lane = threadIdx.x & 63, wave = ef_wave(), wr = wave >> 1, wc = wave & 1;
  const int h = lane >> 5;
  const bool mine = valid && wr == 0 && (lane & 31) == 0;
  const long cb = (long)(e0 / EF_T) * n;
  const f32x4* X = (const f32x4*)(red + wc * 64 + h * 32);
  const f32x4* Y = (const f32x4*)(red + (wc + 2) * 64 + h * 32);
#pragma unroll
  for (int rn = 0; rn < 2; ++rn) {
    f32x4 x[4], y[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      x[q] = X[rn * 4 + q];
      y[q] = Y[rn * 4 + q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = i0 + wc * 64 + rn * 32 + 8 * q + 4 * h;
      const f32x4 o = x[q] + y[q];
      const unsigned off = (mine && i < n) ? (unsigned)((cb + i) * 4) : EF_DROP;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rp, off, 0, 0);
    }
  }
}

#ifdef PT2Q_DEV_PROBES
// ef_gemm_kernel (one workgroup per CU): superseded by ef2_gemm_kernel; kept for A/B runs in
// development builds only (PT2Q_EF_V2=0), never reachable from a release library.
template <int J>
PT2Q_DEV void ef_wbar_all(const int (&prow)[2], const u32x4 (&pend)[EF_CV], float* red) {
  if constexpr (J < 32) {
    ef_wbar_step<J>(prow, pend, red);
    ef_wbar_all<J + 1>(prow, pend, red);
  }
}

__global__ __launch_bounds__(256) void ef_gemm_kernel(EfArgs a0, long wt_bytes, long part_bytes) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * EF_STAGE];
  __shared__ __attribute__((aligned(16))) float red[EF_RED];  // w-bar wave sums (ef_wbar_step)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  const int total = a0.ntile * a0.nz;
  int t = blockIdx.x;
  if (t >= total) return;
  // tile t of the work line: linear t / ntile, corner (e0, i0) of its output
  auto corner = [&](int t, EfArgs& a, int& e0, int& i0) {
    const int z = t / a0.ntile, tl = t - z * a0.ntile;
    a = ef_linear(a0, z);
    e0 = (tl / a0.ti) * EF_T;
    i0 = (tl % a0.ti) * EF_T;
  };
  auto rsrc = [&](const EfArgs& a) { return __builtin_amdgcn_make_buffer_rsrc(a.Wt, 0, (int)wt_bytes, 0x00020000); };
  auto prsrc = [&](const EfArgs& x) { return __builtin_amdgcn_make_buffer_rsrc(x.part, 0, (int)part_bytes, 0x00020000); };
  const int P = a0.part ? EF_PS : 0;  // part stores per tile, younger than the tile's stages
  EfArgs a;
  int e0, i0, wrow[2];
  corner(t, a, e0, i0);
  __amdgpu_buffer_rsrc_t rc = rsrc(a), prc = rc;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  ef_rows(a, e0, wrow);
  EfVo vo;
  ef_voff(a0, vo);
  ef_stage_any(a, e0, i0, 0, smem, lds0, vo, true);
  if (a.nh == 2) ef_stage_any(a, e0, i0, 1, smem + EF_STAGE, lds0 + EF_STAGE, vo, true);
  // P dropped stores: every tile's first wait then sees the same count of younger operations
  for (int j = 0; j < P; ++j) __builtin_amdgcn_raw_buffer_store_b128(u32x4{}, rc, EF_DROP, 0, 0);
  int prow[2] = {-1, -1}, pi0 = 0, pe0 = -1;
  __amdgpu_buffer_rsrc_t prp = rc;  // the previous tile's part buffer (its linear's)
  u32x4 c[EF_CV], pend[EF_CV];
#pragma unroll
  for (int j = 0; j < EF_CV; ++j) pend[j] = u32x4{};
  // issue order per tile: [stores of the previous tile + this tile's old values, interleaved
  // with K half 0] [next stage 0] [K half 1] [next stage 1]
  int S1 = a.nh == 2 ? EF_DMA : 0;  // this tile's stage-1 DMAs (per wave), issued before its top
  int nt = 0;  // tiles done (probe stamps only)
  (void)nt;
  for (;;) {
    PT2Q_EF_STAMP(nt, 0);
    const int tn = t + (int)gridDim.x;
    const bool more = tn < total;
    int en = 0, in = 0, nrow[2] = {-1, -1};
    EfArgs an = a;
    if (more) corner(tn, an, en, in);
    // the next tile's E panel is this one's when it has the same linear and column block (tiles
    // gridDim.x apart on the line share i0 whenever ti divides it: n = 4096)
    const bool newB = !(more && an.Et == a.Et && in == i0);
    int D0 = 0, D1 = 0;  // the next tile's stage DMAs per wave
    EfAcc F;
#pragma unroll
    for (int rm = 0; rm < 2; ++rm)
#pragma unroll
      for (int rn = 0; rn < 2; ++rn) F.acc[rm][rn] = f32x16{};
    ef_vmcnt(S1 + P);  // stage 0 landed (younger: stage 1, the previous tile's part stores)
    PT2Q_EF_STAMP(nt, 1);
    asm volatile("s_barrier" ::: "memory");
    PT2Q_EF_STAMP(nt, 2);
    if (more) ef_rows(an, en, nrow);
    {
      uint32_t rb[2], prb[2];
      ef_rowbase(a, wrow, i0, rb);
      ef_rowbase(a, prow, pi0, prb);
      EfIO io{a, rc, prc, prow, rb, prb, pend, c, red, {}};
      F.half(lds0, io);
    }
    PT2Q_EF_STAMP(nt, 3);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave done with stage 0
    PT2Q_EF_STAMP(nt, 8);
    if (more) D0 = ef_stage_any(an, en, in, 0, smem, lds0, vo, newB);
    PT2Q_EF_STAMP(nt, 9);
    if (P) ef_wbar_store(a0.n, prp, pe0 >= 0, pe0, pi0, red);  // the previous tile's partials
    PT2Q_EF_STAMP(nt, 10);
    if (a.nh == 2) {
      ef_vmcnt(P + 2 * EF_CV + D0);  // stage 1 landed
      PT2Q_EF_STAMP(nt, 4);
      asm volatile("s_barrier" ::: "memory");
      PT2Q_EF_STAMP(nt, 5);
      EfNoIO nio;
      F.half(lds0 + EF_STAGE, nio);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (more) D1 = ef_stage_any(an, en, in, 1, smem + EF_STAGE, lds0 + EF_STAGE, vo, newB);
    }
    PT2Q_EF_STAMP(nt, 6);
    ef_vmcnt(more ? D0 + P + D1 : 0);  // the old values landed (younger: next stages, part stores)
    PT2Q_EF_STAMP(nt, 7);
    ++nt;
#pragma unroll
    for (int rm = 0; rm < 2; ++rm)
#pragma unroll
      for (int rn = 0; rn < 2; ++rn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = (rm * 2 + rn) * 4 + q;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            pend[j][u] = __float_as_uint(__uint_as_float(c[j][u]) - F.acc[rm][rn][4 * q + u]);
        }
    prow[0] = wrow[0];
    prow[1] = wrow[1];
    pi0 = i0;
    pe0 = e0;
    if (P) prp = prsrc(a);
    prc = rc;
    if (!more) break;
    S1 = D1;
    t = tn;
    a = an;
    rc = rsrc(a);
    e0 = en;
    i0 = in;
    wrow[0] = nrow[0];
    wrow[1] = nrow[1];
  }
#pragma unroll
  for (int j = 0; j < EF_CV; ++j)
    __builtin_amdgcn_raw_buffer_store_b128(pend[j], prc, ef_coff(a, prow, pi0, j >> 3, (j >> 2) & 1, j & 3), 0, 0);
  if (P) {  // the last tile's partials (the earlier ones were formed in the next tile's first half)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // red free (last readers done)
    ef_wbar_all<0>(prow, pend, red);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    ef_wbar_store(a0.n, prp, true, pe0, pi0, red);
  }
}

#endif  // PT2Q_DEV_PROBES

// ---- ef2_gemm_kernel: the same product with two workgroups per CU ----------------------------
// ef_gemm_kernel holds ONE workgroup per CU (two 64-row K stages = 128 KiB of LDS, 336 registers):
// each SIMD runs a single wave, so every stall of that wave -- an LDS-read wait, a barrier, a DMA
// still landing -- idles the MFMA pipe (MFMA busy 0.48 in the 7B step).  Here a workgroup keeps
// a ring of two 32-row K stages (32 KiB each; 66 KiB with the w-bar scratch) and at most 256
// registers per lane, so two workgroups share every CU and each SIMD interleaves two waves: one
// issues MFMAs while the other waits.  Per tile: the old Wt values are loaded at the top (their
// latency hides under the tile's MFMAs), the K stages stream through the ring (the stage after
// next is fetched into the slot just consumed, running on into the next tile's first two stages),
// and the epilogue subtracts, stores, and forms the tile's own w-bar partials.  The k-pairs are
// issued in ascending order into the same accumulators, the product is subtracted once, and the
// w-bar is the same CHUNK128 tree: bit-identical to ef_gemm_kernel.
constexpr int E2_KS = 32;                  // k rows per stage (16 k-pairs)
constexpr int E2_PANEL = E2_KS * EF_ROWB;  // 16 KiB
constexpr int E2_STAGE = 2 * E2_PANEL;     // A + B: 32 KiB

// One 16-B chunk q (< 4) of stage s of tile (e0, i0) by per-lane addresses (ragged stages); the
// conventions of ef_stage_q (zero chunk past bs, in-range garbage in dropped rows / columns).
PT2Q_DEV void e2_stage_q(const EfArgs& a, int e0, int i0, int s, uint8_t* stg, int q, bool withB) {
  const int lane = threadIdx.x & 63, wave = ef_wave();
  typedef __attribute__((address_space(3))) void* lptr;
  const int kr = (wave * 4 + q) * 2 + (lane >> 5);
  const int k = s * E2_KS + kr;
  const int d = 4 * (lane & 31);
  const bool kin = k < a.bs;
  const int e = e0 + d, i = i0 + d;
  const void* sa = kin ? (const void*)(a.Ck + (e < a.nr ? (long)k * a.ldk + e : 0)) : (const void*)&ef_zero16;
  const void* sb = kin ? (const void*)(a.Et + (i < a.ldw ? (long)k * a.ldw + i : 0)) : (const void*)&ef_zero16;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  __builtin_amdgcn_global_load_lds(sa, (lptr)(stg + (wv * 4 + q) * 1024), 16, 0, 0);
  if (withB) __builtin_amdgcn_global_load_lds(sb, (lptr)(stg + E2_PANEL + (wv * 4 + q) * 1024), 16, 0, 0);
}

struct E2Vo {
  uint32_t a[4], b[4];
};

PT2Q_DEV void e2_voff(const EfArgs& a, E2Vo& v) {
  const int lane = threadIdx.x & 63, wave = ef_wave();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int kr = (wave * 4 + q) * 2 + (lane >> 5), d = 4 * (lane & 31);
    v.a[q] = (uint32_t)(((long)kr * a.ldk + d) * 4);
    v.b[q] = (uint32_t)(((long)kr * a.ldw + d) * 4);
  }
}

// stage s of tile (e0, i0) into slot `stg`: scalar-base DMAs when whole (ef_stage_any), else per
// lane; returns the DMA instructions issued per wave (8, or 4 without the B panel)
PT2Q_DEV int e2_stage(const EfArgs& a, int e0, int i0, int s, uint8_t* stg, uint32_t stg_lds, const E2Vo& v,
                      bool withB) {
  if (a.probe & 2) {  // knock-out: every DMA from the one zero chunk (L2-hot)
    typedef __attribute__((address_space(3))) void* lptr;
    const int wv = __builtin_amdgcn_readfirstlane(ef_wave());
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_global_load_lds(&ef_zero16, (lptr)(stg + (wv * 4 + q) * 1024), 16, 0, 0);
      if (withB) __builtin_amdgcn_global_load_lds(&ef_zero16, (lptr)(stg + E2_PANEL + (wv * 4 + q) * 1024), 16, 0, 0);
    }
    return withB ? 8 : 4;
  }
  const bool fast = (s + 1) * E2_KS <= a.bs && e0 + EF_T <= a.nr && i0 + EF_T <= a.ldw;
  if (!fast) {
#pragma unroll
    for (int q = 0; q < 4; ++q) e2_stage_q(a, e0, i0, s, stg, q, withB);
    return withB ? 8 : 4;
  }
  const int wv = __builtin_amdgcn_readfirstlane(ef_wave());
  const char* ba = (const char*)(a.Ck + (long)s * E2_KS * a.ldk + e0);
  const char* bb = (const char*)(a.Et + (long)s * E2_KS * a.ldw + i0);
  const uint32_t mA = stg_lds + (uint32_t)(wv * 4 * 1024), mB = mA + E2_PANEL;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ef_dma_asm(ba, v.a[q], mA + q * 1024);
    if (withB) ef_dma_asm(bb, v.b[q], mB + q * 1024);
  }
  return withB ? 8 : 4;
}

// s_waitcnt vmcnt(n), n < 64 (immediate operand)
PT2Q_DEV void e2_vmcnt(int n) {
  switch (n) {
#define E2_W(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    E2_W(0) E2_W(1) E2_W(2) E2_W(3) E2_W(4) E2_W(5) E2_W(6) E2_W(7) E2_W(8) E2_W(9) E2_W(10) E2_W(11) E2_W(12)
    E2_W(13) E2_W(14) E2_W(15) E2_W(16) E2_W(17) E2_W(18) E2_W(19) E2_W(20) E2_W(21) E2_W(22) E2_W(23) E2_W(24)
    E2_W(25) E2_W(26) E2_W(27) E2_W(28) E2_W(29) E2_W(30) E2_W(31) E2_W(32) E2_W(33) E2_W(34) E2_W(35) E2_W(36)
    E2_W(37) E2_W(38) E2_W(39) E2_W(40) E2_W(41) E2_W(42) E2_W(43) E2_W(44) E2_W(45) E2_W(46) E2_W(47) E2_W(48)
    E2_W(49) E2_W(50) E2_W(51) E2_W(52) E2_W(53) E2_W(54) E2_W(55) E2_W(56) E2_W(57) E2_W(58) E2_W(59) E2_W(60)
    E2_W(61) E2_W(62)
#undef E2_W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int J, int JE>
PT2Q_DEV void ef_wbar_span(const int (&prow)[2], const u32x4 (&pend)[EF_CV], float* red) {
  if constexpr (J < JE) {
    ef_wbar_step<J>(prow, pend, red);
    ef_wbar_span<J + 1, JE>(prow, pend, red);
  }
}

// old values of column group rn (c[j], j = (rm * 2 + rn) * 4 + q: 8 loads), or their results
template <int RN>
PT2Q_DEV void e2_load(u32x4 (&c)[EF_CV], __amdgpu_buffer_rsrc_t rc, const uint32_t (&rb)[2]) {
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      c[(rm * 2 + RN) * 4 + q] = __builtin_amdgcn_raw_buffer_load_b128(rc, rb[rm] + 4 * (32 * RN + 8 * q), 0, 0);
}

template <int RN, int KS>
PT2Q_DEV void e2_sub(u32x4 (&c)[EF_CV], const EfAccT<KS>& F) {
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (rm * 2 + RN) * 4 + q;
#pragma unroll
      for (int u = 0; u < 4; ++u) c[j][u] = __float_as_uint(__uint_as_float(c[j][u]) - F.acc[rm][RN][4 * q + u]);
    }
}

// Column group 0's old Wt values are loaded this many stages before the tile's last (clamped to
// the first stage): 3 = at the tile's top, under all its MFMAs -- the grouped 16-linear 4096^2 loop
// 13.26-13.34 -> 12.93-13.03 ms (1 and 2 stages: 13.22-13.26; tools/ef2_g0_lib_ab.sh)
#ifndef PT2Q_EF2_G0_EARLY
#define PT2Q_EF2_G0_EARLY 3
#endif
// cache policy of the Wt stores (probe builds may set it: 16 = sc1, the line dropped from L2; 2 = nt)
#ifndef PT2Q_EF2_STORE_AUX
#define PT2Q_EF2_STORE_AUX 0
#endif
template <int RN>
PT2Q_DEV void e2_store(const u32x4 (&c)[EF_CV], __amdgpu_buffer_rsrc_t rc, const uint32_t (&rb)[2]) {
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(c[(rm * 2 + RN) * 4 + q], rc, rb[rm] + 4 * (32 * RN + 8 * q), 0,
                                             PT2Q_EF2_STORE_AUX);
}

// Column group 1's old values by LDS-DMA (G1L): 8 buffer-to-LDS loads per wave, 16 bytes per lane,
// into the wave's own chunks of a ring slot -- exactly the bytes its own stage DMAs (e2_stage: wave
// w owns A chunks (4 w + q) and B chunks E2_PANEL + (4 w + q) KiB) write next, so no other wave
// reads or writes them in between.  The loads are row-contiguous: load j brings rows 8 j .. 8 j + 7
// of the wave's 64 output rows, 8 lanes per row covering its 128-byte group-1 segment (a whole
// cache line per row, 8 lines per instruction -- the register-path loads touched 32 rows x 32
// bytes each); lane L of load j holds row 8 j + L / 8, 16-byte piece L % 8, and the epilogue
// reads each lane's own pieces back from there.
PT2Q_DEV uint32_t e2_g1_chunk(int wv, int j) {
  return (uint32_t)(j < 4 ? (wv * 4 + j) * 1024 : E2_PANEL + (wv * 4 + j - 4) * 1024);
}
PT2Q_DEV void e2_g1_dma(__amdgpu_buffer_rsrc_t rc, const uint32_t (&rb)[2], uint8_t* slot) {
  typedef __attribute__((address_space(3))) void* lptr;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(ef_wave());
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // row 8 j + lane / 8 of the wave: row block rm = j / 4, its base from that row's h = 0 lane
    const uint32_t src = (uint32_t)__shfl((int)rb[j >> 2], 8 * (j & 3) + (lane >> 3));
    const uint32_t off = src == EF_DROP ? EF_DROP : src + 4 * (32 + 4 * (lane & 7));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (lptr)(slot + e2_g1_chunk(wv, j)), 16, off, 0, 0, 0);
  }
}
PT2Q_DEV void e2_g1_read(u32x4 (&c)[EF_CV], const uint8_t* slot) {
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(ef_wave());
  const int li = lane & 31, h = lane >> 5;
#pragma unroll
  for (int rm = 0; rm < 2; ++rm)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = rm * 4 + (li >> 3), piece = ((li & 7) << 3) | (2 * q + h);
      c[(rm * 2 + 1) * 4 + q] = *(const u32x4*)(slot + e2_g1_chunk(wv, j) + 16 * piece);
    }
}

// NST = K stages per tile (2: bs <= 64, 4: bs <= 128; stages past bs are zero chunks: no-op pairs).
// Issue order per tile, for the hand-counted vmcnt waits: [next rows: 2] [stage s + 2 after each
// compute s (the last two: the next tile's stages 0 and 1)] with [old values, column group 0: 8]
// before stage G0S's compute (the tile's first; PT2Q_EF2_G0_EARLY); the epilogue then [waits for group 0] [loads group 1: 8]
// [stores group 0: 8] [waits for group 1] [stores it: 8] [w-bar partials: P].  So at the next
// tile's top only that tile's stores (SP) may still be in flight beside its stages.
// G1L (NST = 4): column group 1's old values come by LDS-DMA (e2_g1_dma) issued after stage 2's
// compute into the slot it freed, so their latency hides under stage 3's MFMAs instead of the
// epilogue's; the next tile's stage 0 then goes into stage 3's slot and its stage 1 into the
// group-1 slot once the waves have read it (mid-epilogue), so the slots' roles alternate from
// tile to tile (par).  Issue order: [rows: 2] [stage 2, 3 after compute 0, 1] [group 1: 8 after
// compute 2] [group 0 loads: 8] [next stage 0 after compute 3] [epilogue: stores 0: 8, next stage
// 1, stores 1: 8, w-bar: P].  Same products, same order: the same bits.
//
// TEAMS = 2 (development builds only, PT2Q_EF2_TEAMS): the two co-resident workgroups of a CU as
// the two teams (waves 0-3, 4-7) of one 8-wave workgroup, each with its own ring, tiles and w-bar
// scratch -- the same per-team code and bits -- but with every s_barrier common to both and team 1
// started a0.toff barriers behind team 0, to hold one team's epilogue under the other's MFMAs.
// Measured slower at every offset (13.9-14.4 vs 13.24 ms per 16-linear 4096^2 loop, offsets 0-7,
// tools/ef2_teams_ab.sh): the loop's MFMA work (6.8 ms at the f32 peak) and its Wt read-modify-
// write (33 GB, 6.6 ms at 5 TB/s) add up to the measured time, and the clock drops while both run
//  -- the coupling only adds barrier waits.
template <int NST, bool G1L = false, int TEAMS = 1>
__global__ __launch_bounds__(256 * TEAMS) __attribute__((amdgpu_waves_per_eu(2, 2))) void ef2_gemm_kernel(
    EfArgs a0, long wt_bytes, long part_bytes) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem_all[TEAMS][2 * E2_STAGE];
  __shared__ __attribute__((aligned(16))) float red_all[TEAMS][EF_RED];  // w-bar wave sums (ef_wbar_step)
  const int team = TEAMS > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8)) : 0;
  uint8_t* const smem = smem_all[team];
  float* const red = red_all[team];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  const int total = a0.ntile * a0.nz;
  const int tstride = (int)gridDim.x * TEAMS;
  int t = (int)blockIdx.x * TEAMS + team;
  if (t >= total) return;  // (a terminated wave leaves every later s_barrier of its workgroup)
  a0.probe |= PT2Q_EF2_KPROBE;
  PT2Q_EF2_CLK(0);
  auto corner = [&](int t, EfArgs& a, int& e0, int& i0) {
    const int z = t / a0.ntile, tl = t - z * a0.ntile;
    a = ef_linear(a0, z);
    e0 = (tl / a0.ti) * EF_T;
    i0 = (tl % a0.ti) * EF_T;
  };
  auto rsrc = [&](const EfArgs& a) { return __builtin_amdgcn_make_buffer_rsrc(a.Wt, 0, (int)wt_bytes, 0x00020000); };
  auto prsrc = [&](const EfArgs& x) { return __builtin_amdgcn_make_buffer_rsrc(x.part, 0, (int)part_bytes, 0x00020000); };
  const int P = a0.part ? EF_PS : 0;  // w-bar partial stores per wave per tile
  EfArgs a;
  int e0, i0, wrow[2];
  corner(t, a, e0, i0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  ef_rows(a, e0, wrow);
  E2Vo vo;
  e2_voff(a0, vo);
  // de-phase the two workgroups of a CU (the second half of the grid lands on CUs already holding
  // one): identical tiles would keep them in lock step, both in their MFMA stages or both in their
  // epilogues at once (PT2Q_EF2_STAGGER = sleeps of ~4K cycles; development knob)
  if (a0.stagger > 0 && (int)blockIdx.x >= (int)gridDim.x / 2)
    for (int z = a0.stagger; z > 0; --z) __builtin_amdgcn_s_sleep(64);
  e2_stage(a, e0, i0, 0, smem, lds0, vo, true);
  int Dn1 = e2_stage(a, e0, i0, 1, smem + E2_STAGE, lds0 + E2_STAGE, vo, true);
  if (TEAMS > 1 && team == 1)  // behind team 0 (10 barriers per tile)
    for (int k = 0; k < a0.toff; ++k) asm volatile("s_barrier" ::: "memory");
  int SP = 0;
  int par = 0;  // G1L: the slot of this tile's stage 0 (stage s in slot (s + par) & 1)
  static_assert(!G1L || NST == 4, "G1L: four K stages per tile");
  constexpr int G0S = NST - 1 - PT2Q_EF2_G0_EARLY < 0 ? 0 : NST - 1 - PT2Q_EF2_G0_EARLY;
  for (;;) {
    const int tn = t + tstride;
    const bool more = tn < total;
    int en = e0, in = i0, nrow[2];
    EfArgs an = a;
    if (more) corner(tn, an, en, in);
    // the next tile's stage j lands in the slot that held this tile's stage NST - 2 + j: its E
    // panel is still there only when that is the same stage (NST == 2), same linear, same i0
    const bool newB = NST != 2 || !(more && an.Et == a.Et && in == i0);
    const __amdgpu_buffer_rsrc_t rc = rsrc(a);
    uint32_t rb[2];
    ef_rowbase(a, wrow, i0, rb);
    if (a0.probe & 1) rb[0] = rb[1] = EF_DROP;
    // probe tools only (build-time PT2Q_EF2_KPROBE 8 / 16): the old-value loads / the stores go to
    // the first rows of Wt (L2-hot) -- same instructions and counts, results garbage
    uint32_t rbl[2] = {rb[0], rb[1]}, rbs[2] = {rb[0], rb[1]};
    if constexpr ((PT2Q_EF2_KPROBE & 8) != 0) rbl[0] = rbl[1] = 0;
    if constexpr ((PT2Q_EF2_KPROBE & 16) != 0) rbs[0] = rbs[1] = 0;
    ef_rows(an, en, nrow);  // 2 loads, issued by every wave whether or not a next tile exists
    EfAccT<E2_KS> F;
#pragma unroll
    for (int rm = 0; rm < 2; ++rm)
#pragma unroll
      for (int rn = 0; rn < 2; ++rn) F.acc[rm][rn] = f32x16{};
    u32x4 c[EF_CV];
    int X[NST];  // DMAs issued after compute s (into the slot it freed)
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      // this stage landed: everything younger than it may still be in flight (G1L: the stage-1
      // DMA of this tile was issued after the previous tile's group-0 stores, not before them)
      // (group 0's old values issued after stage 0's wait are younger than stage 1's DMAs)
      const int young = s == 0   ? Dn1 + SP + 2
                        : s == 1 ? (G1L && SP > 0 ? SP - EF_CV / 2 : SP) + 2 + (G0S == 0 ? EF_CV / 2 : 0) + X[0]
                                 : X[s - 1];
      e2_vmcnt(young);
      asm volatile("s_barrier" ::: "memory");
      if (s == G0S) e2_load<0>(c, rc, rbl);  // column group 0's old values (PT2Q_EF2_G0_EARLY)
      const int sl = G1L ? (s + par) & 1 : s & 1;
      EfNoIO nio;
      if (!(a0.probe & 4)) F.half(lds0 + sl * E2_STAGE, nio);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave done with the slot
      uint8_t* slot = smem + sl * E2_STAGE;
      const uint32_t slot_lds = lds0 + sl * E2_STAGE;
      if (s + 2 < NST) {
        X[s] = e2_stage(a, e0, i0, s + 2, slot, slot_lds, vo, true);
      } else if (G1L && s == NST - 2) {
        e2_g1_dma(rc, rbl, slot);  // column group 1's old values into the slot stage 2 freed
        X[s] = EF_CV / 2;
      } else if (G1L) {
        X[s] = more ? e2_stage(an, en, in, 0, slot, slot_lds, vo, newB) : 0;
      } else if (more) {
        X[s] = e2_stage(an, en, in, s + 2 - NST, slot, slot_lds, vo, newB);
        if (s == NST - 1) Dn1 = X[s];
      } else {
        X[s] = 0;
      }
    }
    e2_vmcnt(X[NST - 1]);  // column group 0's old values landed (G1L: and group 1's, older)
    e2_sub<0>(c, F);
    if constexpr (!G1L) e2_load<1>(c, rc, rbl);  // before group 0's stores: waiting for it then leaves those in flight
    e2_store<0>(c, rc, rbs);
    if (P) {  // this tile's w-bar partials (the next block's SSR mean, DESIGN.md §3 CHUNK128)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // red free (last readers done)
      ef_wbar_span<0, 16>(wrow, c, red);
    }
    if constexpr (G1L) {
      uint8_t* g1 = smem + par * E2_STAGE;  // stage 2's slot
      e2_g1_read(c, g1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's chunks read: its DMAs may overwrite them
      Dn1 = more ? e2_stage(an, en, in, 1, g1, lds0 + par * E2_STAGE, vo, newB) : 0;
      par ^= 1;
    } else {
      e2_vmcnt(EF_CV / 2);  // group 1 landed (younger: group 0's stores)
    }
    e2_sub<1>(c, F);
    e2_store<1>(c, rc, rbs);
    if (P) {
      ef_wbar_span<16, 32>(wrow, c, red);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      ef_wbar_store(a0.n, prsrc(a), true, e0, i0, red);
    }
    SP = EF_CV + P;
    if (!more) break;
    t = tn;
    a = an;
    e0 = en;
    i0 = in;
    wrow[0] = nrow[0];
    wrow[1] = nrow[1];
  }
  PT2Q_EF2_CLK(1);
}

}  // namespace

// Wt[crow[e]][i] -= sum_k Ck[k][e] * Et[k][i] for e < nr, i < ldw (the padding columns of Wt
// beyond n are scratch), k < bs <= 128.  Wt has wt_rows rows of ldw floats.
int pt2q_launch_ef(const float* Ck, long ldk, const float* Et, float* Wt, long ldw, long wt_rows,
                   const int* crow, int nr, int bs, hipStream_t st, const Grp* grp, float* part, int n) {
  if (nr <= 0) return PT2Q_OK;
  const long wt_bytes = wt_rows * ldw * 4;
  const long part_bytes = part ? (long)ceil_div(nr, EF_T) * n * 4 : 0;
  if (bs <= 0 || bs > 2 * EF_KH || ldw % 4 || ldk % 4 || (uintptr_t)Ck % 16 || (uintptr_t)Et % 16 ||
      (uintptr_t)Wt % 16 || wt_bytes >= (long)EF_DROP || wt_rows > 65536)
    return PT2Q_E_UNSUPPORTED;
  if (part && (n <= 0 || n % 4 || n > ldw || (uintptr_t)part % 16 || part_bytes >= (long)EF_DROP))
    return PT2Q_E_UNSUPPORTED;
  EfArgs a{Ck, ldk, Et, Wt, ldw, crow, nr, bs, ceil_div(nr, EF_T), ceil_div(ldw, EF_T), 0, bs > EF_KH ? 2 : 1,
           grp ? grp->ws : 0l, (int)grp_z(grp), part, n, pt2q_tuning().ef2_stagger, pt2q_tuning().ef2_probe,
           pt2q_tuning().ef2_team_offset};
  a.ntile = a.te * a.ti;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (pt2q_tuning().ef_v2 == 1) {  // two workgroups per CU (ef2_gemm_kernel)
    // workgroups per CU (PT2Q_EF2_PER_CU, 1 or 2): with one, another lane's latency-bound
    // kernels (SSR, ATQ) find registers and LDS beside the error feedback on every CU
    const int grid2 = std::min(a.ntile * a.nz, pt2q_tuning().ef2_per_cu * cus);
#ifdef PT2Q_DEV_PROBES
    // two barrier-coupled teams (development A/B only: 13.9-14.4 vs 13.24 ms per 16-linear loop
    // at every offset, tools/ef2_teams_ab.sh)
    if (bs > 2 * E2_KS && pt2q_tuning().ef2_teams == 2) {  // one 8-wave workgroup of two teams per CU
      const int gridt = std::min(ceil_div(a.ntile * a.nz, 2), cus);
      hipLaunchKernelGGL((ef2_gemm_kernel<4, true, 2>), dim3(gridt), dim3(512), 0, st, a, wt_bytes, part_bytes);
      PT2Q_LAUNCH_CHECK();
      return PT2Q_OK;
    }
#endif
    if (bs <= 2 * E2_KS)
      hipLaunchKernelGGL(ef2_gemm_kernel<2>, dim3(grid2), dim3(256), 0, st, a, wt_bytes, part_bytes);
#ifdef PT2Q_DEV_PROBES
    else if (!pt2q_tuning().ef2_g1lds)  // development A/B only (PT2Q_EF2_G1LDS=0)
      hipLaunchKernelGGL(ef2_gemm_kernel<4>, dim3(grid2), dim3(256), 0, st, a, wt_bytes, part_bytes);
#endif
    else
      hipLaunchKernelGGL((ef2_gemm_kernel<4, true>), dim3(grid2), dim3(256), 0, st, a, wt_bytes, part_bytes);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
#ifdef PT2Q_DEV_PROBES
  const int grid = std::min(a.ntile * a.nz, cus);
  hipLaunchKernelGGL(ef_gemm_kernel, dim3(grid), dim3(256), 0, st, a, wt_bytes, part_bytes);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
#else
  return PT2Q_E_UNSUPPORTED;  // unreachable: ef_v2 is 1 in a release library
#endif
}
