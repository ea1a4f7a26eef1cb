// Per-channel ATQ rows (block = every column of the layer, b = m > 512): init -> ITF -> AGA on the
// caller's row-major W, codes kept on-chip between the ITF passes.
//
// Reference: quantizer.py:32-248 (ternary_init, build_optimal_grid, flexible_round,
// iterative_ternary_fitting, activation_aware_grid_alignment) at block_size = m (main.py:176-189
// with one block; BASELINE config 5, Llama-2-13B per-channel).
//
// The arithmetic is atq.hip's wide path, term for term: a wave holds 4 rows, the 16 lanes of a row
// own the columns k = l + 16 s (SUM16 partials, one chain per lane in s order, bfly16 folds), so
// every value is bit-identical to atq_wide_block_kernel and to the oracle.  What changes is where
// the data lives between the passes (sum w, sum |w - mu|, init, one per ITF iteration, AGA + the
// code write):
//  * W is streamed once per pass in chunks of 512 columns (1 KiB of a bf16 row): each lane loads
//    16-byte pieces of its wave's 4 rows into registers one chunk ahead, stores them into a
//    wave-private two-stage LDS ring (row stride 1056 B: rows 8 banks apart), and reads back its
//    own strided elements (ds_read_u16 / b32 at 32 B steps) -- 16-byte global loads instead of one
//    2-byte load per element, no code loads or stores at all;
//  * the codes live as two bit masks per lane and chunk (Z: t != 0, S: t < 0 where Z), 2 bits per
//    element in a wave-private LDS area, so an ITF pass writes nothing to global memory; sum t and
//    sum t^2 (exact integers) come from popcounts of the masks; T is written once, in the last
//    pass.
// The codes of one pass are compared with the previous pass's masks for the wave-level ITF stop.
#include <algorithm>
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace {

constexpr int PC_COLS = 512;   // columns per chunk: 32 per lane
constexpr int PC_J = 32;       // elements per lane per chunk
constexpr int PC_WAVES = 2;    // waves (4 rows each) per workgroup
constexpr int PCR_NW = 10;     // register-resident rows: m = 512 * PCR_NW (5120: Llama-2-13B)

template <class T>
using lds_t = __attribute__((address_space(3))) T;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef lds_t<char> lds_char;

// storage type of W: element bytes and the exact conversion of its raw bits to fp32
template <class TI>
struct PcIn;
template <>
struct PcIn<uint16_t> {  // bf16 bits
  static constexpr int E = 2;
  PT2Q_DEV static float cvt(uint32_t raw) { return __uint_as_float(raw << 16); }
};
template <>
struct PcIn<_Float16> {
  static constexpr int E = 2;
  PT2Q_DEV static float cvt(uint32_t raw) { return (float)__builtin_bit_cast(_Float16, (uint16_t)raw); }
};
template <>
struct PcIn<float> {
  static constexpr int E = 4;
  PT2Q_DEV static float cvt(uint32_t raw) { return __uint_as_float(raw); }
};

template <class TI>
struct PcGeom {
  static constexpr int E = PcIn<TI>::E;
  static constexpr int CHUNK_B = PC_COLS * E;          // bytes of one row's chunk
  static constexpr int ROWB = CHUNK_B + 16 * E;        // LDS row stride: rows 8 (E=2) / 16 (E=4) banks apart
  static constexpr int STAGE = 4 * ROWB;               // one chunk of the wave's 4 rows
  static constexpr int PIECES = CHUNK_B / 16 / 64 * 4;  // 16-byte pieces per lane per chunk (4 or 8)
  static_assert(CHUNK_B % 1024 == 0, "a row's chunk is whole 1 KiB wave loads");
};

struct PcArgs {
  const void* W;     // n x m row-major (ldw elements)
  long ldw;
  int n, m;
  const float* S1;   // m, or nullptr (no AGA)
  const float* d;    // device scalar (AGA)
  int max_iter;
  float* alpha;      // n
  float* mu;         // n
  void* T;           // n x m row-major codes (ldt), int8 or fp32
  long ldt;
  int* iters;        // atomicMax of the wave iteration counts
  int* counters;     // [0] rows whose init codes are all zero
  int probe;         // development knock-outs (PT2Q_ATQ_PROBE, DEV_PROBES builds; results garbage):
                     // 1 = no code stores, 2 = AGA with S1 = 1 (no S1 loads), 4 = ITF skipped
};

// A wave's LDS: ONE ring stage (the streamed kernel), then its code masks.  The stage is
// wave-private and the LDS unit runs a wave's instructions in order, so the next chunk's stores
// may follow the current chunk's read-back into the same bytes without a wait (a second stage
// would only cost LDS: at m = 13824, 22.3 KiB per wave held the kernel to 6 waves per CU; one
// stage, 18.0 KiB, lets the 8 its registers allow fit).
constexpr int PC_RING = 1;
__host__ __device__ inline size_t pc_wave_bytes(int stage, int nchunks) {
  return PC_RING * (size_t)stage + (size_t)nchunks * 64 * 8;
}

// One wave's 4 rows, streamed pass by pass.
template <class TI>
struct PcRows {
  typedef PcGeom<TI> G;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const PcArgs& A;
  int lane, l, r;       // lane, residue class (column k = l + 16 s), row of the wave (0..3)
  int i;                // this lane's row (clamped to 0 when invalid: loads stay in range)
  bool valid;
  int nc;               // chunks per pass
  const char* rowp[4];  // the wave's 4 rows (clamped)
  lds_char* ring;       // wave-private: 2 stages, then the masks [chunk][lane] (Z, S)
  lds_char* masks;
  int par = 0;           // parity of the stream position q (which runs on across passes)
  int c3 = 0;            // chunk of q + 3 (= (q + 3) % nc, advanced incrementally)
  u32x4 stg[2][G::PIECES];  // the next two chunks' pieces (registers, in flight)

  PT2Q_DEV void load_chunk(int c, u32x4 (&dst)[G::PIECES]) const {  // global -> registers: piece p =
#pragma unroll                                                       // row p % 4, 1 KiB part p / 4
    for (int p = 0; p < G::PIECES; ++p) {
      const long off = (long)c * G::CHUNK_B + (p / 4) * 1024 + 16 * lane;
      const long lim = (long)A.m * G::E;  // m % (16 / E) == 0: pieces never straddle the row end
      dst[p] = *(const u32x4*)(rowp[p % 4] + (off < lim ? off : 0));
    }
  }
  PT2Q_DEV void store_stage(int st, const u32x4 (&src)[G::PIECES]) {  // registers -> LDS stage st
#pragma unroll
    for (int p = 0; p < G::PIECES; ++p)
      *(lds_t<u32x4>*)(ring + (st % PC_RING) * G::STAGE + (p % 4) * G::ROWB + (p / 4) * 1024 + 16 * lane) = src[p];
  }
  // this lane's 32 elements of the chunk in stage st (element j = column c*512 + l + 16 j)
  PT2Q_DEV void read_stage(int st, float (&x)[PC_J]) const {
    const lds_char* b = ring + (st % PC_RING) * G::STAGE + r * G::ROWB + G::E * l;
#pragma unroll
    for (int j = 0; j < PC_J; ++j) {
      uint32_t raw;
      if constexpr (G::E == 2) raw = *(const lds_t<uint16_t>*)(b + 32 * j);
      else raw = *(const lds_t<uint32_t>*)(b + 64 * j);
      x[j] = PcIn<TI>::cvt(raw);
    }
  }
  // The stream: at the start of step q, the stage holds chunk q, register set (q + 1) & 1 chunk
  // q + 1 and set q & 1 chunk q + 2 (both in flight).  Every pass reads the same chunks in the
  // same order, so the stream wraps from one pass into the next without a cold restart, and each
  // chunk's loads are issued two chunks ahead.
  PT2Q_DEV void prime() {
    load_chunk(0, stg[0]);
    store_stage(0, stg[0]);
    load_chunk(1 % nc, stg[1]);
    load_chunk(2 % nc, stg[0]);
    c3 = 3 % nc;
  }
  template <int P>
  PT2Q_DEV void step(float (&x)[PC_J]) {  // P = q & 1 (static: the register sets never move)
    read_stage(P, x);
    asm volatile("" ::: "memory");   // (one stage: the stores below follow the reads in LDS order)
    store_stage(P ^ 1, stg[P ^ 1]);  // chunk q + 1 (into the bytes just read back)
    load_chunk(c3, stg[P ^ 1]);      // chunk q + 3
    c3 = c3 + 1 == nc ? 0 : c3 + 1;
  }
  // One streamed pass: f.template chunk<TAIL>(rows, c, x, jn, masks) for every chunk in order (jn:
  // this lane's elements in the chunk, < 32 only in the last chunk).  No barriers: the ring is
  // wave-private.
  template <typename F>
  PT2Q_DEV void pass(F&& f) {
    for (int c = 0; c < nc; ++c, par ^= 1) {
      float x[PC_J];
      if (par) step<1>(x);
      else step<0>(x);
      u32x2 mk = {0u, 0u};
      if constexpr (std::decay_t<F>::MASKS_IN) mk = *mask_at(c);
      if ((c + 1) * PC_COLS <= A.m) {  // wave-uniform
        f.template chunk<false>(*this, c, x, PC_J, mk);
      } else {
        const int rem = A.m - c * PC_COLS - l;  // columns of this residue class left (< 512)
        f.template chunk<true>(*this, c, x, rem > 0 ? (rem + 15) / 16 : 0, mk);
      }
      if constexpr (std::decay_t<F>::MASKS_OUT) *mask_at(c) = mk;
    }
  }
  PT2Q_DEV lds_t<u32x2>* mask_at(int c) const { return (lds_t<u32x2>*)masks + c * 64 + lane; }
};

// The register-resident rows (bf16 W, m = 512 NW: C5's 5120 columns at NW = 10): the
// lane's 32 NW elements held as 16-bit pairs (element 2p in the low half of wr[p], 2p + 1 in the
// high half), the masks in registers; the passes are fully unrolled, W is read from HBM once.
template <class TI, int NW>
struct PcRegs {
  const PcArgs& A;
  int lane, l, r, i;
  bool valid;
  uint32_t wr[16 * NW];
  u32x2 M[NW];
  // W into the registers: 16-byte loads of the wave's 4 rows, staged through a wave-private
  // two-stage LDS ring (PcRows' geometry, loads two chunks ahead), each lane reading back its
  // strided elements.  (One 2-byte load per element, 320 per lane in batches of 16 with a wait
  // after each, left the waves parked 34 % of their cycles.)
  PT2Q_DEV void load(const char* const (&rowp)[4], lds_char* ring) {
    typedef PcGeom<TI> G;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 stg[2][4];
    auto ld = [&](int c, u32x4 (&dst)[4]) {
#pragma unroll
      for (int p = 0; p < 4; ++p) dst[p] = *(const u32x4*)(rowp[p] + (long)c * G::CHUNK_B + 16 * lane);
    };
    auto st = [&](int sg, const u32x4 (&src)[4]) {
#pragma unroll
      for (int p = 0; p < 4; ++p) *(lds_t<u32x4>*)(ring + sg * G::STAGE + p * G::ROWB + 16 * lane) = src[p];
    };
    ld(0, stg[0]);
    st(0, stg[0]);
    if (NW > 1) ld(1, stg[1]);
    if (NW > 2) ld(2, stg[0]);
#pragma unroll
    for (int c = 0; c < NW; ++c) {
      const lds_char* b = ring + (c & 1) * G::STAGE + r * G::ROWB + 2 * l;
#pragma unroll
      for (int p = 0; p < 16; ++p) {  // elements 2p, 2p + 1 of the chunk: columns +32p, +32p + 16
        const uint32_t lo = *(const lds_t<uint16_t>*)(b + 64 * p);
        const uint32_t hi = *(const lds_t<uint16_t>*)(b + 64 * p + 32);
        wr[16 * c + p] = lo | (hi << 16);
      }
      if (c + 1 < NW) {
        st((c + 1) & 1, stg[(c + 1) & 1]);
        if (c + 3 < NW) ld(c + 3, stg[(c + 1) & 1]);
      }
    }
  }
  // Makes a chunk's 16 packed registers opaque to the optimiser: without it, LLVM unpacks every
  // element once (320 fp32 registers, spilled) -- at the load, and by hoisting a pass's unpacks out
  // of the ITF loop.  No instruction is emitted.
  PT2Q_DEV void opaque(int c) {
    uint32_t* v = wr + 16 * c;
    asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                 "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]),
                 "+v"(v[14]), "+v"(v[15]));
  }
  PT2Q_DEV float elem(int s) const {
    const uint32_t v = wr[s >> 1];
    if constexpr (std::is_same<TI, uint16_t>::value)
      return __uint_as_float((s & 1) ? (v & 0xffff0000u) : (v << 16));
    else
      return (float)__builtin_bit_cast(_Float16, (uint16_t)((s & 1) ? (v >> 16) : v));
  }
  template <typename F>
  PT2Q_DEV void pass(F&& f) {
#pragma unroll
    for (int c = 0; c < NW; ++c) {
      opaque(c);
      float x[PC_J];
#pragma unroll
      for (int j = 0; j < PC_J; ++j) x[j] = elem(32 * c + j);
      f.template chunk<false>(*this, c, x, PC_J, M[c]);
      asm volatile("" ::: "memory");  // one chunk's loads / stores at a time (register pressure)
    }
  }
};

// ---- the passes (each mirrors its atq.hip wide_* counterpart's per-element arithmetic)

struct PcSumW {  // sum w (wide_sum_w)
  static constexpr bool MASKS_IN = false, MASKS_OUT = false;
  float p = 0.0f;
  template <bool TAIL, class R>
  PT2Q_DEV void chunk(const R&, int, const float (&x)[PC_J], int jn, u32x2&) {
#pragma unroll
    for (int j = 0; j < PC_J; ++j)
      if (!TAIL || j < jn) p = p + x[j];
  }
};

struct PcSumAbs {  // sum |w - mu| (wide_init, first pass)
  static constexpr bool MASKS_IN = false, MASKS_OUT = false;
  float mu, p = 0.0f;
  template <bool TAIL, class R>
  PT2Q_DEV void chunk(const R&, int, const float (&x)[PC_J], int jn, u32x2&) {
#pragma unroll
    for (int j = 0; j < PC_J; ++j)
      if (!TAIL || j < jn) p = p + fabsf(x[j] - mu);
  }
};

// ternary_init's codes (wide_init, second pass) with the first grid's partials; masks written
struct PcInit {
  static constexpr bool MASKS_IN = false, MASKS_OUT = true;
  float mu, delta;
  float pn = 0.0f, pwt = 0.0f;
  int nz = 0, neg = 0;
  template <bool TAIL, class R>
  PT2Q_DEV void chunk(const R&, int, const float (&x)[PC_J], int jn, u32x2& mk) {
    uint32_t zn = 0, sn = 0;
#pragma unroll
    for (int j = 0; j < PC_J; ++j) {
      const float w = x[j];
      const float wc = w - mu;
      const bool cp = wc > delta, cq = wc < -delta;
      const bool ok = !TAIL || j < jn;
      const float t = (ok && cp) ? 1.0f : ((ok && cq) ? -1.0f : 0.0f);
      pn = fmaf(t, wc, pn);  // t * wc exact; t = 0 adds +-0: p is never -0 (it starts at +0)
      pwt = fmaf(w, t, pwt);
      zn = (zn << 1) | (uint32_t)(t != 0.0f);
      sn = (sn << 1) | (uint32_t)(t < 0.0f);
    }
    mk = u32x2{zn, sn};
    nz += __builtin_popcount(zn);
    neg += __builtin_popcount(sn);
  }
};

// one ITF iteration: flexible_round against (a, m) and the next grid's partials (wide_round_pass)
struct PcRound {
  static constexpr bool MASKS_IN = true, MASKS_OUT = true;
  float m;
  RoundTh th;
  float pwt = 0.0f;
  int nz = 0, neg = 0;
  bool changed = false;
  template <bool TAIL, class R>
  PT2Q_DEV void chunk(const R&, int, const float (&x)[PC_J], int jn, u32x2& mk) {
    const u32x2 old = mk;
    uint32_t zn = 0, sn = 0;
#pragma unroll
    for (int j = 0; j < PC_J; ++j) {
      const float w = x[j];
      const float dd = w - m;
      const bool cz = (fabsf(dd) - th.hs > th.eps) && (!TAIL || j < jn);
      const float t = cz ? copysignf(1.0f, dd) : 0.0f;
      pwt = fmaf(w, t, pwt);  // exact product (row_grid)
      zn = (zn << 1) | (uint32_t)cz;
      sn = __builtin_amdgcn_alignbit(sn, __float_as_uint(dd), 31);  // (sn << 1) | sign(dd)
    }
    sn &= zn;
    changed |= ((zn ^ old.x) | (sn ^ old.y)) != 0u;
    mk = u32x2{zn, sn};
    nz += __builtin_popcount(zn);
    neg += __builtin_popcount(sn);
  }
};

// activation_aware_grid_alignment (wide_aga) over the final codes, and the codes written to T
template <class TO>
struct PcAgaOut {
  static constexpr bool MASKS_IN = true, MASKS_OUT = false;
  const float* S1;  // nullable: codes only
  float pv = 0.0f, pws = 0.0f, pwts = 0.0f, pt2s = 0.0f;
  template <bool TAIL, class Rows>
  PT2Q_DEV void chunk(const Rows& R, int c, const float (&x)[PC_J], int jn, u32x2& mk) {
    const PcArgs& A = R.A;
    TO* trow = (TO*)A.T + (long)R.i * A.ldt + (long)c * PC_COLS + R.l;
    const float* s1 = S1 ? S1 + (long)c * PC_COLS + R.l : nullptr;
#pragma unroll
    for (int j = 0; j < PC_J; ++j) {
      if (TAIL && j >= jn) continue;
      const uint32_t bit = 1u << (PC_J - 1 - j);
      const float t = (mk.x & bit) ? ((mk.y & bit) ? -1.0f : 1.0f) : 0.0f;
#ifdef PT2Q_DEV_PROBES
      if (A.probe & 2) {
        const float w = x[j], cv = 1.0f;
        pv = fmaf(t, cv, pv);
        pws = fmaf(w, cv, pws);
        pwts = fmaf(w * t, cv, pwts);
        pt2s = fmaf(t * t, cv, pt2s);
        if (R.valid && !(A.probe & 1)) trow[16 * j] = (TO)t;
        continue;
      }
      if (A.probe & 1) {
        if (s1) {
          const float w = x[j], cv = s1[16 * j];
          pv = fmaf(t, cv, pv);
          pws = fmaf(w, cv, pws);
          pwts = fmaf(w * t, cv, pwts);
          pt2s = fmaf(t * t, cv, pt2s);
        }
        continue;
      }
#endif
      if (s1) {
        const float w = x[j], cv = s1[16 * j];
        pv = fmaf(t, cv, pv);
        pws = fmaf(w, cv, pws);
        pwts = fmaf(w * t, cv, pwts);
        pt2s = fmaf(t * t, cv, pt2s);
      }
      if (R.valid) trow[16 * j] = (TO)t;
    }
  }
};

// The row program on either data source R (PcRows: streamed, PcRegs: registers): sum w, sum
// |w - mu|, init, ITF, AGA + codes; alpha / mu written by lane l = 0 of each row.
template <class TO, class R>
PT2Q_DEV void pc_rows(R& rows) {
  const PcArgs& A = rows.A;
  const float fb = (float)A.m;
  PcSumW sw;
  rows.pass(sw);
  const float wsum = bfly16(sw.p);
  // ternary_init (quantizer.py:32-69)
  const float mu0 = wsum / fb;
  PcSumAbs sa{mu0};
  rows.pass(sa);
  const float delta = 0.75f * (bfly16(sa.p) / fb);
  PcInit in{mu0, delta};
  rows.pass(in);
  const float num = bfly16(in.pn), cnt = bfly16((float)in.nz);
  float g[3] = {bfly16(in.pwt), bfly16((float)(in.nz - 2 * in.neg)), cnt};
  float a = num / clampmin(cnt), m = mu0;
  if (rows.valid && rows.l == 0 && cnt == 0.0f) atomicAdd(&A.counters[0], 1);
  // iterative_ternary_fitting (quantizer.py:136-175), wave-level stop (atq.hip wide_itf)
  int it = 0;
  bool any = true;
#ifdef PT2Q_DEV_PROBES
  if (A.probe & 4) any = false;
#endif
  for (; it < A.max_iter; ++it) {
    if (!any) break;
    {
      const float den = clampmin(fb * g[2] - g[1] * g[1]);
      a = (fb * g[0] - g[1] * wsum) / den;
      m = (g[2] * wsum - g[1] * g[0]) / den;
    }
    PcRound rd{m, round_th(clampmin(a))};
    rows.pass(rd);
    g[0] = bfly16(rd.pwt);
    g[1] = bfly16((float)(rd.nz - 2 * rd.neg));
    g[2] = bfly16((float)rd.nz);
    any = __any(rd.changed);
  }
  // AGA (quantizer.py:177-248) and the codes
  PcAgaOut<TO> ag{A.S1};
  rows.pass(ag);
  if (A.S1) {
    const float dv = *A.d;
    const float v = bfly16(ag.pv), ws1 = bfly16(ag.pws), wts1 = bfly16(ag.pwts), t2s1 = bfly16(ag.pt2s);
    const float v2 = v * v;
    const float den = clampmin(dv * t2s1 - v2);
    a = (dv * wts1 - v * ws1) / den;
    m = (t2s1 * ws1 - v * wts1) / den;
  }
  if (A.iters && rows.lane == 0) atomicMax(A.iters, it);
  if (rows.valid && rows.l == 0) {
    A.alpha[rows.i] = a;
    A.mu[rows.i] = m;
  }
}

// One row group (4 consecutive rows) per wave, a static grid.  (Claiming groups dynamically from a
// counter, so a wave takes the next group when its ITF ends, measured slower: the loop around the
// unrolled register-resident body raised its spills 47 -> 246 VGPRs, 230 -> 264 us per 5120-column
// linear; the streamed kernel 498 -> 517 us per 5120 x 13824.)
//
// Grouped launches (PcGroup): the rows of up to PC_GROUP_MAX linears of one width in ONE 1-D grid,
// linear z taking workgroups [wg0[z], wg0[z + 1]) -- a single 5120-row linear fills only 1.25
// waves per SIMD, so launched alone its last wave leaves most of the chip idle; a group of 16
// keeps every SIMD at the kernel's occupancy until the grid drains.  Per row, the program and its
// arithmetic are unchanged (the same bits).
struct PcGroup {
  int count;
  int wg0[PT2Q_PC_GROUP_MAX + 1];
  PcArgs a[PT2Q_PC_GROUP_MAX];
};

// This workgroup's linear (its args, selected with constant indices so they stay in scalar
// registers: a dynamically indexed kernarg array is copied to scratch) and its workgroup index.
PT2Q_DEV PcArgs pc_linear(const PcGroup& G, int& wg) {
  const int b = (int)blockIdx.x;
  PcArgs A = G.a[0];
  wg = b;
#pragma unroll
  for (int k = 1; k < PT2Q_PC_GROUP_MAX; ++k)
    if (k < G.count && b >= G.wg0[k]) {
      A = G.a[k];
      wg = b - G.wg0[k];
    }
  return A;
}

template <class TI, class TO>
__global__ __launch_bounds__(64 * PC_WAVES) void atq_pc_kernel(PcGroup G) {
  extern __shared__ __attribute__((aligned(16))) char pc_lds[];
  typedef PcGeom<TI> G_;
  int wg;
  const PcArgs A = pc_linear(G, wg);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nc = (A.m + PC_COLS - 1) / PC_COLS;
  PcRows<TI> R{A, lane, lane & 15, lane >> 4, 0, false, nc, {}, nullptr, nullptr};
  const int row0 = (wg * PC_WAVES + wave) * 4;
  R.i = row0 + R.r;
  R.valid = R.i < A.n;
  if (!R.valid) R.i = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int iq = row0 + q < A.n ? row0 + q : 0;
    R.rowp[q] = (const char*)A.W + (long)iq * A.ldw * G_::E;
  }
  R.ring = (lds_char*)pc_lds + (size_t)wave * pc_wave_bytes(G_::STAGE, nc);
  R.masks = R.ring + PC_RING * G_::STAGE;
  R.prime();
  pc_rows<TO>(R);
}

constexpr int PCR_WAVES = 4;
template <class TI, class TO, int NW>
__global__ __launch_bounds__(64 * PCR_WAVES) __attribute__((amdgpu_waves_per_eu(2, 2))) void atq_pcr_kernel(PcGroup G) {
  typedef PcGeom<TI> G_;
  __shared__ __attribute__((aligned(16))) char ring_lds[PCR_WAVES * 2 * G_::STAGE];
  int wg;
  const PcArgs A = pc_linear(G, wg);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  PcRegs<TI, NW> R{A, lane, lane & 15, lane >> 4, 0, false, {}, {}};
  const int row0 = (wg * PCR_WAVES + wave) * 4;
  R.i = row0 + R.r;
  R.valid = R.i < A.n;
  if (!R.valid) R.i = 0;
  const char* rowp[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) rowp[q] = (const char*)A.W + (long)(row0 + q < A.n ? row0 + q : 0) * A.ldw * 2;
  R.load(rowp, (lds_char*)ring_lds + wave * 2 * G_::STAGE);
  pc_rows<TO>(R);
}

}  // namespace

// Whether the streamed per-channel kernel takes this call (else atq.hip's wide kernel): 16-byte
// aligned rows whose length is whole 16-byte pieces, and the LDS the wave areas need.
bool pt2q_atq_pc_supported(const void* W, int wdtype, long ldw, int m) {
  if (!pt2q_tuning().atq_pc) return false;
  const int E = wdtype == PT2Q_F32 ? 4 : 2;
  if (wdtype != PT2Q_F32 && wdtype != PT2Q_F16 && wdtype != PT2Q_BF16) return false;
  if (((uintptr_t)W & 15) != 0 || (ldw * E) % 16 != 0 || (m * E) % 16 != 0 || m <= 512) return false;
  const int stage = 4 * (PC_COLS * E + 16 * E);
  return PC_WAVES * pc_wave_bytes(stage, ceil_div(m, PC_COLS)) <= 160 * 1024;
}

// Up to PT2Q_PC_GROUP_MAX linears of width m (every W accepted by pt2q_atq_pc_supported) in one
// launch; their row counts may differ.
int pt2q_launch_atq_pc_group(int count, const PcLinear* lin, int wdtype, int m, int max_iter, int tdtype,
                             hipStream_t st) {
  if (count <= 0 || count > PT2Q_PC_GROUP_MAX) return PT2Q_E_ARG;
  const bool regs = m == PC_COLS * PCR_NW && wdtype == PT2Q_BF16 && pt2q_tuning().atq_pc_regs;
  const int rows_wg = 4 * (regs ? PCR_WAVES : PC_WAVES);
  PcGroup G{};
  G.count = count;
  int wg = 0;
  for (int z = 0; z < count; ++z) {
    const PcLinear& L = lin[z];
    G.a[z] = PcArgs{L.W, L.ldw, L.n, m, L.S1, L.d, max_iter, L.alpha, L.mu, L.T, L.ldt, L.iters, L.counters,
                    pt2q_tuning().atq_probe};
    G.wg0[z] = wg;
    wg += ceil_div(L.n, rows_wg);
  }
  G.wg0[count] = wg;
  if (wg == 0) return PT2Q_OK;
  const bool i8 = tdtype == PT2Q_I8;
  if (regs) {
    auto gor = [&](auto ti, auto to) {
      hipLaunchKernelGGL((atq_pcr_kernel<decltype(ti), decltype(to), PCR_NW>), dim3(wg), dim3(64 * PCR_WAVES), 0,
                         st, G);
      PT2Q_LAUNCH_CHECK();
      return PT2Q_OK;
    };
    return i8 ? gor(uint16_t{}, int8_t{}) : gor(uint16_t{}, float{});
  }
  auto go = [&](auto ti, auto to) {
    typedef decltype(ti) TI;
    typedef decltype(to) TO;
    const size_t lds = PC_WAVES * pc_wave_bytes(PcGeom<TI>::STAGE, ceil_div(m, PC_COLS));
    hipLaunchKernelGGL((atq_pc_kernel<TI, TO>), dim3(wg), dim3(64 * PC_WAVES), lds, st, G);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  };
  switch (wdtype) {
    case PT2Q_F32: return i8 ? go(float{}, int8_t{}) : go(float{}, float{});
    case PT2Q_F16: return i8 ? go(_Float16{}, int8_t{}) : go(_Float16{}, float{});
    case PT2Q_BF16: return i8 ? go(uint16_t{}, int8_t{}) : go(uint16_t{}, float{});
  }
  return PT2Q_E_ARG;
}

int pt2q_launch_atq_pc(const void* W, int wdtype, long ldw, int n, int m, const float* S1, const float* d,
                       int max_iter, float* alpha, float* mu, void* T, int tdtype, long ldt, int* iters,
                       int* counters, hipStream_t st) {
  const PcLinear L{W, ldw, n, S1, d, alpha, mu, T, ldt, iters, counters, nullptr};
  return pt2q_launch_atq_pc_group(1, &L, wdtype, m, max_iter, tdtype, st);
}
