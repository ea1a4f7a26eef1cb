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

// Upper tiles of the 128 x 256 grid (tile (ti, tj) exists iff ti <= 2tj + 1), ordered by
// super-blocks of (2SJ) x SJ tiles (column-block major over super-blocks, column major inside
// one), so that a contiguous run of the order -- one XCD's share -- covers a compact square of
// G and its workgroups read few distinct panels of X through their common L2.
PT2Q_DEV int gx_col_count(int tj, int lo, int hi) {  // tiles ti in [lo, hi) of column tj
  return max(0, min(hi, 2 * tj + 2) - lo);
}

PT2Q_DEV void gx_tile(int a, int TI, int TJ, int SJ, int& ti, int& tj) {
  const int SI = 2 * SJ;
  for (int J = 0; J * SJ < TJ; ++J) {
    const int tj1 = min(TJ, (J + 1) * SJ);
    for (int I = 0; I * SI < TI; ++I) {
      const int lo = I * SI, hi = min(TI, lo + SI);
      int c = 0;
      for (int t = J * SJ; t < tj1; ++t) c += gx_col_count(t, lo, hi);
      if (a >= c) {
        a -= c;
        continue;
      }
      for (int t = J * SJ; t < tj1; ++t) {
        const int ct = gx_col_count(t, lo, hi);
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

long gx_ntile(int m) {
  const int TI = ceil_div(m, GX_BM), TJ = ceil_div(m, GX_BN);
  long s = 0;
  for (int t = 0; t < TJ; ++t) s += std::min(2 * t + 2, TI);
  return s;
}

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
#ifdef GX_PROBE_NO_DMA  // tools/gram16_probe.hip: compute-only timing (stale LDS)
  return;
#endif
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
#ifdef GX_PROBE_NO_MFMA  // tools/gram16_probe.hip: fetch-only timing
    return;
#endif
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

// g: M = N = m, K = rows, A = X (ld lda), C = G (ldc), mode STORE / ADD / CHAIN_POS.
// D data-parallel waves first: in wave v workgroup w = x + NG*r takes whole tile
// v*grid + x*R + r, so the R workgroups of one XCD run 32 neighbouring tiles of the order at the
// same k and share their X panels through that XCD's L2.  The rest of the tile line (stream-K)
// is cut into NG contiguous groups; group x is worked by workgroups w = x, x + NG, x + 2NG, ...
// (R of them), which on the round-robin dispatch share an XCD and so its L2 (speed only).
// Inside a group, team r/P takes rows [team*L, (team+1)*L) of the group's line of cnt * Kp rows
// (units of P tiles): tail piece first (chains from the start of its last unit), full units,
// then the head piece of its first unit, continuing the partial that the same member of the
// previous team (w - P*NG, dispatched earlier) published.  L >= Kp.  NG = 1 and L = Kp: no split.
template <bool BF16, bool DMA>
__global__ __launch_bounds__(256) void gram16x_kernel(GemmDesc g, int TI, int TJ, int SJ, int Kp, long ntile, int NG,
                                                      int R, int P, int D, int* flags, int* status,
                                                      long cap) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[GX_LDS];
  const uint16_t* X = (const uint16_t*)g.A;
  const int w = blockIdx.x;
  const int x = w % NG, r = w / NG;
  const long base = (long)D * gridDim.x;  // first stream-K tile
  // P = 2: the line is cut into tile pairs (2j, 2j+1), which share their column block tj, and
  // workgroups r = 2i, 2i+1 (a team) walk the same stretch of pairs in step, one tile of each
  // pair apiece, so the X panel of tj is fetched into L2 once for both.
  const int mem = r % P, team = r / P, nteam = R / P;
  const long npair = (ntile - base) / P;
  const long t0 = P * (npair * x / NG), cnt = npair * (x + 1) / NG - npair * x / NG;
  const long W = cnt * Kp;
  const long L = (R == 0) ? Kp : ((W + nteam - 1) / nteam + GX_BK - 1) / GX_BK * GX_BK;
  const long s = (long)team * L, e = min(s + L, W);
  const int a0 = (int)(s / Kp), k0 = (int)(s % Kp);
  const int a1 = (int)((e - 1) / Kp), k1 = (int)(e - (long)a1 * Kp);
  const bool head = k0 > 0;
  const bool tail = k1 < Kp && !(head && a1 == a0);
  const int f0 = head ? a0 + 1 : a0, f1 = tail ? a1 - 1 : a1;
  const int nfull = f1 >= f0 ? f1 - f0 + 1 : 0;
  const int npieces = s >= e ? 0 : (tail ? 1 : 0) + nfull + (head ? 1 : 0);
  const bool vec4 = ((uintptr_t)g.C % 16 == 0) && (g.ldc % 4 == 0);
  for (int pc = -D; pc < npieces; ++pc) {
    int a, kb, ke;
    bool from_partial = false;
    if (pc < 0) {
      a = (pc + D) * (int)gridDim.x + x * R + r; kb = 0; ke = Kp;
    } else {
      if (tail && pc == 0) {
        a = a1; kb = 0; ke = k1;
      } else if (head && pc == npieces - 1) {
        a = a0; kb = k0; ke = (a0 == a1) ? k1 : Kp; from_partial = true;
      } else {
        a = f0 + pc - (tail ? 1 : 0); kb = 0; ke = Kp;
      }
      a = (int)(base + t0) + P * a + mem;  // global tile index (flags are per tile)
    }
    int ti, tj;
    gx_tile(a, TI, TJ, SJ, ti, tj);
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

}  // namespace

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
  void (*k)(GemmDesc, int, int, int, int, long, int, int, int, int, int*, int*, long) =
      bf ? (dma ? gram16x_kernel<true, true> : gram16x_kernel<true, false>)
         : (dma ? gram16x_kernel<false, true> : gram16x_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, g, TI, TJ, SJ, Kp, ntile, NG, R, P, D, flags, status,
                     tu.spin_cap_long);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}
