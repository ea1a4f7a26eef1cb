// SSR (structural-similarity reordering) block selection and the error-feedback coefficients.
//
// Reference: reorder.py:36-61 (compute_column_similarity_to_mean), reorder.py:107-143
// (select_next_block_ssr), main.py:176-177 / gptq.py:142-150 (block operands),
// main.py:199-209 (coefficients Hinv[blk][:,rem] / diag).
//
// Weights live feature-major (Wt[j] = column j of W, contiguous over the n rows), so every
// "column" gather of the reference is a gather of whole contiguous rows here.
#include "common.hpp"
#include "internal.hpp"
#include "probe.hpp"

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

constexpr int CHUNK = 128;  // canonical wbar chunk (rem entries per partial sum)

// Leaf k of the CHUNK128 half tree: bfly16 over l in [0, 16) (leaves in 4-bit bit-reversed
// order), then the same over [16, 32), the two sums added.
PT2Q_DEV constexpr int brev5(int k) {
  return (k & 16) | ((k & 1) << 3) | ((k & 2) << 1) | ((k & 4) >> 1) | ((k & 8) >> 3);
}

// Half of a chunk's w-bar partial (DESIGN.md §3 CHUNK128): x_l = v[o+l] + v[o+l+32] (l < 32),
// bfly16(x[0..16)) + bfly16(x[16..32)), evaluated as a pairwise stack over the leaves in the
// tree's order, 8 leaves' loads in flight at a time.  ld(j) = v[j] (zero past the chunk's end).
template <typename V, typename LD>
PT2Q_DEV V wbar_half(LD&& ld, int o) {
  V acc[6];
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 8) {
    V a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = ld(o + brev5(k0 + u));
      b[u] = ld(o + brev5(k0 + u) + 32);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u;
      V v = a[u] + b[u];
      int lvl = 0;
#pragma unroll
      for (; lvl < 5 && ((k >> lvl) & 1); ++lvl) v = acc[lvl] + v;
      acc[lvl] = v;
    }
  }
  return acc[5];
}

// The w-bar partial of one chunk: X + Y (X over entries 0..63, Y over 64..127) -- the order the
// error-feedback tile that last wrote these columns forms it in (ef.hip), oracle orc_wbar_chunk.
template <typename V, typename LD>
PT2Q_DEV V wbar_chunk(LD&& ld) {
  const V x = wbar_half<V>(ld, 0);
  return x + wbar_half<V>(ld, 64);
}

// part[c][i] = wbar_chunk over rem[c*128 .. c*128+127] of Wt[rem[e]][i]
__global__ __launch_bounds__(256) void ssr_wbar_partial_kernel(const float* Wt, long ldw, int n,
                                                               const int* rem, int r,
                                                               float* part) {
  __shared__ long rows[CHUNK];
  const int c = blockIdx.x;
  const int e0 = c * CHUNK, cnt = min(r, e0 + CHUNK) - e0;
  for (int e = threadIdx.x; e < cnt; e += blockDim.x) rows[e] = (long)rem[e0 + e] * ldw;
  __syncthreads();
  const int i = blockIdx.y * 256 + threadIdx.x;
  if (i >= n) return;
  part[(long)c * n + i] = wbar_chunk<float>([&](int j) { return j < cnt ? Wt[rows[j] + i] : 0.0f; });
}

// The three wbar steps in one launch (n <= 16384, n % 4 == 0): every workgroup (one wave: 256
// rows i, four per lane, so the reads spread over every CU) forms its partial
// part[c][i] as ssr_wbar_partial_kernel; the last workgroup to finish a 256-row slice sums that
// slice's partials in chunk order (wbar = sum / r); the last slice to finish forms
// nw = clamp(sqrt(SUMN fma wbar^2)) and wn = wbar / nw.  Hand-offs: write-through (sc1) stores,
// drained by every storing wave before the barrier that precedes the counter add, and sc1 loads
// on the consuming side (no fences).  cnt: nslices + 1 ints, zero before the first launch; the
// last arrivers put them back to zero.
__global__ __launch_bounds__(256) void ssr_wbar_fused_kernel(const float* Wt, long ldw, int n,
                                                             const int* rem, int r, float* part,
                                                             float* wn, int* cnt, long zs, int pre) {
  __shared__ long rows[CHUNK];
  Wt = zws(Wt, zs);  // grouped launch: linear blockIdx.z's slice
  rem = zws(rem, zs);
  part = zws(part, zs);
  wn = zws(wn, zs);
  cnt = zws(cnt, zs);
  __shared__ int last;
  const int c = blockIdx.x, nchunks = (r + CHUNK - 1) / CHUNK, nsl = gridDim.y;
  const int e0 = c * CHUNK, ce = min(r, e0 + CHUNK) - e0;
  if (!pre) {
    for (int e = threadIdx.x; e < ce; e += blockDim.x) rows[e] = (long)rem[e0 + e] * ldw;
    __syncthreads();
  }
  // four consecutive rows i per thread (float4; n % 4 == 0), each its own chain over e
  typedef float f4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(part, 0, nchunks * n * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(wn, 0, n * 4, 0x00020000);
  const int i = (blockIdx.y * blockDim.x + threadIdx.x) * 4;
  if (!pre) {  // (pre: the partials came from the error feedback that wrote these columns)
    if (i < n) {
      const f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
      const f4 p = wbar_chunk<f4>([&](int j) { return j < ce ? *(const f4*)(Wt + rows[j] + i) : z; });
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, p), rp, (c * n + i) * 4, 0, 16);  // sc1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(cnt + blockIdx.y, 1) == nchunks - 1;
    __syncthreads();
    if (!last) return;
  }
  if (i < n) {
    f4 t = {0.0f, 0.0f, 0.0f, 0.0f};
    int k = 0;
    for (; k + 8 <= nchunks; k += 8) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rp, ((k + u) * n + i) * 4, 0, 16));
#pragma unroll
      for (int u = 0; u < 8; ++u) t = t + v[u];
    }
    for (; k < nchunks; ++k) t = t + __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rp, (k * n + i) * 4, 0, 16));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, t / (float)r), rw, i * 4, 0, 16);  // sc1
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(cnt + blockIdx.y, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = atomicAdd(cnt + nsl, 1) == nsl - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x >= 64) return;
  // wave 0: lane t takes elements {256u + 4t + q} (sumn_lane's order), 16 float4 in flight;
  // a second pass writes wn = wbar / nw (loads past n return zero, stores past n are dropped)
  const __amdgpu_buffer_rsrc_t rs = rw;
  const int t = threadIdx.x;
  float q = 0.0f;
  for (int u0 = 0; u0 < n; u0 += 4096) {
    f4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u0 + 4 * t + 256 * u) * 4, 0, 16));
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (u0 + 4 * t + 256 * u < n) {
        q = fmaf(v[u][0], v[u][0], q);
        q = fmaf(v[u][1], v[u][1], q);
        q = fmaf(v[u][2], v[u][2], q);
        q = fmaf(v[u][3], v[u][3], q);
      }
  }
  const float nw = clampmin(sqrtf(bfly64(q)));
  for (int u0 = 0; u0 < n; u0 += 4096) {
    f4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u0 + 4 * t + 256 * u) * 4, 0, 16));
#pragma unroll
    for (int u = 0; u < 16; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v[u] / nw), rs,
                                             (u0 + 4 * t + 256 * u) * 4, 0, 0);
  }
  if (t == 0) __hip_atomic_store(cnt + nsl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wbar[i] = (chunk partials summed in chunk order) / r
__global__ __launch_bounds__(256) void ssr_wbar_sum_kernel(const float* part, int nchunks, int n,
                                                           int r, float* wbar) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float t = 0.0f;
  for (int c = 0; c < nchunks; ++c) t = t + part[(long)c * n + i];
  wbar[i] = t / (float)r;
}

// wbar[i] = (chunk partials summed in chunk order) / r, then nw = clamp(sqrt(SUMN fma wbar^2))
// and wn = wbar / nw -- one workgroup, n <= SUMN_LDS_MAX (ssr_wbar_sum + ssr_wbar_final fused)
__global__ __launch_bounds__(1024) void ssr_wbar_sumfinal_kernel(const float* part, int nchunks,
                                                                 int n, int r, float* wn) {
  __shared__ float nws, tot;
  __shared__ float stage[SUMN_LDS_MAX];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float t = 0.0f;
    int c = 0;
    for (; c + 8 <= nchunks; c += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(c + u) * n + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) t = t + v[u];
    }
    for (; c < nchunks; ++c) t = t + part[(long)c * n + i];
    stage[i] = t / (float)r;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float p = sumn_lane<true>(stage, n, 1, threadIdx.x);
    p = bfly64(p);
    if (threadIdx.x == 0) nws = clampmin(sqrtf(p));
  }
  __syncthreads();
  const float nw = nws;
  for (int i = threadIdx.x; i < n; i += blockDim.x) wn[i] = stage[i] / nw;
  (void)tot;
}

// nw = clamp(sqrt(SUMN fma wbar^2)) ; wn = wbar / nw   (in place)
__global__ __launch_bounds__(1024) void ssr_wbar_final_kernel(float* wn, int n) {
  __shared__ float nws, tot;
  __shared__ float stage[SUMN_LDS_MAX];
  if (n <= SUMN_LDS_MAX) {
    const float p = block_sumn_lds<true>(wn, n, 1, stage, &tot);
    if (threadIdx.x == 0) nws = clampmin(sqrtf(p));
  } else if (threadIdx.x < 64) {
    float p = sumn_lane<true>(wn, n, 1, threadIdx.x);
    p = bfly64(p);
    if (threadIdx.x == 0) nws = clampmin(sqrtf(p));
  }
  __syncthreads();
  const float nw = nws;
  for (int i = threadIdx.x; i < n; i += blockDim.x) wn[i] = wn[i] / nw;
}

// RN(x / nj) from one correctly rounded reciprocal y = RN(1 / nj) (Markstein): with r = x - nj q
// exact (fma), RN(q + r y) = RN(x / nj) whenever q is within one ulp of x / nj and nothing
// underflows.  q0 = RN(x y) can be 1.5 ulp off, so one correction first brings it within
// 0.5 ulp + 2^-23 ulp, and the second is exact.  No underflow: every nonzero |x| >= 2^-80 and
// nj in [1e-8, 2^40] (nj >= |x|: the clamped norm of the column holding x), so |q| >= 2^-120 is
// normal and r (about 2^-24 |x|) is too.  x = 0 gives a zero quotient (its sign may differ from
// the division's: q0 = -0, the corrections +0), and a signed zero cannot change the similarity
// chain p = fma(q, w, p) -- p starts at +0 and an exactly-zero fma result is -0 only if both
// addends are, so p is never -0 and fma(+-0, w, p) = p.  A column with a nonzero |x| < 2^-80 or
// a norm above 2^40 takes the division (wave-uniform branch).  5 VALU instead of the division's
// scaled Newton sequence; pinned against the division by orc_fp_rule_mismatches (rule 1).
constexpr float RCP_X_MIN = 0x1p-80f, RCP_NJ_MAX = 0x1p40f;
PT2Q_DEV float div_rcp(float x, float nj, float y) {
  const float q0 = x * y;
  const float q1 = fmaf(fmaf(-nj, q0, x), y, q0);
  return fmaf(fmaf(-nj, q1, x), y, q1);
}
PT2Q_DEV bool rcp_column_ok(float minabs, float nj) { return minabs >= RCP_X_MIN && nj <= RCP_NJ_MAX; }
// The gate's re-check when a lane's min |x| failed it: the smallest NONZERO |x| of its registers
// (zeros -- pruned or padded weights -- keep the fast path; rare, so off the common path).
template <int U, typename V>
PT2Q_DEV float min_nonzero_abs(const V (&v)[U], int n, int t, int u0) {
  float mz = 0x1p64f;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (4 * t + 256 * (u0 + u) < n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) mz = fminf(mz, v[u][q] == 0.0f ? 0x1p64f : fabsf(v[u][q]));
    }
  return mz;
}

// One wave per remaining column: nj = clamp(sqrt(SUMN fma x^2)); s = SUMN fma (x/nj) * wn.
// NV > 0 (n % 4 == 0, n <= 256 NV): one pass over the column, its NV float4 per lane kept in
// registers for both chains; NV == 0: the generic two-pass paths.
template <int NV>
__global__ __launch_bounds__(256) void ssr_sim_kernel(const float* Wt, long ldw, int n,
                                                      const int* rem, int r, const float* wn,
                                                      float* sim, long zs) {
  Wt = zws(Wt, zs);  // grouped launch: linear blockIdx.z's slice
  rem = zws(rem, zs);
  wn = zws(wn, zs);
  sim = zws(sim, zs);
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int t = threadIdx.x & 63;
  if (e >= r) return;
  const float* x = Wt + (long)rem[e] * ldw;
  float p = 0.0f;
  typedef float f4 __attribute__((ext_vector_type(4)));
  if constexpr (NV > 0) {
    // NV <= 16: the column and the (shared, L2-resident) mean vector are both loaded up front, so
    // the dot pass does not wait a second L2 round trip after the norm (NV = 48 keeps the mean's
    // loads in the dot loop: 256 VGPRs)
    constexpr bool PRE = NV <= 16;
    f4 v[NV], w[PRE ? NV : 1];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const long base = 4 * t + 256 * u;
      if (base < n) v[u] = *(const f4*)(x + base);
    }
    if constexpr (PRE) {
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const long base = 4 * t + 256 * u;
        if (base < n) w[u] = *(const f4*)(wn + base);
      }
    }
    float ss = 0.0f, mn = 0x1p64f;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      if (4 * t + 256 * u < n) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ss = fmaf(v[u][q], v[u][q], ss);
          mn = fminf(mn, fabsf(v[u][q]));
        }
      }
    }
    const float nj = clampmin(sqrtf(bfly64(ss)));
    bool fast = __all(rcp_column_ok(mn, nj));
    if (!fast && nj <= RCP_NJ_MAX) fast = __all(min_nonzero_abs(v, n, t, 0) >= RCP_X_MIN);
    if (fast) {
      const float y = 1.0f / nj;
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const long base = 4 * t + 256 * u;
        if (base < n) {
          const f4 wu = PRE ? w[PRE ? u : 0] : *(const f4*)(wn + base);
#pragma unroll
          for (int q = 0; q < 4; ++q) p = fmaf(div_rcp(v[u][q], nj, y), wu[q], p);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const long base = 4 * t + 256 * u;
        if (base < n) {
          const f4 wu = PRE ? w[PRE ? u : 0] : *(const f4*)(wn + base);
#pragma unroll
          for (int q = 0; q < 4; ++q) p = fmaf(v[u][q] / nj, wu[q], p);
        }
      }
    }
  } else if ((n & 3) == 0 && (ldw & 3) == 0) {
    // float4 path (same per-lane element order {256u + 4t + q})
    float ss = 0.0f;
    for (long base = 4 * t; base < n; base += 256) {
      f4 v = *(const f4*)(x + base);
      ss = fmaf(v[0], v[0], ss);
      ss = fmaf(v[1], v[1], ss);
      ss = fmaf(v[2], v[2], ss);
      ss = fmaf(v[3], v[3], ss);
    }
    const float nj = clampmin(sqrtf(bfly64(ss)));
    for (long base = 4 * t; base < n; base += 256) {
      f4 v = *(const f4*)(x + base);
      f4 w = *(const f4*)(wn + base);
      p = fmaf(v[0] / nj, w[0], p);
      p = fmaf(v[1] / nj, w[1], p);
      p = fmaf(v[2] / nj, w[2], p);
      p = fmaf(v[3] / nj, w[3], p);
    }
  } else {
    float ss = bfly64(sumn_lane<true>(x, n, 1, t));
    const float nj = clampmin(sqrtf(ss));
    for (long base = 4 * t; base < n; base += 256) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        long i = base + q;
        if (i < n) p = fmaf(x[i] / nj, wn[i], p);
      }
    }
  }
  p = bfly64(p);
  if (t == 0) sim[e] = p;
}

// Columns of 4096 < n <= 16384 rows (n % 4 == 0): S = ceil(n / 4096) waves per column, wave s
// holding the float4s u in [16 s, 16 s + 16) of lane t (elements {256u + 4t + q}) in registers,
// so the whole column is loaded at once with 16 float4 per lane (~110 VGPRs: 4 waves per SIMD,
// where one wave holding all 48 needs 256 VGPRs and runs alone on its SIMD).  Each lane's chain
// continues across the waves in s order through LDS -- the per-lane order of ssr_sim_kernel<48>
// -- and wave S-1 folds it (bfly64): the same bits.
template <int S>
__global__ __launch_bounds__(64 * S) void ssr_sim_split_kernel(const float* Wt, long ldw, int n, const int* rem,
                                                               int r, const float* wn, float* sim, long zs) {
  __shared__ float part[64];
  __shared__ float njs;
  __shared__ bool okw[S];
  Wt = zws(Wt, zs);
  rem = zws(rem, zs);
  wn = zws(wn, zs);
  sim = zws(sim, zs);
  const int e = blockIdx.x;
  const int s = threadIdx.x >> 6, t = threadIdx.x & 63;
  const float* x = Wt + (long)rem[e] * ldw;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 v[16], w[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const long base = 4 * t + 256 * (16 * s + u);
    if (base < n) v[u] = *(const f4*)(x + base);
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const long base = 4 * t + 256 * (16 * s + u);
    if (base < n) w[u] = *(const f4*)(wn + base);
  }
  float ss = 0.0f, mn = 0x1p64f;
#pragma unroll
  for (int u = 0; u < 16; ++u)
    if (4 * t + 256 * (16 * s + u) < n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) mn = fminf(mn, fabsf(v[u][q]));
    }
  for (int q = 0; q < S; ++q) {
    if (s == q) {
      if (q > 0) ss = part[t];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (4 * t + 256 * (16 * s + u) < n) {
          ss = fmaf(v[u][0], v[u][0], ss);
          ss = fmaf(v[u][1], v[u][1], ss);
          ss = fmaf(v[u][2], v[u][2], ss);
          ss = fmaf(v[u][3], v[u][3], ss);
        }
      if (q < S - 1) part[t] = ss;
    }
    __syncthreads();
  }
  bool wave_ok = __all(mn >= RCP_X_MIN);
  if (!wave_ok) wave_ok = __all(min_nonzero_abs(v, n, t, 16 * s) >= RCP_X_MIN);
  if (t == 0) okw[s] = wave_ok;
  if (s == S - 1) {
    const float tot = bfly64(ss);
    if (t == 0) njs = clampmin(sqrtf(tot));
  }
  __syncthreads();
  const float nj = njs;
  bool fast = nj <= RCP_NJ_MAX;
  for (int q = 0; q < S; ++q) fast = fast && okw[q];  // workgroup-uniform
  // chain p = fma(x / nj, w, p) over this wave's elements, continued across the waves in order.
  float p = 0.0f;
  if (fast) {  // workgroup-uniform
    // the quotients in place first, every wave at once: only the chain is serial over the waves
    const float y = 1.0f / nj;
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = div_rcp(v[u][c], nj, y);
    for (int q = 0; q < S; ++q) {
      if (s == q) {
        if (q > 0) p = part[t];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (4 * t + 256 * (16 * s + u) < n) {
#pragma unroll
            for (int c = 0; c < 4; ++c) p = fmaf(v[u][c], w[u][c], p);
          }
        if (q < S - 1) part[t] = p;
      }
      __syncthreads();
    }
  } else {
    // the division (rare columns): a rolled loop re-reading the column and the mean (L2 hits),
    // so its register image stays small -- unrolled beside the fast path, the two need 200 VGPRs
    // (two waves per SIMD instead of three)
    for (int q = 0; q < S; ++q) {
      if (s == q) {
        if (q > 0) p = part[t];
#pragma unroll 1
        for (int u = 0; u < 16; ++u) {
          const long base = 4 * t + 256 * (16 * s + u);
          if (base < n) {
            const f4 xv = *(const f4*)(x + base), wv = *(const f4*)(wn + base);
#pragma unroll
            for (int c = 0; c < 4; ++c) p = fmaf(xv[c] / nj, wv[c], p);
          }
        }
        if (q < S - 1) part[t] = p;
      }
      __syncthreads();
    }
  }
  if (s == S - 1) {
    p = bfly64(p);
    if (t == 0) sim[e] = p;
  }
}

PT2Q_DEV uint32_t orderable(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// S1[j] = l-ascending sum of A[blk_j][blk_l], d = j-ascending sum of S1 (aga_s1 order) for
// b <= 128, by one workgroup: every gather load of a thread is in flight before the first LDS
// store; gb >= b*(b+1) floats of LDS, s1 >= b floats of LDS, bl = the b indices in LDS.
PT2Q_DEV void s1_block(const float* A, long lda, const int* bl, int b, float* gb, float* s1,
                       float* S1, float* d) {
  const int tid = threadIdx.x, nt = blockDim.x, ld = b + 1, tot = b * b;
  for (int q0 = 0; q0 < tot; q0 += 16 * nt) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + u * nt + tid, qq = q < tot ? q : 0;
      v[u] = A[(long)bl[qq / b] * lda + bl[qq % b]];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + u * nt + tid;
      if (q < tot) gb[(q / b) * ld + (q % b)] = v[u];
    }
  }
  __syncthreads();
  for (int j = tid; j < b; j += nt) {
    float sj = 0.0f;
    for (int l = 0; l < b; ++l) sj = sj + gb[j * ld + l];
    s1[j] = sj;
    S1[j] = sj;
  }
  __syncthreads();
  if (tid == 0) {
    float dd = 0.0f;
    for (int j = 0; j < b; ++j) dd = dd + s1[j];
    *d = dd;
  }
}

// Single-kernel S1 for the sequential / take-the-rest selections (b <= 128, raw Gram).
__global__ __launch_bounds__(1024) void s1_fused_kernel(const float* A, long lda, const int* blk,
                                                        int b, float* S1, float* d) {
  __shared__ float gb[128 * 129];
  __shared__ float s1[128];
  __shared__ int bl[128];
  for (int j = threadIdx.x; j < b; j += blockDim.x) bl[j] = blk ? blk[j] : j;
  __syncthreads();
  s1_block(A, lda, bl, b, gb, s1, S1, d);
}

PT2Q_DEV int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(v, off);
    if (lane >= off) v += y;
  }
  return v;
}

// Exclusive workgroup scan of v (blockDim.x <= 4096); sc >= 65 ints of LDS.  *total = sum.
PT2Q_DEV int block_excl_scan(int v, int* sc, int* total) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  const int incl = wave_incl_scan(v);
  if (lane == 63) sc[wv] = incl;
  __syncthreads();
  if (wv == 0) {
    const int x = lane < nw ? sc[lane] : 0;
    const int xi = wave_incl_scan(x);
    if (lane < nw) sc[lane] = xi - x;
    if (lane == 63) sc[64] = xi;
  }
  __syncthreads();
  const int r = sc[wv] + incl - v;
  *total = sc[64];
  __syncthreads();  // sc may be reused at once
  return r;
}

constexpr int TOPK_THREADS = 1024;
constexpr int TOPK_HPAD = 257;  // per-wave histogram stride (bank-spread)

// Ordered top-b of r similarities under the total order (value desc, position asc) -- the order
// torch.topk(sorted=True) gives here (reorder.py:133), keys being unique -- by radix selection:
// four 8-bit histogram passes over the orderable value bits find the b-th largest value v*;
// every value > v* is taken, plus the first (by position) b - #(> v*) values equal to v*; the
// b picks are then ranked among themselves.  Writes blk (selection order), newrem (ascending,
// reorder.py:139-141), perm_out (int64, nullable).  With G != nullptr (variant M, b <= 128)
// the same workgroup then forms S1/d for AGA from the raw Gram over the block it just selected.
// LDS: region0 (max(r + 32*257, b*(b+1)) words: values + two banks of wave histograms, later the S1 gather),
// r flag bytes, scan ints, b picks / their values / block indices / partial sums.
constexpr int S1_ROWS = TOPK_THREADS / 128;  // S1 rows per helper workgroup

// Helper workgroups 1.. of the top-k launch (variant M): wait for workgroup 0's pick, gather
// rows of G[blk][blk] in parallel and sum each in l order; the last one to finish forms d in j
// order (the s1_block order).  Workgroup 0 is dispatched first and waits on nobody, so the
// spin cannot deadlock.  sync[0]: pick published; sync[1]: helpers done.

PT2Q_DEV void s1_helper(const float* G, long ldg, const int* blk, int b, float* S1, float* d,
                        int* sync, float* gb, int* status, long cap) {
  const int tid = threadIdx.x, nh = gridDim.x - 1;
  // hand-offs (pick -> helpers, S1 -> the last helper): write-through (sc1) stores drained
  // before the flag / counter, sc1 loads on the consuming side, no fences
  if (tid == 0) wait_flag_ge<1>(&sync[0], 1, cap, status, STALL_TOPK);
  __syncthreads();
  PT2Q_TOPK_STAMP(8);
  const int jj = tid >> 7, l = tid & 127;
  const int j = (blockIdx.x - 1) * S1_ROWS + jj;
  if (j < b && l < b) {
    const int bj = __hip_atomic_load(&blk[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int bl = __hip_atomic_load(&blk[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gb[jj * 129 + l] = G[(long)bj * ldg + bl];
  }
  __syncthreads();
  if (l == 0 && j < b) {
    const float* row = gb + jj * 129;
    float s = 0.0f;
    int q = 0;
    for (; q + 8 <= b; q += 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = row[q + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) s = s + t[u];
    }
    for (; q < b; ++q) s = s + row[q];
    __hip_atomic_store(&S1[j], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  PT2Q_TOPK_STAMP(9);
  if (tid == 0) last = atomicAdd(&sync[1], 1) == nh - 1;
  __syncthreads();
  if (!last) return;
  if (tid < b) gb[tid] = __hip_atomic_load(&S1[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (tid == 0) {
    float dd = 0.0f;
    for (int q = 0; q < b; ++q) dd = dd + gb[q];
    *d = dd;
  }
}

__global__ __launch_bounds__(TOPK_THREADS) void ssr_topk_kernel(const float* sim, const int* rem, int r,
                                                                int b, int* blk, int* newrem,
                                                                int64_t* perm_out, const float* G,
                                                                long ldg, float* S1, float* d,
                                                                int region0, int* sync, int* status,
                                                                long cap, long zs) {
  extern __shared__ uint32_t vals[];
  sim = zws(sim, zs);  // grouped launch (no S1 helpers): linear blockIdx.z's slice
  rem = zws(rem, zs);
  blk = zws(blk, zs);
  newrem = zws(newrem, zs);
  perm_out = zws(perm_out, zs);
  if (blockIdx.x > 0) {
    s1_helper(G, ldg, blk, b, S1, d, sync, (float*)vals, status, cap);
    return;
  }
  int* hist = (int*)(vals + r);
  unsigned char* sel = (unsigned char*)(vals + region0);
  int* sc = (int*)(sel + ((r + 15) & ~15));
  int* pick = sc + 80;                  // b positions, ascending
  uint32_t* pv = (uint32_t*)(pick + b); // their values
  int* bl = (int*)(pv + b);             // b block indices (selection order)
  float* s1 = (float*)(bl + b);
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wv = tid >> 6;
  PT2Q_TOPK_STAMP(0);
  for (int e = tid; e < r; e += nt) vals[e] = orderable(sim[e]);
  uint32_t prefix = 0, pmask = 0;
  int kk = b;  // rank (1-based) of v* among the values matching prefix
  // Two banks of 16 per-wave histograms: a pass counts into one while clearing the other, and
  // wave 0 merges + scans in one go -- two barriers per pass.  res: the pass results, in two
  // alternating slots (read after the pass's second barrier, rewritten two passes later).
  for (int i = tid; i < 32 * TOPK_HPAD; i += nt) hist[i] = 0;
  __syncthreads();
  PT2Q_TOPK_STAMP(4);
  int* res = sc + 70;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    const int shift = 24 - 8 * p;
    int* hcur = hist + (p & 1) * 16 * TOPK_HPAD;
    int* hnext = hist + ((p + 1) & 1) * 16 * TOPK_HPAD;
    int* hw = hcur + wv * TOPK_HPAD;
    // similarities crowd into one bin in the high passes: a wave whose active lanes all share
    // a bin adds once (same-word LDS atomics of 64 lanes would serialise), others per lane
    for (int base = 0; base < r; base += nt) {
      const int e = base + tid;
      const uint32_t u = e < r ? vals[e] : 0u;
      const bool act = e < r && (u & pmask) == prefix;
      const int bin = (int)((u >> shift) & 255);
      const uint64_t am = __ballot(act);
      if (am) {
        const int leader = __ffsll((unsigned long long)am) - 1;
        const int lb = __shfl(bin, leader);
        const uint64_t same = __ballot(act && bin == lb);
        if (same == am) {
          if (lane == leader) atomicAdd(&hw[lb], __popcll(am));
        } else if (act) {
          atomicAdd(&hw[bin], 1);
        }
      }
    }
    if (p + 1 < 4)
      for (int i = tid; i < 16 * TOPK_HPAD; i += nt) hnext[i] = 0;
    __syncthreads();
    if (wv == 0) {  // lane l owns bins 255-4l .. 252-4l (descending)
      int c[4] = {0, 0, 0, 0}, s = 0;
#pragma unroll
      for (int w = 0; w < TOPK_THREADS / 64; ++w)
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] += hcur[w * TOPK_HPAD + 255 - 4 * lane - q];
#pragma unroll
      for (int q = 0; q < 4; ++q) s += c[q];
      const int incl = wave_incl_scan(s);
      int run = incl - s;
      if (run < kk && kk <= incl) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (run < kk && kk <= run + c[q]) {
            res[2 * (p & 1)] = 255 - 4 * lane - q;
            res[2 * (p & 1) + 1] = kk - run;
          }
          run += c[q];
        }
      }
    }
    __syncthreads();
    if (p == 0) PT2Q_TOPK_STAMP(5);
    prefix |= (uint32_t)res[2 * (p & 1)] << shift;
    pmask |= 255u << shift;
    kk = res[2 * (p & 1) + 1];
  }
  PT2Q_TOPK_STAMP(1);
  // prefix = v*; the first kk positions holding v* are picked, with every value above it
  const int per = (r + nt - 1) / nt;
  const int e0 = min(r, tid * per), e1 = min(r, e0 + per);
  int ceq = 0, tot;
  for (int e = e0; e < e1; ++e) ceq += vals[e] == prefix;
  int eq = block_excl_scan(ceq, sc, &tot);
  int cs = 0, cu = 0;
  for (int e = e0; e < e1; ++e) {
    const uint32_t u = vals[e];
    const bool s = u > prefix || (u == prefix && eq++ < kk);
    sel[e] = s;
    cs += s;
    cu += !s;
  }
  PT2Q_TOPK_STAMP(2);
  // one scan for both compactions (r < 2^16): picks and the unselected remainder, ascending
  const int both = block_excl_scan((cs << 16) | cu, sc, &tot);
  int os = both >> 16, ou = both & 0xFFFF;
  for (int e = e0; e < e1; ++e) {
    if (sel[e]) {
      pick[os] = e;
      pv[os++] = vals[e];
    } else {
      newrem[ou++] = rem[e];
    }
  }
  __syncthreads();
  PT2Q_TOPK_STAMP(3);
  // rank of pick t: picks above it in (value desc, position asc); picks are position-ascending.
  // Eight threads per pick, each over every eighth other pick, then summed across the eight.
  for (int t0 = 0; t0 < b; t0 += nt / 8) {
    const int t = t0 + tid / 8, sub = tid & 7;
    int rank = 0;
    if (t < b) {
      const uint32_t ut = pv[t];
      for (int s = sub; s < b; s += 8) {
        const uint32_t us = pv[s];
        rank += (us > ut) | ((us == ut) & (s < t));
      }
    }
    rank += __shfl_xor(rank, 4);
    rank += __shfl_xor(rank, 2);
    rank += __shfl_xor(rank, 1);
    if (t < b && sub == 0) {
      const int j = rem[pick[t]];
      __hip_atomic_store(&blk[rank], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: helpers read it
      if (perm_out) perm_out[rank] = j;
    }
  }
  (void)lane;
  (void)bl;
  (void)s1;
  PT2Q_TOPK_STAMP(6);
  if (G) {  // publish the pick to the S1 helpers (every storing wave drained first)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  PT2Q_TOPK_STAMP(7);
}

// Sequential block (use_ssr=False: main.py:167-169, gptq.py:135-137) or "take the rest"
// (reorder.py:125-126 when |rem| <= b).
__global__ void select_seq_kernel(int mode, int p0, int bs, int m, const int* rem, int* blk,
                                  int* newrem, int64_t* perm_out, long zs) {
  rem = zws(rem, zs);  // grouped launch: linear blockIdx.z's slice
  blk = zws(blk, zs);
  newrem = zws(newrem, zs);
  perm_out = zws(perm_out, zs);
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < bs) {
    int j = (mode == 0) ? p0 + t : rem[t];
    blk[t] = j;
    if (perm_out) perm_out[t] = j;
  }
  if (mode == 0) {
    int nr = m - p0 - bs;
    for (int e = t; e < nr; e += gridDim.x * blockDim.x) newrem[e] = p0 + bs + e;
  }
}

// S1 = S·1 and d = 1ᵀS1 for the AGA of one block.
//   src 1 (variant M): S[j][l] = A[blk_j][blk_l], A = raw Gram XᵀX (== X_bᵀX_b).
//   src 2 (variant G): S = Hbbᵀ Hbb with Hbb = A[blk][:,blk] (k-ascending fmaf chains).
// S1[j] = l-ascending sum; d = j-ascending sum (oracle s1_from_gram / s1_from_hess_block).
__global__ __launch_bounds__(256) void aga_s1_kernel(int src, const float* A, long lda,
                                                     const int* blk, int b, float* S1,
                                                     float* d) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x;
  float* s1 = sm;  // b
  if (src == 1 && b <= 128) {
    // gather the b x b sub-block cooperatively (independent loads), then row sums in order
    float* gb = sm + b;  // b x (b+1)
    int* idx = (int*)(gb + b * (b + 1));
    const int ld = b + 1;
    for (int j = tid; j < b; j += blockDim.x) idx[j] = blk ? blk[j] : j;
    __syncthreads();
    const int tot = b * b, step = blockDim.x;
    for (int q0 = 0; q0 < tot; q0 += 8 * step) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {  // 8 independent gathers in flight per thread
        int q = q0 + u * step + tid;
        int qq = q < tot ? q : 0;
        v[u] = A[(long)idx[qq / b] * lda + idx[qq % b]];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int q = q0 + u * step + tid;
        if (q < tot) gb[(q / b) * ld + (q % b)] = v[u];
      }
    }
    __syncthreads();
    for (int j = tid; j < b; j += blockDim.x) {
      float s = 0.0f;
      for (int l = 0; l < b; ++l) s = s + gb[j * ld + l];
      s1[j] = s;
    }
  } else if (src == 1) {
    int* idx = (int*)(sm + b);
    for (int j = tid; j < b; j += blockDim.x) idx[j] = blk ? blk[j] : j;
    __syncthreads();
    for (int j = tid; j < b; j += blockDim.x) {
      const float* row = A + (long)idx[j] * lda;
      float s = 0.0f;
      int l = 0;
      for (; l + 8 <= b; l += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = row[idx[l + u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) s = s + v[u];
      }
      for (; l < b; ++l) s = s + row[idx[l]];
      s1[j] = s;
    }
  } else {
    float* hb = sm + b;          // b x (b+1)
    float* S = hb + b * (b + 1); // b x (b+1)
    const int ld = b + 1;
    for (int q = tid; q < b * b; q += blockDim.x) {
      int t = q / b, j = q % b;
      hb[t * ld + j] = A[(long)(blk ? blk[t] : t) * lda + (blk ? blk[j] : j)];
    }
    __syncthreads();
    for (int q = tid; q < b * b; q += blockDim.x) {
      int j = q / b, l = q % b;
      float acc = 0.0f;
      for (int t = 0; t < b; ++t) acc = fmaf(hb[t * ld + j], hb[t * ld + l], acc);
      S[j * ld + l] = acc;
    }
    __syncthreads();
    for (int j = tid; j < b; j += blockDim.x) {
      float s = 0.0f;
      for (int l = 0; l < b; ++l) s = s + S[j * ld + l];
      s1[j] = s;
    }
  }
  __syncthreads();
  for (int j = tid; j < b; j += blockDim.x) S1[j] = s1[j];
  if (tid == 0) {
    float dd = 0.0f;
    for (int j = 0; j < b; ++j) dd = dd + s1[j];
    *d = dd;
  }
}

// Wide blocks (b > 512, per-channel): S1[j] = sequential row sum of A[blk_j][blk_l] over l (the
// same order as aga_s1_kernel).  A workgroup owns S1W_ROWS rows j: all 256 threads stage a
// S1W_ROWS x S1W_COLS tile of them (coalesced along l) into one of two LDS buffers while lanes
// 0..S1W_ROWS-1 of wave 0 run their rows' serial chains over the other buffer, so the chains never
// wait on a global load and every load instruction reads whole rows segments (one thread per j
// striding over whole rows read 64 rows per instruction and ran 3.3 ms at b = 13824).
constexpr int S1W_ROWS = 32, S1W_COLS = 256;
__global__ __launch_bounds__(256) void s1_rows_kernel(const float* A, long lda, const int* blk,
                                                      int b, float* S1, long sA, long sS) {
  __shared__ float tile[2][S1W_ROWS][S1W_COLS + 1];
  A += blockIdx.y * sA;  // batched: item blockIdx.y (strides 0 for one item)
  S1 += blockIdx.y * sS;
  const int tid = threadIdx.x, j0 = blockIdx.x * S1W_ROWS;
  const int nj = min(S1W_ROWS, b - j0);
  auto stage = [&](int c, int buf) {  // columns [c, c + S1W_COLS) of the workgroup's rows
    const int l = c + tid;
    const int bl = l < b ? (blk ? blk[l] : l) : 0;
    float v[S1W_ROWS];
#pragma unroll
    for (int r = 0; r < S1W_ROWS; ++r) {
      const int j = j0 + (r < nj ? r : 0);
      v[r] = A[(long)(blk ? blk[j] : j) * lda + bl];
    }
#pragma unroll
    for (int r = 0; r < S1W_ROWS; ++r) tile[buf][r][tid] = v[r];
  };
  float s = 0.0f;
  stage(0, 0);
  __syncthreads();
  int buf = 0;
  for (int c = 0; c < b; c += S1W_COLS) {
    if (c + S1W_COLS < b) stage(c + S1W_COLS, buf ^ 1);
    if (tid < nj) {
      const int len = min(S1W_COLS, b - c);
      const float* row = tile[buf][tid];
      int l = 0;
      for (; l + 8 <= len; l += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = row[l + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) s = s + t[u];
      }
      for (; l < len; ++l) s = s + row[l];
    }
    __syncthreads();
    buf ^= 1;
  }
  if (tid < nj) S1[j0 + tid] = s;
}

// Blocks up to 512 columns: one workgroup per row j gathers A[blk_j][blk_l] (all loads in
// flight at once), then one lane sums them in l order (the aga_s1_kernel order).
__global__ __launch_bounds__(128) void s1_row_wg_kernel(const float* A, long lda, const int* blk,
                                                        int b, float* S1, long sA, long sS) {
  __shared__ float v[512];
  A += blockIdx.y * sA;
  S1 += blockIdx.y * sS;
  const int j = blockIdx.x;
  const float* row = A + (long)(blk ? blk[j] : j) * lda;
  for (int l = threadIdx.x; l < b; l += 128) v[l] = row[blk ? blk[l] : l];
  __syncthreads();
  if (threadIdx.x != 0) return;
  float s = 0.0f;
  int l = 0;
  for (; l + 8 <= b; l += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = v[l + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + t[u];
  }
  for (; l < b; ++l) s = s + v[l];
  S1[j] = s;
}

// S1 of whole wide Grams (the batched per-channel S1 / d, m > 512; m % 4 == 0, 16-byte aligned
// rows): the same sequential row chains as s1_rows_kernel, fed by a wave-private LDS-DMA ring.
// s1_rows_kernel staged each tile by register loads whose LDS stores waited for them before the
// chains ran, one tile in flight per workgroup: ~3.5 TB/s, and a shard's few Grams could not
// hide the round trips (1.8 ms for the S1 phase of one rank's C5 shard).  Here a one-wave
// workgroup owns 64 rows (lane l: row r0 + l's chain) and DMAs them 32 columns per tile (8 KiB,
// 8 x 1 KiB global_load_lds_dwordx4) into an S1R_STAGES-deep LDS ring, S1R_STAGES - 1 tiles ahead,
// with no barrier.  32 KiB per workgroup: five share a CU, so a shard's 1,080 row groups of its
// m = 13824 Grams are resident at once (256-row workgroups left a second round of 14 on a few CUs,
// doubling the launch).  LDS layout: row rr at 128 rr bytes,
// its 16-byte chunk k at slot k ^ ((rr >> 1) & 7) -- the DMA lanes load the permuted chunks, so
// the chain lanes' ds_read_b128 of one chunk index hit 16 distinct bank groups per 16 lanes.
constexpr int S1R_COLS = 32, S1R_STAGES = 4, S1R_WROWS = 64;
constexpr int S1R_WSTAGE = S1R_WROWS * S1R_COLS * 4;  // 8 KiB per wave and stage

typedef float s1f4 __attribute__((ext_vector_type(4)));

template <int N>
PT2Q_DEV void s1r_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
PT2Q_DEV void s1r_vmcnt(int younger) {  // tiles still in flight after the one to read (x 8 DMAs)
  switch (younger) {
    case 0: s1r_vm<0>(); break;
    case 1: s1r_vm<8>(); break;
    case 2: s1r_vm<16>(); break;
    case 3: s1r_vm<24>(); break;
    default: s1r_vm<32>(); break;
  }
}

__global__ __launch_bounds__(64) void s1_ring_kernel(const float* G, long ldg, int m, float* S1, long sG, long sS) {
  __shared__ __attribute__((aligned(1024))) uint8_t ring[S1R_STAGES * S1R_WSTAGE];
  typedef __attribute__((address_space(3))) void* lptr;
  const int lane = threadIdx.x & 63;
  G += blockIdx.y * sG;
  S1 += blockIdx.y * sS;
  const int r0 = blockIdx.x * S1R_WROWS;
  uint8_t* wring = ring;
  const uint32_t wlds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)wring;
  const int ntile = (m + S1R_COLS - 1) / S1R_COLS;
  // this lane's DMA source in each of a tile's 8 instructions: row rr = 8 q + lane / 8, chunk
  // k = (lane % 8) ^ ((rr >> 1) & 7) -- rows past m read row 0 (results dropped)
  const float* src[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int rr = 8 * q + (lane >> 3);
    const int row = r0 + rr < m ? r0 + rr : 0;
    src[q] = G + (long)row * ldg + 4 * ((lane & 7) ^ ((rr >> 1) & 7));
  }
  auto issue = [&](int t) {
    uint8_t* stg = wring + (t % S1R_STAGES) * S1R_WSTAGE;
    const int c0 = t * S1R_COLS;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      // chunks past m (only in the last tile; m % 4 == 0) read column 0 and are masked below
      const int col = c0 + 4 * ((lane & 7) ^ (((8 * q + (lane >> 3)) >> 1) & 7));
      __builtin_amdgcn_global_load_lds(col < m ? src[q] + c0 : src[q] - 4 * ((lane & 7) ^ (((8 * q + (lane >> 3)) >> 1) & 7)),
                                       (lptr)(stg + q * 1024), 16, 0, 0);
    }
  };
  const int pre = ntile < S1R_STAGES - 1 ? ntile : S1R_STAGES - 1;
  for (int t = 0; t < pre; ++t) issue(t);
  const int f = (lane >> 1) & 7;
  float s = 0.0f;
  for (int t = 0; t < ntile; ++t) {
    if (t + S1R_STAGES - 1 < ntile) issue(t + S1R_STAGES - 1);
    const int ahead = ntile - 1 - t;  // tiles issued after tile t
    s1r_vmcnt(ahead < S1R_STAGES - 1 ? ahead : S1R_STAGES - 1);
    const uint32_t base = wlds + (t % S1R_STAGES) * S1R_WSTAGE + lane * 128;
    s1f4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      asm volatile("ds_read_b128 %0, %1" : "=v"(x[k]) : "v"(base + ((k ^ f) << 4)));
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                 :: "memory");
    if ((t + 1) * S1R_COLS <= m) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) s = s + x[k][u];
    } else {  // the last, partial tile: only the columns < m (whole chunks)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (t * S1R_COLS + 4 * k < m)
#pragma unroll
          for (int u = 0; u < 4; ++u) s = s + x[k][u];
    }
  }
  if (r0 + lane < m) S1[r0 + lane] = s;
}

// S1 of UPPER-only Grams (G[r][c] stored for c >= r only: pt2q_gram_batched_upper): row j's chain
// takes G[l][j] for l < j and G[j][l] for l >= j, l ascending -- on a Gram whose mirror is an
// exact copy these are s1_ring_kernel's values in s1_ring_kernel's order, so S1 is bit-identical.
// A one-wave workgroup owns rows j0 .. j0 + 63 (lane: row j = j0 + lane) and streams 8 KiB tiles
// through the same four-stage LDS-DMA ring:
//  * column tiles t < nA = j0 / 32: G rows l = 32 t .. 32 t + 31, columns j0 .. j0 + 63 (natural
//    layout, 256 B per row; 16 lanes x 16 B per row in a DMA): lane j reads its column, l < j;
//  * row tiles u = t - nA: rows j0 .. j0 + 63, columns j0 + 32 u .. + 31 (s1_ring_kernel's
//    swizzled layout): lane j reads its own row, l >= j -- except in the two diagonal tiles
//    (u = 0, 1), where l < j reads element (l, j) of the tile holding column j (both resident).
__global__ __launch_bounds__(64) void s1_upper_ring_kernel(const float* G, long ldg, int m, float* S1, long sG,
                                                           long sS) {
  __shared__ __attribute__((aligned(1024))) uint8_t ring[S1R_STAGES * S1R_WSTAGE];
  typedef __attribute__((address_space(3))) void* lptr;
  const int lane = threadIdx.x & 63;
  G += blockIdx.y * sG;
  S1 += blockIdx.y * sS;
  const int j0 = blockIdx.x * S1R_WROWS;
  const int j = j0 + lane;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)ring;
  const int nA = j0 / S1R_COLS, nC = (m - j0 + S1R_COLS - 1) / S1R_COLS, ntile = nA + nC;
  auto issue = [&](int t) {
    uint8_t* stg = ring + (t % S1R_STAGES) * S1R_WSTAGE;
    if (t < nA) {  // rows 32 t + 4 q + lane / 16, 16-byte chunk lane % 16 of columns j0 ..
      const int col = j0 + 4 * (lane & 15);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int row = S1R_COLS * t + 4 * q + (lane >> 4);
        __builtin_amdgcn_global_load_lds(G + (long)row * ldg + (col < m ? col : 0), (lptr)(stg + q * 1024), 16, 0, 0);
      }
    } else {  // s1_ring_kernel's row tile at columns c0
      const int c0 = j0 + S1R_COLS * (t - nA);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int rr = 8 * q + (lane >> 3);
        const int row = j0 + rr < m ? j0 + rr : 0;
        const int col = c0 + 4 * ((lane & 7) ^ ((rr >> 1) & 7));
        __builtin_amdgcn_global_load_lds(G + (long)row * ldg + (col < m ? col : 0), (lptr)(stg + q * 1024), 16, 0,
                                         0);
      }
    }
  };
  const int pre = ntile < S1R_STAGES - 1 ? ntile : S1R_STAGES - 1;
  for (int t = 0; t < pre; ++t) issue(t);
  const int f = (lane >> 1) & 7;
  float s = 0.0f;
  for (int t = 0; t < ntile; ++t) {
    if (t + S1R_STAGES - 1 < ntile) issue(t + S1R_STAGES - 1);
    // this tile landed -- and at the first diagonal tile the second one too
    const int need = (t == nA && nC > 1) ? t + 1 : t;
    const int ahead = ntile - 1 - need;
    s1r_vmcnt(ahead < S1R_STAGES - 1 - (need - t) ? ahead : S1R_STAGES - 1 - (need - t));
    const uint32_t st0 = lds0 + (t % S1R_STAGES) * S1R_WSTAGE;
    if (t < nA) {  // column tile: l = 32 t + r < j0 <= j
      float x[S1R_COLS];
#pragma unroll
      for (int r = 0; r < S1R_COLS; ++r)
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(x[r]) : "v"(st0 + 4 * lane), "i"(256 * r));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < S1R_COLS; ++r) s = s + x[r];
      continue;
    }
    const int u = t - nA;
    const int c0 = j0 + S1R_COLS * u;
    if (u >= 2) {  // own row only (l >= j0 + 64 > j)
      s1f4 x[8];
      const uint32_t base = st0 + lane * 128;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        asm volatile("ds_read_b128 %0, %1" : "=v"(x[k]) : "v"(base + ((k ^ f) << 4)));
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                   :: "memory");
      if (c0 + S1R_COLS <= m) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int q = 0; q < 4; ++q) s = s + x[k][q];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (c0 + 4 * k < m)
#pragma unroll
            for (int q = 0; q < 4; ++q) s = s + x[k][q];
      }
      continue;
    }
    // diagonal tile u (l = c0 + c): l < j -> element (l, j) of the tile holding column j; else
    // element (j, l) of this tile (own row)
    const int uj = lane >> 5, cj = lane & 31;  // column j's tile (0 / 1) and column in it
    const uint32_t colj = lds0 + ((nA + uj) % S1R_STAGES) * S1R_WSTAGE + (uint32_t)((cj & 3) << 2);
    float x[S1R_COLS];
#pragma unroll
    for (int c = 0; c < S1R_COLS; ++c) {
      const int l = c0 + c, rr = l - j0;  // row of the diagonal block
      const uint32_t a_col = colj + rr * 128 + ((((cj >> 2) ^ ((rr >> 1) & 7))) << 4);
      const uint32_t a_row = st0 + lane * 128 + ((((c >> 2) ^ f)) << 4) + ((c & 3) << 2);
      asm volatile("ds_read_b32 %0, %1" : "=v"(x[c]) : "v"(l < j ? a_col : a_row));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < S1R_COLS; ++c)
      if (c0 + c < m) s = s + x[c];
  }
  if (j < m) S1[j] = s;
}

// d = sequential sum of S1 (j ascending); S1 is staged through LDS in chunks so the serial
// chain never waits on a global load.
__global__ __launch_bounds__(256) void s1_total_kernel(const float* S1, int b, float* d, long sS, long sD) {
  __shared__ float v[4096];
  S1 += blockIdx.x * sS;  // batched: item blockIdx.x (strides 0 for one item)
  d += blockIdx.x * sD;
  float dd = 0.0f;
  for (int j0 = 0; j0 < b; j0 += 4096) {
    const int len = min(4096, b - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < len; j += 256) v[j] = S1[j0 + j];
    __syncthreads();
    if (threadIdx.x == 0) {
      // the next 16 values are read while the current 16 are added (the chain never waits on LDS)
      int j = 0;
      if (len >= 16) {
        float t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) t[u] = v[u];
        for (; j + 32 <= len; j += 16) {
          float nx[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) nx[u] = v[j + 16 + u];
#pragma unroll
          for (int u = 0; u < 16; ++u) dd = dd + t[u];
#pragma unroll
          for (int u = 0; u < 16; ++u) t[u] = nx[u];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) dd = dd + t[u];
        j += 16;
      }
      for (; j < len; ++j) dd = dd + v[j];
    }
  }
  if (threadIdx.x == 0) *d = dd;
}

// C[k][e] = Hinv[blk_k][rem_e] / clamp(Hinv[blk_k][blk_k])   (main.py:201-209)
__global__ __launch_bounds__(256) void ef_coeff_kernel(const float* Hinv, long ldh,
                                                       const int* blk, const int* rem, int nr,
                                                       float* C, long ldc) {
  const int k = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= nr) return;
  const long rowb = (long)blk[k] * ldh;
  const float dg = clampmin(Hinv[rowb + blk[k]]);
  C[(long)k * ldc + e] = Hinv[rowb + rem[e]] / dg;
}

}  // namespace

size_t pt2q_ssr_scratch_floats(int n, int m) {
  // part (ceil(m/128) x n) + wn (n) + sim (m)
  return (size_t)ceil_div(m, CHUNK) * n + (size_t)n + (size_t)m;
}

int pt2q_launch_ssr_similarity(const float* Wt, long ldw, int n, const int* rem, int r,
                               float* part, float* wn, float* sim, hipStream_t st, int* cnt,
                               const Grp* grp, bool pre) {
  if (r <= 0 || n <= 0) return PT2Q_E_ARG;
  if ((size_t)(n + 1) * sizeof(float) > 160 * 1024) return PT2Q_E_UNSUPPORTED;
  int nchunks = ceil_div(r, CHUNK);
  const unsigned nz = grp_z(grp);
  const long zs = grp ? grp->ws : 0;
  const bool fused = cnt && n <= 16384 && n % 4 == 0 && ldw % 4 == 0 && (uintptr_t)Wt % 16 == 0 &&
                     pt2q_tuning().wbar_fused;
  if ((nz > 1 || pre) && !fused) return PT2Q_E_UNSUPPORTED;  // grouped launches use the fused w-bar only
  if (fused) {
    hipLaunchKernelGGL(ssr_wbar_fused_kernel, dim3(pre ? 1 : nchunks, ceil_div(n, 256), nz), dim3(64), 0, st, Wt,
                       ldw, n, rem, r, part, wn, cnt, zs, pre ? 1 : 0);
    PT2Q_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(ssr_wbar_partial_kernel, dim3(nchunks, ceil_div(n, 256)), dim3(256), 0, st,
                       Wt, ldw, n, rem, r, part);
    PT2Q_LAUNCH_CHECK();
    if (n <= SUMN_LDS_MAX) {
      hipLaunchKernelGGL(ssr_wbar_sumfinal_kernel, dim3(1), dim3(1024), 0, st, part, nchunks, n, r, wn);
      PT2Q_LAUNCH_CHECK();
    } else {
      hipLaunchKernelGGL(ssr_wbar_sum_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, part, nchunks,
                         n, r, wn);
      PT2Q_LAUNCH_CHECK();
      hipLaunchKernelGGL(ssr_wbar_final_kernel, dim3(1), dim3(1024), 0, st, wn, n);
      PT2Q_LAUNCH_CHECK();
    }
  }
  const bool v4 = (n & 3) == 0 && (ldw & 3) == 0 && (uintptr_t)Wt % 16 == 0;
  const int S = ceil_div(n, 4096);
  if (v4 && n > 4096 && n <= 16384 && pt2q_tuning().sim_split) {
    auto k = S == 2 ? ssr_sim_split_kernel<2> : S == 3 ? ssr_sim_split_kernel<3> : ssr_sim_split_kernel<4>;
    hipLaunchKernelGGL(k, dim3(r, 1, nz), dim3(64 * S), 0, st, Wt, ldw, n, rem, r, wn, sim, zs);
  } else {
    auto sim_k = !v4 ? ssr_sim_kernel<0> : n <= 4096 ? ssr_sim_kernel<16> : n <= 12288 ? ssr_sim_kernel<48>
                                                                                     : ssr_sim_kernel<0>;
    hipLaunchKernelGGL(sim_k, dim3(ceil_div(r, 4), 1, nz), dim3(256), 0, st, Wt, ldw, n, rem, r, wn, sim, zs);
  }
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_ssr_topk(const float* sim, const int* rem, int r, int b, int* blk, int* newrem,
                         int64_t* perm_out, hipStream_t st, const float* G, long ldg, float* S1,
                         float* d, int* sync, int* status, const Grp* grp) {
  if (G && b > 128) return PT2Q_E_ARG;
  const unsigned nz = grp_z(grp);
  if (nz > 1 && G) return PT2Q_E_UNSUPPORTED;  // grouped: S1/d are formed in the ATQ launch
  if (b <= 0 || b > r || r >= 65536) return PT2Q_E_UNSUPPORTED;
  if (G && !sync) return PT2Q_E_ARG;  // sync: 2 ints the caller zeroed before this launch
  const int region0 = (r + 32 * TOPK_HPAD + 3) & ~3;  // >= S1_ROWS * 129 for the helpers
  const size_t lds = (size_t)region0 * 4 + (size_t)((r + 15) & ~15) + 80 * sizeof(int) +
                     (size_t)b * 4 * sizeof(int);
  if (lds > 160 * 1024) return PT2Q_E_UNSUPPORTED;
  const int grid = G ? 1 + ceil_div(b, S1_ROWS) : 1;
  hipLaunchKernelGGL(ssr_topk_kernel, dim3(grid, 1, nz), dim3(TOPK_THREADS), lds, st, sim, rem, r, b, blk,
                     newrem, perm_out, G, ldg, S1, d, region0, sync, status,
                     pt2q_tuning().spin_cap_short, grp ? grp->ws : 0l);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_select_seq(int mode, int p0, int bs, int m, const int* rem, int* blk,
                           int* newrem, int64_t* perm_out, hipStream_t st, const Grp* grp) {
  int work = (mode == 0) ? (m - p0) : bs;
  int grid = ceil_div(work > 0 ? work : 1, 256);
  if (grid > 64) grid = 64;
  hipLaunchKernelGGL(select_seq_kernel, dim3(grid, 1, grp_z(grp)), dim3(256), 0, st, mode, p0, bs, m, rem,
                     blk, newrem, perm_out, grp ? grp->ws : 0l);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_aga_s1(int src, const float* A, long lda, const int* blk, int b, float* S1,
                       float* d, hipStream_t st) {
  if (src == 1 && b <= 128) {
    hipLaunchKernelGGL(s1_fused_kernel, dim3(1), dim3(1024), 0, st, A, lda, blk, b, S1, d);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  if (src == 1) {
    if (b > 512)
      hipLaunchKernelGGL(s1_rows_kernel, dim3(ceil_div(b, S1W_ROWS)), dim3(256), 0, st, A, lda, blk, b, S1, 0l, 0l);
    else
      hipLaunchKernelGGL(s1_row_wg_kernel, dim3(b), dim3(128), 0, st, A, lda, blk, b, S1, 0l, 0l);
    PT2Q_LAUNCH_CHECK();
    hipLaunchKernelGGL(s1_total_kernel, dim3(1), dim3(256), 0, st, S1, b, d, 0l, 0l);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  size_t lds = (size_t)b * sizeof(float);
  if (src == 2) lds += 2 * (size_t)b * (b + 1) * sizeof(float);
  else if (b <= 128) lds += (size_t)b * (b + 1) * sizeof(float) + (size_t)b * sizeof(int);
  else lds += (size_t)b * sizeof(int);
  if (lds > 160 * 1024) return PT2Q_E_UNSUPPORTED;
  hipLaunchKernelGGL(aga_s1_kernel, dim3(1), dim3(256), lds, st, src, A, lda, blk, b, S1, d);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

// S1 = S·1, d = 1ᵀS1 of `batch` whole m x m raw Grams (item z at G + z * sG) in one launch pair:
// S1d[z * (m + 1) + j] = S1[j] of item z, S1d[z * (m + 1) + m] = its d.  Same kernels and order as
// pt2q_launch_aga_s1 (src 1, no block indices), so every value is bit-identical to the per-item
// call; the batch fills the chip where one item's serial d chain ran on one workgroup.
int pt2q_launch_s1_batched(const float* G, long ldg, int m, int batch, long sG, float* S1d, hipStream_t st,
                           bool upper) {
  if (upper) {  // upper-only Grams: the ring kernel's DMA conditions are required
    if (m <= 512 || m % 4 || ldg % 4 || sG % 4 || ((uintptr_t)G & 15)) return PT2Q_E_UNSUPPORTED;
    const long sS = m + 1;
    hipLaunchKernelGGL(s1_upper_ring_kernel, dim3(ceil_div(m, S1R_WROWS), batch), dim3(64), 0, st, G, ldg, m, S1d,
                       sG, sS);
    PT2Q_LAUNCH_CHECK();
    hipLaunchKernelGGL(s1_total_kernel, dim3(batch), dim3(256), 0, st, S1d, m, S1d + m, sS, sS);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  if (m <= 128) {
    for (int z = 0; z < batch; ++z) {
      const int rc = pt2q_launch_aga_s1(1, G + z * sG, ldg, nullptr, m, S1d + (long)z * (m + 1),
                                        S1d + (long)z * (m + 1) + m, st);
      if (rc != PT2Q_OK) return rc;
    }
    return PT2Q_OK;
  }
  const long sS = m + 1;
  const bool ring = m % 4 == 0 && ldg % 4 == 0 && sG % 4 == 0 && ((uintptr_t)G & 15) == 0;
  if (m > 512 && ring)
    hipLaunchKernelGGL(s1_ring_kernel, dim3(ceil_div(m, S1R_WROWS), batch), dim3(64), 0, st, G, ldg, m, S1d, sG, sS);
  else if (m > 512)
    hipLaunchKernelGGL(s1_rows_kernel, dim3(ceil_div(m, S1W_ROWS), batch), dim3(256), 0, st, G, ldg, nullptr, m,
                       S1d, sG, sS);
  else
    hipLaunchKernelGGL(s1_row_wg_kernel, dim3(m, batch), dim3(128), 0, st, G, ldg, nullptr, m, S1d, sG, sS);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(s1_total_kernel, dim3(batch), dim3(256), 0, st, S1d, m, S1d + m, sS, sS);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_ef_coeffs(const float* Hinv, long ldh, const int* blk, int bs, const int* rem,
                          int nr, float* C, long ldc, hipStream_t st) {
  hipLaunchKernelGGL(ef_coeff_kernel, dim3(ceil_div(nr, 256), bs), dim3(256), 0, st, Hinv, ldh,
                     blk, rem, nr, C, ldc);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}
