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

namespace {

constexpr int CHUNK = 128;  // canonical wbar chunk (rem entries per partial sum)

// part[c][i] = sum over rem[c*128 .. c*128+127] (ascending) of Wt[rem[e]][i]
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
  float p = 0.0f;
  int e = 0;
  for (; e + 8 <= cnt; e += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = Wt[rows[e + u] + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) p = p + v[u];
  }
  for (; e < cnt; ++e) p = p + Wt[rows[e] + i];
  part[(long)c * n + i] = p;
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

// One wave per remaining column: nj = clamp(sqrt(SUMN fma x^2)); s = SUMN fma (x/nj) * wn.
__global__ __launch_bounds__(256) void ssr_sim_kernel(const float* Wt, long ldw, int n,
                                                      const int* rem, int r, const float* wn,
                                                      float* sim) {
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int t = threadIdx.x & 63;
  if (e >= r) return;
  const float* x = Wt + (long)rem[e] * ldw;
  float p = 0.0f;
  if ((n & 3) == 0 && (ldw & 3) == 0) {
    // float4 path (same per-lane element order {256u + 4t + q})
    typedef float f4 __attribute__((ext_vector_type(4)));
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

// Ordered top-b of r similarities: keys (value desc, position asc), bitonic sort in LDS.
// Writes blk (selection order), newrem (ascending), perm_out (int64, nullable).
// With G != nullptr (variant M, b <= 128) the same workgroup then forms S1/d for AGA from the
// raw Gram over the block it just selected (one launch instead of three).
__global__ __launch_bounds__(1024) void ssr_topk_kernel(const float* sim, const int* rem, int r,
                                                        int b, int P, int* blk, int* newrem,
                                                        int64_t* perm_out, const float* G,
                                                        long ldg, float* S1, float* d,
                                                        int keys_floats) {
  // LDS: keys region (P keys; reused for the S1 gather), r flag bytes, scan ints, b indices,
  // b partial sums
  extern __shared__ unsigned long long keys[];
  unsigned char* sel = (unsigned char*)((float*)keys + keys_floats);
  int* scan = (int*)(sel + ((r + 15) & ~15));
  int* bl = scan + 1024;
  float* s1 = (float*)(bl + 128);
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < P; e += nt)
    keys[e] = (e < r) ? (((unsigned long long)orderable(sim[e]) << 32) |
                         (unsigned long long)(0xFFFFFFFFu - (uint32_t)e))
                      : 0ull;
  for (int e = tid; e < r; e += nt) sel[e] = 0;
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int idx = tid; idx < P / 2; idx += nt) {
        int lo = 2 * idx - (idx & (stride - 1));
        int hi = lo + stride;
        bool desc = ((lo & size) == 0);
        unsigned long long a = keys[lo], c = keys[hi];
        if ((a < c) == desc) {
          keys[lo] = c;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int t = tid; t < b; t += nt) {
    int e = (int)(0xFFFFFFFFu - (uint32_t)(keys[t] & 0xFFFFFFFFull));
    int j = rem[e];
    blk[t] = j;
    if (G) bl[t] = j;
    if (perm_out) perm_out[t] = j;
    sel[e] = 1;
  }
  __syncthreads();
  if (G) s1_block(G, ldg, bl, b, (float*)keys, s1, S1, d);  // keys are dead after the pick
  // stable compaction of the unselected positions (ascending)
  const int per = (r + nt - 1) / nt;
  const int e0 = min(r, tid * per), e1 = min(r, e0 + per);
  int cnt = 0;
  for (int e = e0; e < e1; ++e) cnt += !sel[e];
  // block exclusive scan of cnt: wave-inclusive scan by shuffles, then wave totals
  const int lane = tid & 63, wv = tid >> 6;
  int incl = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  if (lane == 63) scan[wv] = incl;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int q = 0; q < (nt >> 6); ++q) {
      int v = scan[q];
      scan[q] = acc;
      acc += v;
    }
  }
  __syncthreads();
  int o = scan[wv] + incl - cnt;
  for (int e = e0; e < e1; ++e)
    if (!sel[e]) newrem[o++] = rem[e];
}

// Sequential block (use_ssr=False: main.py:167-169, gptq.py:135-137) or "take the rest"
// (reorder.py:125-126 when |rem| <= b).
__global__ void select_seq_kernel(int mode, int p0, int bs, int m, const int* rem, int* blk,
                                  int* newrem, int64_t* perm_out) {
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

// Wide blocks (b > 512, per-channel): S1[j] = sequential row sum of A[blk_j][blk_l] over l, one
// thread per j across many workgroups (the same order as aga_s1_kernel), then d in order.
__global__ __launch_bounds__(256) void s1_rows_kernel(const float* A, long lda, const int* blk,
                                                      int b, float* S1) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= b) return;
  const float* row = A + (long)(blk ? blk[j] : j) * lda;
  float s = 0.0f;
  int l = 0;
  for (; l + 8 <= b; l += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = row[blk ? blk[l + u] : l + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + v[u];
  }
  for (; l < b; ++l) s = s + row[blk ? blk[l] : l];
  S1[j] = s;
}

// Blocks up to 512 columns: one workgroup per row j gathers A[blk_j][blk_l] (all loads in
// flight at once), then one lane sums them in l order (the aga_s1_kernel order).
__global__ __launch_bounds__(128) void s1_row_wg_kernel(const float* A, long lda, const int* blk,
                                                        int b, float* S1) {
  __shared__ float v[512];
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

// d = sequential sum of S1 (j ascending); S1 is staged through LDS in chunks so the serial
// chain never waits on a global load.
__global__ __launch_bounds__(256) void s1_total_kernel(const float* S1, int b, float* d) {
  __shared__ float v[4096];
  float dd = 0.0f;
  for (int j0 = 0; j0 < b; j0 += 4096) {
    const int len = min(4096, b - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < len; j += 256) v[j] = S1[j0 + j];
    __syncthreads();
    if (threadIdx.x == 0) {
      int j = 0;
      for (; j + 8 <= len; j += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = v[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) dd = dd + t[u];
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
                               float* part, float* wn, float* sim, hipStream_t st) {
  if (r <= 0 || n <= 0) return PT2Q_E_ARG;
  if ((size_t)(n + 1) * sizeof(float) > 160 * 1024) return PT2Q_E_UNSUPPORTED;
  int nchunks = ceil_div(r, CHUNK);
  hipLaunchKernelGGL(ssr_wbar_partial_kernel, dim3(nchunks, ceil_div(n, 256)), dim3(256), 0, st,
                     Wt, ldw, n, rem, r, part);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(ssr_wbar_sum_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, part, nchunks,
                     n, r, wn);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(ssr_wbar_final_kernel, dim3(1), dim3(1024), 0, st, wn, n);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(ssr_sim_kernel, dim3(ceil_div(r, 4)), dim3(256), 0, st, Wt, ldw, n, rem, r,
                     wn, sim);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_ssr_topk(const float* sim, const int* rem, int r, int b, int* blk, int* newrem,
                         int64_t* perm_out, hipStream_t st, const float* G, long ldg, float* S1,
                         float* d) {
  int P = 1;
  while (P < r) P <<= 1;
  if (G && b > 128) return PT2Q_E_ARG;
  int keys_floats = 2 * P;
  if (G && keys_floats < b * (b + 1)) keys_floats = b * (b + 1);
  keys_floats = (keys_floats + 3) & ~3;
  size_t lds = (size_t)keys_floats * 4 + (size_t)((r + 15) & ~15) + 1024 * sizeof(int) +
               128 * sizeof(int) + 128 * sizeof(float);
  if (lds > 160 * 1024) return PT2Q_E_UNSUPPORTED;
  hipLaunchKernelGGL(ssr_topk_kernel, dim3(1), dim3(1024), lds, st, sim, rem, r, b, P, blk,
                     newrem, perm_out, G, ldg, S1, d, keys_floats);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_select_seq(int mode, int p0, int bs, int m, const int* rem, int* blk,
                           int* newrem, int64_t* perm_out, hipStream_t st) {
  int work = (mode == 0) ? (m - p0) : bs;
  int grid = ceil_div(work > 0 ? work : 1, 256);
  if (grid > 64) grid = 64;
  hipLaunchKernelGGL(select_seq_kernel, dim3(grid), dim3(256), 0, st, mode, p0, bs, m, rem, blk,
                     newrem, perm_out);
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
      hipLaunchKernelGGL(s1_rows_kernel, dim3(ceil_div(b, 256)), dim3(256), 0, st, A, lda, blk, b, S1);
    else
      hipLaunchKernelGGL(s1_row_wg_kernel, dim3(b), dim3(128), 0, st, A, lda, blk, b, S1);
    PT2Q_LAUNCH_CHECK();
    hipLaunchKernelGGL(s1_total_kernel, dim3(1), dim3(256), 0, st, S1, b, d);
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

int pt2q_launch_ef_coeffs(const float* Hinv, long ldh, const int* blk, int bs, const int* rem,
                          int nr, float* C, long ldc, hipStream_t st) {
  hipLaunchKernelGGL(ef_coeff_kernel, dim3(ceil_div(nr, 256), bs), dim3(256), 0, st, Hinv, ldh,
                     blk, rem, nr, C, ldc);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}
