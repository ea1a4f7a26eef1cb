// Layout changes, Hessian damping, dequantisation, 2-bit packing and synthetic inputs.
#include "common.hpp"
#include "internal.hpp"

namespace {

template <typename T>
PT2Q_DEV float ld_f32(const T* p);
template <>
PT2Q_DEV float ld_f32<float>(const float* p) { return *p; }
template <>
PT2Q_DEV float ld_f32<_Float16>(const _Float16* p) { return (float)*p; }
template <>
PT2Q_DEV float ld_f32<uint16_t>(const uint16_t* p) { return __uint_as_float(((uint32_t)*p) << 16); }
template <>
PT2Q_DEV float ld_f32<int8_t>(const int8_t* p) { return (float)*p; }

// dst[c][r] = src[r][c] through a 32x33 LDS tile (coalesced on both sides).
template <typename TS, typename TD>
__global__ __launch_bounds__(256) void transpose_kernel(const TS* src, long lds, int rows, int cols,
                                                        TD* dst, long ldd) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  for (int y = ty; y < 32; y += 8) {
    int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < rows && c < cols) ? (float)ld_f32<TS>(src + (long)r * lds + c) : 0.0f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    int c = c0 + y, r = r0 + tx;
    if (c < cols && r < rows) dst[(long)c * ldd + r] = (TD)tile[tx][y];
  }
}

// 16-bit src -> f32 dst transpose through a 64 x 64 LDS tile: 16-byte loads (8 elements) and
// 16-byte stores (4 rows of one column).  Requires cols % 8 == 0, rows % 4 == 0, lds % 8 == 0,
// ldd % 4 == 0 and 16-byte aligned bases; ragged tile edges are masked.
template <typename TS>
__global__ __launch_bounds__(256) void transpose16_kernel(const TS* src, long lds, int rows, int cols,
                                                          float* dst, long ldd) {
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tid = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = p * 32 + tid / 8, c = (tid % 8) * 8;
    const bool in = r0 + r < rows && c0 + c < cols;
    uint4 v = in ? *(const uint4*)(src + (long)(r0 + r) * lds + c0 + c) : uint4{0, 0, 0, 0};
    const TS* e = (const TS*)&v;
#pragma unroll
    for (int u = 0; u < 8; ++u) tile[r][c + u] = ld_f32<TS>(e + u);
  }
  __syncthreads();
  typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int idx = p * 256 + tid, c = idx / 16, r = (idx % 16) * 4;
    if (c0 + c < cols && r0 + r < rows)
      *(f4*)(dst + (long)(c0 + c) * ldd + r0 + r) = f4{tile[r][c], tile[r + 1][c], tile[r + 2][c], tile[r + 3][c]};
  }
}

// int8 transpose through a 64 x 64 LDS tile: one 16-byte load and one 16-byte store per thread.
// Requires rows, cols, lds, ldd multiples of 16 and 16-byte aligned bases.
__global__ __launch_bounds__(256) void transpose_i8x16_kernel(const int8_t* src, long lds, int rows,
                                                              int cols, int8_t* dst, long ldd) {
  __shared__ int8_t tile[64][64 + 4];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tid = threadIdx.x;
  {
    const int r = tid / 4, c = (tid % 4) * 16;
    const bool in = r0 + r < rows && c0 + c < cols;
    const uint4 v = in ? *(const uint4*)(src + (long)(r0 + r) * lds + c0 + c) : uint4{0, 0, 0, 0};
    const int8_t* e = (const int8_t*)&v;
#pragma unroll
    for (int u = 0; u < 16; ++u) tile[r][c + u] = e[u];
  }
  __syncthreads();
  const int c = tid / 4, r = (tid % 4) * 16;
  if (c0 + c < cols && r0 + r < rows) {
    uint4 v;
    int8_t* e = (int8_t*)&v;
#pragma unroll
    for (int u = 0; u < 16; ++u) e[u] = tile[r + u][c];
    *(uint4*)(dst + (long)(c0 + c) * ldd + r0 + r) = v;
  }
}

__global__ void hess_scale_kernel(const float* G, long ldg, int m, float fn, float* H, long ldh) {
  long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)m * m) return;
  int r = (int)(q / m), c = (int)(q % m);
  H[(long)r * ldh + c] = G[(long)r * ldg + c] / fn;
}

// damp = percdamp * (SUMN(diag H) / m); H_ii += damp   (main.py:132-133, gptq.py:97-98)
__global__ __launch_bounds__(1024) void hess_damp_kernel(float* H, long ldh, int m, float percdamp,
                                                         float* damp_out) {
  __shared__ float dmp, tot;
  __shared__ float stage[SUMN_LDS_MAX];
  if (m <= SUMN_LDS_MAX) {
    const float p = block_sumn_lds<false>(H, m, ldh + 1, stage, &tot);
    if (threadIdx.x == 0) {
      dmp = percdamp * (p / (float)m);
      if (damp_out) *damp_out = dmp;
    }
  } else if (threadIdx.x < 64) {
    float p = sumn_lane<false>(H, m, ldh + 1, threadIdx.x);
    p = bfly64(p);
    if (threadIdx.x == 0) {
      dmp = percdamp * (p / (float)m);
      if (damp_out) *damp_out = dmp;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += blockDim.x) H[(long)i * ldh + i] = H[(long)i * ldh + i] + dmp;
}

// damp from the diagonal alone: h_ii = G_ii / fn (hess_scale's rounding), then the same SUMN
// and scaling as hess_damp_kernel.  *damp_dev feeds hess_fill_kernel (and the caller).
// batched: item blockIdx.x at G + z * bs, damp_dev[z]
__global__ __launch_bounds__(1024) void hess_diag_damp_kernel(const float* G, long ldg, int m, float fn,
                                                              float percdamp, float* damp_dev, long bs) {
  __shared__ float tot;
  G += (long)blockIdx.x * bs;
  damp_dev += blockIdx.x;
  __shared__ float stage[SUMN_LDS_MAX];
  for (int i = threadIdx.x; i < m; i += blockDim.x) stage[i] = G[(long)i * ldg + i] / fn;
  __syncthreads();
  if (threadIdx.x < 64) {
    float p = sumn_lane<false>(stage, m, 1, threadIdx.x);
    p = bfly64(p);
    if (threadIdx.x == 0) tot = percdamp * (p / (float)m);
  }
  __syncthreads();
  if (threadIdx.x == 0) *damp_dev = tot;
}

// H = G / fn with damp on the diagonal (hess_scale + hess_damp in one pass); upper_only: the
// strictly lower part is written as zero (H then is the Cholesky work matrix as is).
// batched: item blockIdx.y at G / H + z * bs, damp_dev[z]
__global__ void hess_fill_kernel(const float* G, long ldg, int m, float fn, const float* damp_dev,
                                 float* H, long ldh, int upper_only, long bs) {
  G += (long)blockIdx.y * bs;
  H += (long)blockIdx.y * bs;
  damp_dev += blockIdx.y;
  long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)m * m) return;
  int r = (int)(q / m), c = (int)(q % m);
  float h = G[(long)r * ldg + c] / fn;
  if (r == c) h = h + *damp_dev;
  H[(long)r * ldh + c] = (upper_only && c < r) ? 0.0f : h;
}

// hess_fill_kernel four columns per thread (m, ldg, ldh multiples of 4, 16-byte aligned)
__global__ void hess_fill4_kernel(const float* G, long ldg, int m, float fn, const float* damp_dev,
                                  float* H, long ldh, int upper_only, long bs) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  G += (long)blockIdx.y * bs;
  H += (long)blockIdx.y * bs;
  damp_dev += blockIdx.y;
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int m4 = m / 4;
  if (q >= (long)m * m4) return;
  const int r = (int)(q / m4), c0 = 4 * (int)(q % m4);
  const f4 g = *(const f4*)(G + (long)r * ldg + c0);
  const float dmp = *damp_dev;
  f4 h;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float x = g[u] / fn;
    if (r == c0 + u) x = x + dmp;
    h[u] = (upper_only && c0 + u < r) ? 0.0f : x;
  }
  *(f4*)(H + (long)r * ldh + c0) = h;
}

// gptq.py:213-228: out[:, perm[k*b + t]] = alpha[:,k] * T[:, col] + mu[:,k]
template <typename TT>
__global__ void dequant_kernel(const float* alpha, const float* mu, const TT* T,
                               const int64_t* perm, int n, int m, int b, int B, float* out) {
  long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)n * m) return;
  int i = (int)(q / m), pos = (int)(q % m);
  int k = pos / b;
  long col = perm ? perm[pos] : pos;
  float t = (float)T[(long)i * m + col];
  out[(long)i * m + col] = alpha[(long)i * B + k] * t + mu[(long)i * B + k];
}

__global__ void pack_kernel(const int8_t* T, long count, uint8_t* out) {
  long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long nb = (count + 3) / 4;
  if (q >= nb) return;
  uint8_t v = 0;
  for (int s = 0; s < 4; ++s) {
    long i = 4 * q + s;
    uint8_t c = (i < count) ? (uint8_t)(T[i] + 1) : 0;
    v |= (uint8_t)(c << (2 * s));
  }
  out[q] = v;
}

// 16 codes per thread (16-byte load, 4-byte store), the same bytes as pack_kernel: per byte
// c = T + 1 in {0, 1, 2} without carries between bytes ((b & 0x7f) + 1: -1 -> 0x80, 0 -> 1, 1 -> 2,
// then & 3), then the four 2-bit fields of a word folded into its low byte.
__global__ void pack16_kernel(const uint4* T, long n16, uint32_t* out) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n16) return;
  const uint4 w = T[q];
  const uint32_t v[4] = {w.x, w.y, w.z, w.w};
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t x = ((v[k] & 0x7f7f7f7fu) + 0x01010101u) & 0x03030303u;
    x |= x >> 6;
    x |= x >> 12;
    r |= (x & 0xffu) << (8 * k);
  }
  out[q] = r;
}

__global__ void unpack_kernel(const uint8_t* in, long count, int8_t* T) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  T[i] = (int8_t)((in[i >> 2] >> (2 * (i & 3))) & 3) - 1;
}

PT2Q_DEV uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_kernel(float* out, long count, uint64_t base, float scale, long cols,
                            int every, uint64_t obase, float oscale) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < count; i += (long)gridDim.x * blockDim.x) {
    uint64_t h = splitmix64(base + (uint64_t)i);
    float c = (float)((int64_t)(h >> 40) - (1ll << 23));
    float s = scale;
    if (every > 0) {
      uint64_t col = (uint64_t)(i % cols);
      if (splitmix64(obase + col) % (uint64_t)every == 0) s = oscale;
    }
    out[i] = c * s;
  }
}

// out[i] = ((P_0[i] + P_1[i]) + P_2[i]) + ... : the rank-ordered fold of per-rank partial Grams
// (intra-layer split, sharding.quantize_layer_split).  Four elements per thread (16-byte loads;
// count % 4 == 0, 16-byte aligned parts), every part's load issued before the first add.  With
// `acc0` the fold continues from acc0 (the result of the previous group of parts).
template <int NP>
__global__ __launch_bounds__(256) void sum_parts_kernel(const float* acc0, const float* P, long stride,
                                                        long count4, int parts, float* out) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < count4; q += (long)gridDim.x * 256) {
    f32x4 v[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if (p < parts) v[p] = *(const f32x4*)(P + p * stride + 4 * q);
    f32x4 acc = acc0 ? *(const f32x4*)(acc0 + 4 * q) : v[0];
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if (p < parts && (acc0 || p > 0)) acc = acc + v[p];
    *(f32x4*)(out + 4 * q) = acc;
  }
}

}  // namespace

int pt2q_launch_transpose_to_f32(const void* src, int dtype, long lds, int rows, int cols,
                                 float* dst, long ldd, hipStream_t st) {
  if ((dtype == PT2Q_F16 || dtype == PT2Q_BF16) && cols % 8 == 0 && rows % 4 == 0 && lds % 8 == 0 &&
      ldd % 4 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0) {
    dim3 g64(ceil_div(cols, 64), ceil_div(rows, 64));
    if (dtype == PT2Q_F16)
      hipLaunchKernelGGL(transpose16_kernel<_Float16>, g64, dim3(256), 0, st, (const _Float16*)src, lds,
                         rows, cols, dst, ldd);
    else
      hipLaunchKernelGGL(transpose16_kernel<uint16_t>, g64, dim3(256), 0, st, (const uint16_t*)src, lds,
                         rows, cols, dst, ldd);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  dim3 grid(ceil_div(cols, 32), ceil_div(rows, 32));
  switch (dtype) {
    case PT2Q_F32:
      hipLaunchKernelGGL((transpose_kernel<float, float>), grid, dim3(256), 0, st,
                         (const float*)src, lds, rows, cols, dst, ldd);
      break;
    case PT2Q_F16:
      hipLaunchKernelGGL((transpose_kernel<_Float16, float>), grid, dim3(256), 0, st,
                         (const _Float16*)src, lds, rows, cols, dst, ldd);
      break;
    case PT2Q_BF16:
      hipLaunchKernelGGL((transpose_kernel<uint16_t, float>), grid, dim3(256), 0, st,
                         (const uint16_t*)src, lds, rows, cols, dst, ldd);
      break;
    default:
      return PT2Q_E_ARG;
  }
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_transpose_i8(const int8_t* src, long lds, int rows, int cols, void* dst,
                             int ddtype, long ldd, hipStream_t st) {
  dim3 grid(ceil_div(cols, 32), ceil_div(rows, 32));
  if (ddtype == PT2Q_I8 && rows % 16 == 0 && cols % 16 == 0 && lds % 16 == 0 && ldd % 16 == 0 &&
      (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0)
    hipLaunchKernelGGL(transpose_i8x16_kernel, dim3(ceil_div(cols, 64), ceil_div(rows, 64)), dim3(256), 0,
                       st, src, lds, rows, cols, (int8_t*)dst, ldd);
  else if (ddtype == PT2Q_I8)
    hipLaunchKernelGGL((transpose_kernel<int8_t, int8_t>), grid, dim3(256), 0, st, src, lds, rows,
                       cols, (int8_t*)dst, ldd);
  else if (ddtype == PT2Q_F32)
    hipLaunchKernelGGL((transpose_kernel<int8_t, float>), grid, dim3(256), 0, st, src, lds, rows,
                       cols, (float*)dst, ldd);
  else
    return PT2Q_E_ARG;
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

int pt2q_launch_transpose_f32(const float* src, long lds, int rows, int cols, float* dst, long ldd,
                              hipStream_t st) {
  return pt2q_launch_transpose_to_f32(src, PT2Q_F32, lds, rows, cols, dst, ldd, st);
}

int pt2q_launch_prepare_hessian(const float* G, long ldg, int m, long nsamples, float percdamp,
                                float* H, long ldh, float* damp, hipStream_t st, bool upper_only, int batch,
                                long bs) {
  if (damp && m <= SUMN_LDS_MAX) {  // damp from the diagonal, then one pass over G (every item at once)
    hipLaunchKernelGGL(hess_diag_damp_kernel, dim3(batch), dim3(1024), 0, st, G, ldg, m, (float)nsamples,
                       percdamp, damp, bs);
    PT2Q_LAUNCH_CHECK();
    if (m % 4 == 0 && ldg % 4 == 0 && ldh % 4 == 0 && bs % 4 == 0 && (uintptr_t)G % 16 == 0 &&
        (uintptr_t)H % 16 == 0)
      hipLaunchKernelGGL(hess_fill4_kernel, dim3(ceil_div((long)m * (m / 4), 256), batch), dim3(256), 0, st, G,
                         ldg, m, (float)nsamples, damp, H, ldh, upper_only ? 1 : 0, bs);
    else
      hipLaunchKernelGGL(hess_fill_kernel, dim3(ceil_div((long)m * m, 256), batch), dim3(256), 0, st, G, ldg, m,
                         (float)nsamples, damp, H, ldh, upper_only ? 1 : 0, bs);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  if (upper_only) return PT2Q_E_UNSUPPORTED;
  if (batch != 1) return PT2Q_E_ARG;  // (the caller loops over items)
  hipLaunchKernelGGL(hess_scale_kernel, dim3(ceil_div((long)m * m, 256)), dim3(256), 0, st, G, ldg,
                     m, (float)nsamples, H, ldh);
  PT2Q_LAUNCH_CHECK();
  hipLaunchKernelGGL(hess_damp_kernel, dim3(1), dim3(1024), 0, st, H, ldh, m, percdamp, damp);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

extern "C" int pt2q_dequantize(const float* alpha, const float* mu, const void* T, int tdtype,
                               const int64_t* perm, int n, int m, int b, float* out,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0 || m <= 0 || b <= 0 || !alpha || !mu || !T || !out) return PT2Q_E_ARG;
  int B = (b < m) ? ceil_div(m, b) : 1;
  int bb = (b < m) ? b : m;
  long tot = (long)n * m;
  if (tdtype == PT2Q_I8)
    hipLaunchKernelGGL((dequant_kernel<int8_t>), dim3(ceil_div(tot, 256)), dim3(256), 0, st, alpha,
                       mu, (const int8_t*)T, perm, n, m, bb, B, out);
  else if (tdtype == PT2Q_F32)
    hipLaunchKernelGGL((dequant_kernel<float>), dim3(ceil_div(tot, 256)), dim3(256), 0, st, alpha,
                       mu, (const float*)T, perm, n, m, bb, B, out);
  else
    return PT2Q_E_ARG;
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

extern "C" int pt2q_pack_ternary(const int8_t* T, int64_t count, uint8_t* packed, void* stream) {
  if (count < 0 || !T || !packed) return PT2Q_E_ARG;
  long nb = (count + 3) / 4;
  if (nb == 0) return PT2Q_OK;
  if (count % 16 == 0 && ((uintptr_t)T & 15) == 0 && ((uintptr_t)packed & 3) == 0) {
    const long n16 = count / 16;
    hipLaunchKernelGGL(pack16_kernel, dim3(ceil_div(n16, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)T, n16, (uint32_t*)packed);
    PT2Q_LAUNCH_CHECK();
    return PT2Q_OK;
  }
  hipLaunchKernelGGL(pack_kernel, dim3(ceil_div(nb, 256)), dim3(256), 0, (hipStream_t)stream, T,
                     (long)count, packed);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

extern "C" int pt2q_unpack_ternary(const uint8_t* packed, int64_t count, int8_t* T, void* stream) {
  if (count < 0 || !T || !packed) return PT2Q_E_ARG;
  if (count == 0) return PT2Q_OK;
  hipLaunchKernelGGL(unpack_kernel, dim3(ceil_div(count, 256)), dim3(256), 0, (hipStream_t)stream,
                     packed, (long)count, T);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

extern "C" int pt2q_fill_synthetic(float* out, int64_t count, uint64_t seed, float scale,
                                   int64_t cols, int outlier_every, float scale_outlier,
                                   void* stream) {
  if (count < 0 || !out || (outlier_every > 0 && cols <= 0)) return PT2Q_E_ARG;
  if (count == 0) return PT2Q_OK;
  // host-side splitmix64 of the seeds (same function as device)
  auto sm = [](uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  uint64_t base = sm(seed);
  uint64_t obase = sm(seed ^ 0x5BD1E995ull);
  long grid = ceil_div(count, 256);
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, out,
                     (long)count, base, scale, (long)cols, outlier_every, obase, scale_outlier);
  PT2Q_LAUNCH_CHECK();
  return PT2Q_OK;
}

// out = ((parts[0] + parts[1]) + ...) + parts[nparts-1], elementwise fp32, parts `stride`
// floats apart (sharding.quantize_layer_split: the rank-ordered fold of partial Grams).
extern "C" int pt2q_sum_partials(const float* parts, int64_t stride, int nparts, int64_t count,
                                 float* out, void* stream) {
  if (nparts <= 0 || count < 0 || !parts || !out || (nparts > 1 && stride < count)) return PT2Q_E_ARG;
  if (count % 4 || stride % 4 || (uintptr_t)parts % 16 || (uintptr_t)out % 16) return PT2Q_E_UNSUPPORTED;
  if (count == 0) return PT2Q_OK;
  hipStream_t st = (hipStream_t)stream;
  const long c4 = count / 4;
  const unsigned grid = (unsigned)std::min<long>(ceil_div(c4, 256), 4096);
  constexpr int NP = 8;
  const float* acc0 = nullptr;
  for (int p0 = 0; p0 < nparts; p0 += NP) {  // groups of 8 parts; each group continues the fold
    const int np = std::min(NP, nparts - p0);
    if (np == 1 && !acc0 && out == parts) return PT2Q_OK;
    hipLaunchKernelGGL(sum_parts_kernel<NP>, dim3(grid), dim3(256), 0, st, acc0, parts + (long)p0 * stride,
                       (long)stride, c4, np, out);
    PT2Q_LAUNCH_CHECK();
    acc0 = out;
  }
  return PT2Q_OK;
}
