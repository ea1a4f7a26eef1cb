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

// Butterfly over the 16 lanes of a lane group (xor 8,4,2,1): every lane ends with the same sum.
PT2Q_DEV float bfly16(float p) {
  p = p + __shfl_xor(p, 8);
  p = p + __shfl_xor(p, 4);
  p = p + __shfl_xor(p, 2);
  p = p + __shfl_xor(p, 1);
  return p;
}

// Butterfly over a whole wave64 (xor 32..1).
PT2Q_DEV float bfly64(float p) {
  p = p + __shfl_xor(p, 32);
  p = p + __shfl_xor(p, 16);
  p = p + __shfl_xor(p, 8);
  p = p + __shfl_xor(p, 4);
  p = p + __shfl_xor(p, 2);
  p = p + __shfl_xor(p, 1);
  return p;
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

#define PT2Q_LAUNCH_CHECK()                                      \
  do {                                                           \
    if (hipGetLastError() != hipSuccess) return PT2Q_E_HIP;      \
  } while (0)
