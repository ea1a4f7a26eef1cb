// Development probes behind ONE switch.  Dev tools under tools/ build a kernel source with
// -DPT2Q_PROBE=<mask>; the library build never defines it, so every constant below is false and
// each hook (`if constexpr (probe::...)`, PT2Q_TOPK_STAMP) compiles to nothing.
#pragma once

#ifndef PT2Q_PROBE
#define PT2Q_PROBE 0
#endif

namespace probe {
constexpr bool gram_no_dma = (PT2Q_PROBE & 1) != 0;   // tools/gram16_probe.hip: compute-only (stale LDS)
constexpr bool gram_no_mfma = (PT2Q_PROBE & 2) != 0;  // tools/gram16_probe.hip: fetch-only
constexpr bool topk_stamps = (PT2Q_PROBE & 4) != 0;   // tools/topk_probe.hip: phase timestamps
constexpr bool ef_drop_wt = (PT2Q_PROBE & 8) != 0;    // tools/ef_probe.hip: Wt loads / stores dropped
constexpr bool ef_no_mfma = (PT2Q_PROBE & 16) != 0;   // tools/ef_probe.hip: no MFMAs
constexpr bool ef_zero_dma = (PT2Q_PROBE & 32) != 0;  // tools/ef_probe.hip: operand DMAs from one chunk
constexpr bool ef_stamps = (PT2Q_PROBE & 64) != 0;    // tools/ef_probe.hip: per-tile phase timestamps
constexpr bool ef_no_dma = (PT2Q_PROBE & 128) != 0;   // tools/ef_probe.hip: no operand DMAs (stale LDS)
}  // namespace probe

#if (PT2Q_PROBE & 4) != 0
// thread 0 of each of the first 64 workgroups of the top-k launch: s_memtime at phase i
__device__ long long topk_stamps[64][16];
#define PT2Q_TOPK_STAMP(i) \
  if (threadIdx.x == 0 && blockIdx.x < 64) topk_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime()
#else
#define PT2Q_TOPK_STAMP(i)
#endif

#if (PT2Q_PROBE & 64) != 0
// thread 0 of each of the first 64 workgroups of the EF launch: s_memrealtime (100 MHz) at phase i of its
// first 8 tiles (ef_stamps[wg][tile][i]); ef_stamp_tile counts the workgroup's tiles
// (ef_clk: s_memtime, the shader clock, at phases 0 and 7: the clock the kernel ran at)
__device__ long long ef_stamps[64][8][12];
__device__ long long ef_clk[64][8][2];
#define PT2Q_EF_STAMP(tile, i)                                                   \
  if (threadIdx.x == 0 && blockIdx.x < 64 && (tile) < 8) {                       \
    ef_stamps[blockIdx.x][tile][i] = __builtin_amdgcn_s_memrealtime();           \
    if ((i) == 0 || (i) == 7) ef_clk[blockIdx.x][tile][(i) / 7] = __builtin_amdgcn_s_memtime(); \
  }
#else
#define PT2Q_EF_STAMP(tile, i)
#endif

#if (PT2Q_PROBE & 64) != 0
// ef2_gemm_kernel: thread 0 of each workgroup, s_memtime (shader clock) and s_memrealtime
// (100 MHz) at the kernel's start (i = 0) and end (i = 1): the clock the launch ran at
__device__ long long ef2_clk[1024][4];
#define PT2Q_EF2_CLK(i)                                                  \
  if (threadIdx.x == 0 && blockIdx.x < 1024) {                           \
    ef2_clk[blockIdx.x][2 * (i)] = __builtin_amdgcn_s_memtime();         \
    ef2_clk[blockIdx.x][2 * (i) + 1] = __builtin_amdgcn_s_memrealtime(); \
  }
#else
#define PT2Q_EF2_CLK(i)
#endif

// ef2_gemm_kernel's runtime knock-out mask, fixed at build time by a probe tool (tools/ef_probe.hip:
// -DPT2Q_EF2_KPROBE=1 no Wt traffic, 2 operand DMAs from one chunk, 4 no MFMAs, 8 old-value loads
// from L2-hot rows, 16 stores to them; results garbage)
#ifndef PT2Q_EF2_KPROBE
#define PT2Q_EF2_KPROBE 0
#endif
