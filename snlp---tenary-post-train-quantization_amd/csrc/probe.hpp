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
}  // namespace probe

#if (PT2Q_PROBE & 4) != 0
// thread 0 of each of the first 64 workgroups of the top-k launch: s_memtime at phase i
__device__ long long topk_stamps[64][16];
#define PT2Q_TOPK_STAMP(i) \
  if (threadIdx.x == 0 && blockIdx.x < 64) topk_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime()
#else
#define PT2Q_TOPK_STAMP(i)
#endif
