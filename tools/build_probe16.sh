#!/bin/bash
# Build tools/_probe/gram16_probe*.bin (normal, fetch-only, compute-only) on the CPU side.
# The variants are the PT2Q_PROBE masks of csrc/probe.hpp (2: no MFMA, 1: no LDS-DMA).
cd "$(dirname "$0")/.."
mkdir -p tools/_probe
for v in "0:" "2:_NO_MFMA" "1:_NO_DMA"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
    -I snlp---tenary-post-train-quantization_amd/csrc -DPT2Q_PROBE=${v%%:*} tools/gram16_probe.hip \
    -o tools/_probe/gram16_probe${v#*:}.bin || exit 1
done
