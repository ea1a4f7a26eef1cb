#!/bin/bash
# Build tools/_probe/gram16_probe*.bin (normal, fetch-only, compute-only) on the CPU side.
cd "$(dirname "$0")/.."
mkdir -p tools/_probe
for v in "" "-DGX_PROBE_NO_MFMA" "-DGX_PROBE_NO_DMA"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
    -I snlp---tenary-post-train-quantization_amd/csrc $v tools/gram16_probe.hip -o tools/_probe/gram16_probe${v}.bin || exit 1
done
