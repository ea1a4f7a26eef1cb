#!/bin/bash
# Build the ef2 clock probes (build container): tools/_probe/ef2clk_<k> (ef.hip compiled in with
# per-workgroup clock stamps and the build-time knock-out mask k: 0 whole, 1 no Wt traffic, 2 operand
# DMAs from one chunk, 4 no MFMAs)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
L=$R/snlp---tenary-post-train-quantization_amd
mkdir -p $R/tools/_probe
for k in 0 1 2 4 5 8 16 24; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -I$R/include \
    -DPT2Q_PROBE=64 -DPT2Q_EF2_KPROBE=$k $R/tools/ef_probe.hip -L$L -lpt2q \
    -Wl,-rpath,'$ORIGIN/../../snlp---tenary-post-train-quantization_amd' -o $R/tools/_probe/ef2clk_$k 2>&1 | grep -v warning &
done
wait
