#!/bin/bash
# Build the error-feedback probes (build container): tools/_probe/ef_probe_<mask> (ef.hip compiled
# in with the probe mask; pt2q_tuning and the rest from libpt2q.so)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
L=$R/snlp---tenary-post-train-quantization_amd
mkdir -p $R/tools/_probe
for mask in 0 8 16 32 56 64 192 200 80 96; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -I$R/include \
    -DPT2Q_PROBE=$mask $R/tools/ef_probe.hip -L$L -lpt2q -Wl,-rpath,'$ORIGIN/../../snlp---tenary-post-train-quantization_amd' \
    -o $R/tools/_probe/ef_probe_$mask 2>&1 | grep -v warning &
done
wait
