#!/bin/bash
# EF probe pass (GPU box): knock-out timings and the per-phase timestamps (tools/build_ef_probe.sh)
set -o pipefail
mkdir -p gpurun_out/efp
for m in ${@:-0 8 16 32 56 64}; do
  timeout -k 10 60 tools/_probe/ef_probe_$m 16384 4096 128 20 1 || exit 1
  timeout -k 10 60 tools/_probe/ef_probe_$m 4096 8192 128 20 1 || exit 1
  timeout -k 10 60 tools/_probe/ef_probe_$m 4096 2048 128 50 1 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/efp/out.txt
