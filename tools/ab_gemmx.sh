#!/bin/bash
# gemmx ring A/B (GPU box): batched inverses (the bench's per-width inverse workloads) per
# PT2Q_GEMMX_STAGES setting, then the inverse parity tests under each setting
set -o pipefail
mkdir -p gpurun_out/abx
for v in 2 4 5 2; do
  for w in "4096 32" "11008 16"; do
    set -- $w
    PT2Q_GEMMX_STAGES=$v timeout -k 10 120 python -u tools/time_inverse.py $1 $2 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/abx/out.txt
for v in 4 5; do
  PT2Q_GEMMX_STAGES=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "inverse or cholesky or hessian" --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
done
