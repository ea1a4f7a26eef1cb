#!/bin/bash
# Cholesky panel / sub-panel A/B on the batched inverses (GPU box)
set -o pipefail
mkdir -p gpurun_out/abp
for cfg in "0 256" "1024 256" "2048 256" "2048 512" "0 512" "0 128" "0 256"; do
  set -- $cfg
  for w in "4096 32" "11008 16"; do
    set -- $cfg $w
    PT2Q_CHOL_PANEL=$1 PT2Q_CHOL_SUBPANEL=$2 timeout -k 10 120 python -u tools/time_inverse.py $3 $4 | sed "s/^/panel=$1 sub=$2 /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/abp/out.txt
