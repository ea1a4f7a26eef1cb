#!/bin/bash
# Round-4 checkpoint c (GPU box): per-channel / layer GPU tests, the C5 one-lane kernel profile
# (wide waves 4 and 8), then the EF v2 check (tools/gpu_ef2.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r04c
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "config or per_channel or perchannel or layer or golden or 16bit" > $R/gpurun_out/r04c/tests.log 2>&1
rc=$?; tail -3 $R/gpurun_out/r04c/tests.log; [ $rc -eq 0 ] || exit $rc
bash $R/tools/c5_prof.sh r04c_c5 4 8 || exit 1
cd $R && bash tools/gpu_ef2.sh r04c_ef2
