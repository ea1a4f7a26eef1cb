#!/bin/bash
# Kernel trace of tools/time_inverse.py (GPU box): bash tools/inv_trace.sh TAG M BATCH [reps]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/tools/time_inverse.py "$@" > $OUT/inv.txt 2> $OUT/err || exit 1
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
gzip -f $f
