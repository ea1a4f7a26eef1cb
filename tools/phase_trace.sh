#!/bin/bash
# Kernel trace of tools/phase_times.py (GPU box): bash tools/phase_trace.sh TAG [phase_times args]
set -o pipefail
TAG=${1:-r03_phase}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/tools/phase_times.py "$@" > $OUT/phase.txt 2> $OUT/err || exit 1
cat $OUT/phase.txt
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/phase_kstats.py $f --json $OUT/stage_kernels.json > $OUT/phase_kstats.txt && cat $OUT/phase_kstats.txt
gzip -f $f
