#!/bin/bash
# Kernel trace of one default-bench step (the whole 7B model) on the GPU box: per-kernel totals.
# usage (repo root, via gpurun): bash tools/trace_model.sh TAG
set -o pipefail
TAG=${1:-trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 $R/tools/kstats.py $(find $OUT -name "run_kernel_trace.csv" | head -1) --top 40 > $OUT/kstats.txt || exit 1
echo "trace done"
python3 $R/tools/overlap.py $(find $OUT -name "run_kernel_trace.csv" | head -1) > $OUT/overlap.txt || exit 1
