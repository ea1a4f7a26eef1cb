#!/bin/bash
# Per-shape kernel traces of the model's three layer shapes at N = 2048 (tails dominate).
# usage (repo root, via gpurun): bash tools/shape_traces.sh TAG
set -o pipefail
TAG=${1:-shapes}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for s in "4096 4096" "11008 4096" "4096 11008"; do
  set -- $s
  OUT=$R/gpurun_out/$TAG/${1}x${2}
  mkdir -p $OUT
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 $R/tools/run_shape.py $1 $2 2048 2 > $OUT/run.log 2>&1 || exit 1
  python3 $R/tools/kstats.py $(find $OUT -name "run_kernel_trace.csv" | head -1) --top 16 > $OUT/kstats.txt || exit 1
  echo "== ${1}x${2}"; cat $OUT/kstats.txt
done
