#!/bin/bash
# Kernel trace of the headline layer run eagerly (tools/run_layer.py) -> per-kernel averages.
# usage (repo root, via gpurun): bash tools/layer_trace.sh TAG
set -o pipefail
TAG=${1:-ltrace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
  python3 $R/tools/run_layer.py 3 > $OUT/run.log 2>&1 || exit 1
python3 $R/tools/kstats.py $(find $OUT -name "run_kernel_trace.csv" | head -1) --top 30 > $OUT/kstats.txt || exit 1
echo "layer trace done"
