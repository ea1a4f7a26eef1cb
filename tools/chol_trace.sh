#!/bin/bash
# Kernel trace of the Cholesky inverse (GPU box, repo root, via gpurun): bash tools/chol_trace.sh TAG M
set -o pipefail
TAG=$1; M=${2:-11008}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/chol_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 $R/tools/bench_chol.py $M > $OUT/bench.txt 2>&1 || exit 1
python3 $R/tools/kstats.py $(find $OUT -name "run_kernel_trace.csv" | head -1) --after hess_fill > $OUT/kstats.txt
