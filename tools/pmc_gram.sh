#!/bin/bash
# PMC passes (one counter set per run) on the batched Gram: bash tools/pmc_gram.sh TAG (GPU box)
set -o pipefail
TAG=${1:-pmc_gram}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters, workload args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/$name -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py "$@" > $OUT/$name.log 2>&1 || { echo "FAIL $name"; tail -3 $OUT/$name.log; exit 1; }
  echo "ok $name"
}
for w in "4096 24" "11008 8"; do
  set -- $w
  run g$1_mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" grams 262144 $1 $2 2
  run g$1_fetch "FETCH_SIZE" grams 262144 $1 $2 2
  run g$1_write "WRITE_SIZE" grams 262144 $1 $2 2
  run g$1_hit "TCC_HIT_sum TCC_MISS_sum" grams 262144 $1 $2 2
done
python3 $R/tools/pmc_multi.py $OUT/g4096_mfma $OUT/g4096_fetch $OUT/g4096_write $OUT/g11008_mfma $OUT/g11008_fetch $OUT/g11008_write > $OUT/summary.txt && cat $OUT/summary.txt
