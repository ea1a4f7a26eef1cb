#!/bin/bash
# PMC passes on one grouped block loop (16 fp16 4096 x 4096 linears, SSR, variant M) and one
# batched inverse (GPU box): clock and MFMA busy, fabric fetch / write bytes, L2 hits, per kernel.
set -o pipefail
TAG=${1:-pmc_tails}
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
for w in "group 4096 4096 16 1" "inverse 11008 16 x 1"; do
  set -- $w
  k=$1
  run ${k}_mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" $w
  run ${k}_fetch "FETCH_SIZE" $w
  run ${k}_write "WRITE_SIZE" $w
done
python3 $R/tools/pmc_multi.py $OUT/group_mfma $OUT/group_fetch $OUT/group_write $OUT/inverse_mfma $OUT/inverse_fetch $OUT/inverse_write > $OUT/summary.txt && cat $OUT/summary.txt
