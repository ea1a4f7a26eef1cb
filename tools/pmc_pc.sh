#!/bin/bash
# PMC passes on the per-channel ATQ (C5 shapes: 13824 x 5120 and 5120 x 13824 bf16): clock, VALU
# instruction counts and busy, wave-cycle split, LDS, fabric bytes.   bash tools/pmc_pc.sh TAG
set -o pipefail
TAG=${1:-pmc_pc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters, shape
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-trace -d $OUT/$1 -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py pc $3 4 1 > $OUT/$1.log 2>&1 || { echo "FAIL $1"; tail -3 $OUT/$1.log; exit 1; }
}
for S in "13824 5120" "5120 13824"; do
  T=${S// /x}
  run ${T}_valu "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "$S" || exit 1
  run ${T}_wait "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "$S" || exit 1
  run ${T}_fetch "FETCH_SIZE" "$S" || exit 1
  python3 $R/tools/pmc_multi.py $OUT/${T}_valu $OUT/${T}_wait $OUT/${T}_fetch > $OUT/summary_$T.txt
  cat $OUT/summary_$T.txt
done
