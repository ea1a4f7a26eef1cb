#!/bin/bash
# PMC passes on the grouped per-channel ATQ (pt2q_quantize_perchannel_group, 16 bf16 linears of
# m = 5120 columns with C5's row counts): clock, VALU issue, wave-cycle split.  bash tools/pmc_pcg.sh TAG
set -o pipefail
TAG=${1:-pmc_pcg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-trace -d $OUT/$1 -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py pcg ${M:-5120} 16 2 > $OUT/$1.log 2>&1 || { echo "FAIL $1"; tail -3 $OUT/$1.log; exit 1; }
}
run valu "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" || exit 1
run wait "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit 1
python3 $R/tools/pmc_multi.py $OUT/valu $OUT/wait > $OUT/summary.txt
cat $OUT/summary.txt
