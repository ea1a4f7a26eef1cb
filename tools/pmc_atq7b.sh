#!/bin/bash
# PMC passes on the block ATQ of a grouped 7B loop (16 fp16 4096 x 4096 linears): VALU issue,
# wave-cycle split; and the ITF iteration counts of one synthetic layer.  bash tools/pmc_atq7b.sh TAG
set -o pipefail
TAG=${1:-pmc_atq7b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-trace -d $OUT/$1 -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py group 4096 4096 16 1 > $OUT/$1.log 2>&1 || { echo "FAIL $1"; tail -3 $OUT/$1.log; exit 1; }
}
run valu "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS" || exit 1
run wait "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit 1
python3 $R/tools/pmc_multi.py $OUT/valu $OUT/wait > $OUT/summary.txt
grep -E "==|atq_" $OUT/summary.txt
cd $R && timeout -k 10 120 python3 tools/itf_iters.py
