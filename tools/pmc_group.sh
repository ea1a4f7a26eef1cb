#!/bin/bash
# PMC passes on the grouped block loop of COUNT n x m linears: bash tools/pmc_group.sh TAG N M COUNT
set -o pipefail
TAG=${1:-pmc_group}; N=${2:-11008}; M=${3:-4096}; C=${4:-16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-trace -d $OUT/$1 -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py group $N $M $C 2 > $OUT/$1.log 2>&1 || { echo "FAIL $1"; tail -3 $OUT/$1.log; exit 1; }
  echo "ok $1"
}
run mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
run wait "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
run occ "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
python3 $R/tools/pmc_multi.py $OUT/mfma $OUT/fetch $OUT/write $OUT/wait > $OUT/summary.txt && cat $OUT/summary.txt
