#!/bin/bash
# PMC passes (one counter set per run) on the batched inverse and the grouped block loop.
set -o pipefail
TAG=${1:-pmc_r03}
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
run inv11008_mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" inverse 11008 8 1 2
run inv4096_mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" inverse 4096 32 1 2
run grp4096_mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" group 4096 4096 16 2
run grp4096_fetch "FETCH_SIZE" group 4096 4096 16 2
run grp4096_write "WRITE_SIZE" group 4096 4096 16 2
run grp4096_wait "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS" group 4096 4096 16 2
