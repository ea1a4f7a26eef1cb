#!/bin/bash
# PMC passes on one grouped block loop (16 fp16 4096 x 4096 linears) with the error feedback of
# PT2Q_EF_V2 = 0 (ef_gemm_kernel) and 1 (ef2_gemm_kernel): clock, MFMA busy, wave-cycle split
# (parked / issue-stall / active), LDS bank conflicts, fabric bytes.   bash tools/pmc_ef2.sh TAG
set -o pipefail
TAG=${1:-pmc_ef2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters
  local name=$1 ctr=$2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/$name -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py group 4096 4096 16 1 > $OUT/$name.log 2>&1 || { echo "FAIL $name"; tail -3 $OUT/$name.log; exit 1; }
}
for V in 0 1; do
  export PT2Q_EF_V2=$V
  run v${V}_mfma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" || exit 1
  run v${V}_wait "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit 1
  run v${V}_lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" || exit 1
  run v${V}_fetch "FETCH_SIZE" || exit 1
  run v${V}_write "WRITE_SIZE" || exit 1
  python3 $R/tools/pmc_multi.py $OUT/v${V}_mfma $OUT/v${V}_wait $OUT/v${V}_lds $OUT/v${V}_fetch $OUT/v${V}_write > $OUT/summary_v$V.txt
  grep -E "==|ef2?_gemm" $OUT/summary_v$V.txt
done
