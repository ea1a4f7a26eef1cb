#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ef
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  PT2Q_EF_WG2=$v timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $OUT/m$v -o run --output-format csv -- python3 $R/tools/kern_workloads.py group 4096 4096 16 2 > $OUT/m$v.log 2>&1 || exit 1
  PT2Q_EF_WG2=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $OUT/w$v -o run --output-format csv -- python3 $R/tools/kern_workloads.py group 4096 4096 16 2 > $OUT/w$v.log 2>&1 || exit 1
done
python3 $R/tools/pmc_multi.py $OUT/m1 $OUT/w1 $OUT/m0 $OUT/w0 | grep -E "==|ef_gemm"
