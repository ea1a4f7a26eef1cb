#!/bin/bash
# PMC passes on tools/gram16_probe.bin (dev tool; GPU box, repo root). One counter group per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
    $R/tools/gram16_probe.bin ${1:-262144} ${2:-4096} 3 > $OUT/p$i.log 2>&1 || exit 1
done
echo pmc done
