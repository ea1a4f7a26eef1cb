#!/bin/bash
# PMC passes of the 16-bit Gram alone (GPU box, repo root, via gpurun), one counter per run:
#   bash tools/pmc_gram.sh TAG M [N]      -> gpurun_out/pmc_<TAG>/<CTR>/  (tools/pmc_table.py reads it)
set -o pipefail
TAG=$1; M=${2:-11008}; N=${3:-262144}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/$ctr -o run --output-format csv -- \
    python3 $R/tools/bench_gram.py $N $M fp16 > $OUT/$ctr.log 2>&1 || exit 1
done
echo "pmc $TAG done"
