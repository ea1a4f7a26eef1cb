#!/bin/bash
# FETCH_SIZE / TCC hit-miss / MFMA busy of the 16-bit Gram (dev tool): tools/pmc_pair.sh m...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcpair
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  i=0
  for ctr in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/m${m}/p$i -o run --output-format csv -- \
      python3 $R/tools/bench_gram.py 262144 $m fp16 > $OUT/m${m}_$i.log 2>&1 || exit 1
  done
done
echo pmc done
