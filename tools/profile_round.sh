#!/bin/bash
# Profiling pass for one round (run on the GPU box from the repo root via gpurun):
#   1. kernel-trace + stats of the default bench (per-kernel durations; the Gram average must
#      agree with bench.py's HIP-event number)
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) on the Gram alone
# Outputs under gpurun_out/prof_<tag>/ ; tools/summarize_profiles.py turns them into profiles/.
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-3}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-n2048 > $OUT/bench_under_trace.json 2> $OUT/trace.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/pmc_$ctr -o run --output-format csv -- \
    python3 $R/tools/bench_gram.py 262144 4096 fp16 > $OUT/pmc_$ctr.log 2>&1 || exit 1
done
echo "profile pass done"
