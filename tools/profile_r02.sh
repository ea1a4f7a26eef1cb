#!/bin/bash
# Round-2 profiling pass (GPU box, repo root, via gpurun): bash tools/profile_r02.sh TAG
#  1. kernel trace + stats of one default-bench step (the whole Llama-2-7B model)
#  2. PMC passes (one counter per run, as MI355X_MICROARCH.md prescribes) on
#     - the 16-bit Gram at both widths of the model (tools/bench_gram.py 262144 {4096,11008})
#     - the headline layer, eager (tools/run_layer.py: Cholesky, SSR, ATQ, EF kernels)
#     - the m = 11008 Cholesky inverse (tools/bench_chol.py 11008: gemmx, rank_update2, panels)
set -o pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra > $OUT/bench_under_trace.json 2> $OUT/trace.err || exit 1
echo "trace done"
for ctr in FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  for m in 4096 11008; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/gram${m}_$ctr -o run --output-format csv -- \
      python3 $R/tools/bench_gram.py 262144 $m fp16 > $OUT/gram${m}_$ctr.log 2>&1 || exit 1
  done
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/layer_$ctr -o run --output-format csv -- \
    python3 $R/tools/run_layer.py 2 > $OUT/layer_$ctr.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/chol_$ctr -o run --output-format csv -- \
    python3 $R/tools/bench_chol.py 11008 > $OUT/chol_$ctr.log 2>&1 || exit 1
  echo "pmc $ctr done"
done
echo "profile pass done"
