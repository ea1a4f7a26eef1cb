#!/bin/bash
# EF v2 check (GPU box): EF-touching GPU tests with PT2Q_EF_V2=1, then the 7B step and its live
# stage busy times with v1 and v2.   bash tools/gpu_ef2.sh TAG
set -o pipefail
TAG=${1:-ef2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export PT2Q_EF_V2=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "error_feedback or blocks_group or quantize_layer or headline or config or grams_first or layer_m or loop16 or unit_pipeline or stage_timing" > $OUT/gputest_v2.log 2>&1
rc=$?; tail -3 $OUT/gputest_v2.log; [ $rc -eq 0 ] || exit $rc
for V in 0 1; do
  export PT2Q_EF_V2=$V
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/bench_v$V.json 2> $OUT/bench_v$V.err || { tail $OUT/bench_v$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_v$V.json'));print('EF_V2=$V', round(d['ms_per_step'],1), d['ranks'][0]['step_ms'])"
  timeout -k 10 300 python -u tools/stage_busy.py > $OUT/busy_v$V.json 2> $OUT/busy_v$V.err || { tail $OUT/busy_v$V.err; exit 1; }
  cat $OUT/busy_v$V.json
done
