#!/bin/bash
# Round-4 A/B (GPU box): bench tests, then the 7B step under several schedules on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for V in "" "--inverse-overlap" "--inv-streams 3 --inv-chunk 11008:16" "--lanes 2" "EF1" ""; do
  if [ "$V" = EF1 ]; then export PT2Q_EF_V2=0; V=""; else export PT2Q_EF_V2=1; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra $V > $OUT/v$i.json 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/v$i.json'));print('variant $i [$V] EF_V2=$PT2Q_EF_V2', round(d['ms_per_step'],1), d['ranks'][0]['step_ms'])"
  i=$((i+1))
done
