#!/bin/bash
# ATQ change check (GPU box): ATQ / layer / group parity tests, then the live per-stage busy times.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${1:-atq}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "atq or ssr or layer or group or gptq or per_channel or model" > $OUT/test.log 2>&1
rc=$?; tail -2 $OUT/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/stage_busy.py > $OUT/busy.json 2> $OUT/busy.err || { tail $OUT/busy.err; exit 1; }
cat $OUT/busy.json
