#!/bin/bash
# 7B step A/B over environment settings on one box: bash tools/gpu_env_ab.sh TAG "ENV=.. ENV=.." ...
# ("-" = defaults).  Each variant: bench.py --steps 3 --warmup 1 --no-extra.
set -o pipefail
TAG=${1:-envab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
i=0
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  env $E timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/v$i.json 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/v$i.json'));print('[$E]', round(d['ms_per_step'],1), d['ranks'][0]['step_ms'])"
  i=$((i+1))
done
