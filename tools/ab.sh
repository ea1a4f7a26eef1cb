#!/bin/bash
# A/B bench variants on one box: bash tools/ab.sh TAG "args A" "args B" ... (each: 1 warmup + 3 steps)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
i=0
for v in "$@"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra $v > $OUT/v$i.json 2> $OUT/v$i.err || { tail -5 $OUT/v$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/v$i.json'));print('%-40s %8.1f ms/step' % (sys.argv[1] or 'default', d['ms_per_step']))" "$v"
  i=$((i+1))
done
