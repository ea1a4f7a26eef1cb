#!/bin/bash
# A/B env settings on one box: bash tools/ab_env.sh TAG "VAR=1 VAR2=0" "VAR=0" ... (bench defaults,
# 1 warmup + 3 steps each; "" = the library defaults)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
i=0
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra > $OUT/v$i.json 2> $OUT/v$i.err || { tail -5 $OUT/v$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/v$i.json'));print('%-40s %8.1f ms/step' % (sys.argv[1] or 'default', d['ms_per_step']))" "$v"
  i=$((i+1))
done
