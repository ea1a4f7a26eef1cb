#!/bin/bash
# Round-3 GPU check: selected tests (-k expr), then the default bench and a variant.
#   bash tools/gpu_r03.sh TAG "pytest -k expr" "extra bench args for the variant line"
set -o pipefail
TAG=${1:-r03}; K=${2:-}; V=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/gputest.log 2>&1
  rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('default', d['value'], d['ms_per_step'])"
if [ -n "$V" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-extra $V > $OUT/bench_v.json 2> $OUT/bench_v.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_v.json'));print('variant', d['value'], d['ms_per_step'])"
fi
