#!/bin/bash
# Round-end pass (GPU box, repo root): bash tools/round_pass.sh TAG
#   pytest -m gpu, smoke(), the default bench line, and a kernel trace of one bench step.
set -o pipefail
TAG=${1:-r02f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/bench_under_trace.json 2> $OUT/trace.err
echo "trace rc $?"
