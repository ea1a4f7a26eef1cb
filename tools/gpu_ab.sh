#!/bin/bash
# A/B of bench variants on one box (GPU box): the full GPU test suite (unless SKIPTESTS=1), then
# the 7B step once per variant (no extras), then the C5 step with a rocprofv3 kernel summary.
#   bash tools/gpu_ab.sh TAG "variant args" ["variant args" ...]
set -o pipefail
TAG=${1:-ab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIPTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
  rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for V in "$@"; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra $V > $OUT/v$i.json 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/v$i.json'));print('variant [$V]', round(d['ms_per_step'],1), d['ranks'][0]['step_ms'])"
  i=$((i+1))
done
if [ -z "$SKIPC5" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5_trace -o run --output-format csv -- \
    python3 $R/bench.py --model llama-2-13b --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $OUT/c5_prof.json 2> $OUT/c5_prof.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c5_prof.json'));print('C5 (under rocprof)', round(d['ms_per_step'],1))"
  f=$(find $OUT/c5_trace -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/kstats.py $f > $OUT/c5_kstats.txt 2>&1 && head -16 $OUT/c5_kstats.txt
  gzip -f $f
fi
