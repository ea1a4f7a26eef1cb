#!/bin/bash
# Round-4 GPU check (GPU box): selected GPU tests (-k expr), the C5 (per-channel) step with a
# rocprofv3 kernel summary, then the default bench line (no CPU baseline).
#   bash tools/gpu_r04.sh TAG "pytest -k expr" [skip-default]
set -o pipefail
TAG=${1:-r04}; K=${2:-}; SKIP=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/gputest.log 2>&1
  rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --model llama-2-13b --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print('C5', d['ms_per_step'], json.dumps(d['roofline'].get('stages',{}).get('dominant')))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5_trace -o run --output-format csv -- \
  python3 $R/bench.py --model llama-2-13b --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $OUT/c5_prof.json 2> $OUT/c5_prof.err || exit 1
f=$(find $OUT/c5_trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kstats.py $f > $OUT/c5_kstats.txt 2>&1 && head -25 $OUT/c5_kstats.txt
gzip -f $f
cd $R
if [ -z "$SKIP" ]; then
  timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('default', d['value'], d['ms_per_step'], json.dumps(d['roofline']['stages']['dominant']), json.dumps({k:v.get('ms_per_step') for k,v in d['extra']['configs'].items()}))"
fi
