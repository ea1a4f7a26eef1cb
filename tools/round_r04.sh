#!/bin/bash
# Round-4 checkpoint (GPU box): full GPU tests, smoke, one-lane phase trace (stage kernels), the
# default bench line, and a rocprofv3 kernel trace of the bench (Gram launch average cross-check).
set -o pipefail
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
rc=$?; tail -2 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 300 bash $R/tools/phase_trace.sh ${TAG}_phase --lanes 1 > $OUT/phase.log 2>&1 || { tail $OUT/phase.log; exit 1; }
cp $R/gpurun_out/${TAG}_phase/stage_kernels.json $R/profiles/stage_kernels.json  # (box copy; copy it locally too)
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['roofline']['stages']['step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-configs --no-h2d > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
f=$(find $OUT/bench_trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kstats.py $f > $OUT/bench_kstats.txt 2>&1 && head -30 $OUT/bench_kstats.txt
gzip -f $f
# live stage busy with the block-ATQ occupancy floor off and on (PT2Q_ATQ_OCC)
cd $R
for occ in 0 6; do
  PT2Q_ATQ_OCC=$occ timeout -k 10 200 python -u tools/stage_busy.py > $OUT/busy_occ$occ.json 2> $OUT/busy_occ$occ.err || exit 1
  echo "occ=$occ $(cat $OUT/busy_occ$occ.json)"
done
