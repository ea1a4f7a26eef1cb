#!/bin/bash
# Round-5 HEAD measurement (GPU box): one-lane phase trace (stage kernels), rocprofv3 kernel trace of
# the 7B bench step, PT2Q_ATQ_OCC A/B of the live stage busy, and the one-lane C5 kernel trace.
set -o pipefail
TAG=${1:-r05a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 bash $R/tools/phase_trace.sh ${TAG}_phase --lanes 1 > $OUT/phase.log 2>&1 || { tail $OUT/phase.log; exit 1; }
tail -25 $OUT/phase.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-configs --no-h2d > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
f=$(find $OUT/bench_trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kstats.py $f > $OUT/bench_kstats.txt 2>&1 && head -30 $OUT/bench_kstats.txt
gzip -f $f
cd $R
for occ in 0 6; do
  PT2Q_ATQ_OCC=$occ timeout -k 10 200 python -u tools/stage_busy.py > $OUT/busy_occ$occ.json 2> $OUT/busy_occ$occ.err || exit 1
  echo "occ=$occ $(cat $OUT/busy_occ$occ.json)"
done
timeout -k 10 400 bash $R/tools/c5_prof.sh ${TAG}_c5 4 > $OUT/c5.log 2>&1 || { tail $OUT/c5.log; exit 1; }
cat $OUT/c5.log
