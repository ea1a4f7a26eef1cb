#!/bin/bash
# Round-5 checkpoint (GPU box): GPU tests (or a -k subset), smoke, one-lane phase trace (stage
# kernels + live stage busy).   bash tools/round_r05.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 300 bash $R/tools/phase_trace.sh ${TAG}_phase --lanes 1 > $OUT/phase.log 2>&1 || { tail $OUT/phase.log; exit 1; }
grep -A12 "== tails" $OUT/phase.log
timeout -k 10 200 python -u tools/stage_busy.py > $OUT/busy.json 2> $OUT/busy.err || exit 1
cat $OUT/busy.json
