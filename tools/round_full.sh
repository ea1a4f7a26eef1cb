#!/bin/bash
# Full checkpoint (GPU box): all GPU tests, smoke, the default bench line, and a one-lane
# C5 kernel trace.   bash tools/round_r05_full.sh TAG
set -o pipefail
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
ts=$(date +%s); timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - ts )) s"
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 1), "frac", round(r["frac"], 3), "frac_2nm2", round(r["frac_2nm2"], 3))
print("stage_busy", r.get("stage_busy_ms"))
for k, v in d["extra"].get("configs", {}).items():
    print(k, round(v.get("ms_per_step", 0), 1), json.dumps(v.get("roofline", {}).get("dominant")))
cb = d.get("cpu_baseline", {})
print("cpu", cb.get("value"), cb.get("reference_estimate", {}).get("value"))
PY
