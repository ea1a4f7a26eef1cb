#!/bin/bash
# HIP runtime calls longer than 1 ms in a short bench run (dev tool, GPU box): finds one-off host
# stalls (allocations, synchronising copies) inside timed steps.  bash tools/slow_api.sh TAG [bench args]
set -o pipefail
TAG=${1:-slowapi}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace -d $OUT/t -o run --output-format csv -- \
  python3 $R/bench.py "$@" > $OUT/b.json 2> $OUT/b.err || exit 1
grep -h "timed\|step_ms" $OUT/b.err | tail -3
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/t/**/*hip_api_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
slow = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Function"]) for r in rows]
slow = [s for s in slow if s[1] > 1e6]
cnt = collections.Counter(s[2] for s in slow)
print("calls > 1 ms:", cnt.most_common(12))
for s in sorted(slow, key=lambda s: -s[1])[:25]:
    print(f"  t={s[0]/1e9:8.3f}s  {s[1]/1e6:8.2f} ms  {s[2]}")
PY
