#!/bin/bash
# rocprofv3 kernel trace + stats of the headline bench line (GPU box): bash tools/final_prof.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-extra --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
t=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 - "$t" "$OUT/bench.json" > $OUT/summary.txt <<'PY'
import csv, json, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("bench:", round(d["ms_per_step"], 1), "ms/step; roofline", json.dumps(d.get("roofline"))[:400])
for n, (c, ms) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{ms:10.2f} ms {c:6d}x avg {ms / c * 1e3:10.1f} us  {n[:90]}")
PY
gzip -f $t
cat $OUT/summary.txt
