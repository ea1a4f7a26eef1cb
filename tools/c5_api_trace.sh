#!/bin/bash
# HIP API trace of one C5 step (dev tool, GPU box): counts of hipMemcpy* / hipMemset* / launches
# by kind and size, to find the per-linear small copies of the C5 tail.  bash tools/c5_api_trace.sh TAG
set -o pipefail
TAG=${1:-c5api}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d $OUT/t -o run --output-format csv -- \
  python3 $R/bench.py --model llama-2-13b --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/c5.json 2> $OUT/c5.err || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = glob.glob(out + "/t/**/*hip_api_trace.csv", recursive=True)
c = collections.Counter()
for r in csv.DictReader(open(f[0])):
    n = r.get("Function") or r.get("Function_Name") or r.get("Operation", "")
    if "Memcpy" in n or "Memset" in n or "MemcpyAsync" in n:
        c[n] += 1
print("hip api:", c.most_common(20))
f = glob.glob(out + "/t/**/*memory_copy_trace.csv", recursive=True)
if f:
    c2 = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        c2[(r.get("Direction", "?"), int(r.get("Size", 0) or 0))] += 1
    print("copies (direction, bytes):", c2.most_common(25))
PY
