#!/bin/bash
# Kernel-time A/B of two library builds on one box: bash tools/lib_ab.sh TAG OLD_SO KERNEL_SUBSTR -- CMD...
# (the package's release libpt2q.so is saved first and restored on exit)
set -o pipefail
TAG=$1; OLD=$2; KS=$3; shift 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PKG=$R/snlp---tenary-post-train-quantization_amd
cp $PKG/libpt2q.so $OUT/libpt2q_new.so || exit 1
trap 'cp $OUT/libpt2q_new.so $PKG/libpt2q.so' EXIT
export TMPDIR=/tmp; cd $R
i=0
for v in new old new old; do
  if [ $v = new ]; then cp $OUT/libpt2q_new.so $PKG/libpt2q.so; else cp $R/$OLD $PKG/libpt2q.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- "$@" > $OUT/t$i.log 2>&1 || { tail -3 $OUT/t$i.log; exit 1; }
  f=$(find $OUT/t$i -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$KS" "$v" >> $OUT/ab.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Name"]]
for r in rows:
    print(sys.argv[3], r["Name"][:70], r["Calls"], "calls, avg", round(float(r["AverageNs"]) / 1e3, 1), "us, total", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms")
PY
  i=$((i+1))
done
cat $OUT/ab.txt
