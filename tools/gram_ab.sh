#!/bin/bash
# batched-Gram A/B (GPU box) on the DEV library tools/_probe/libpt2q_dev.so (tools/build_dev_lib.sh;
# drop ./tools/_probe from .gpurunignore for the run): average gram16b launch time of
# kern_workloads grams N M COUNT per environment setting.  The release library is put back on exit.
#   bash tools/gram_ab.sh TAG N M COUNT [VAR=VALUE ...]   ("-" = no override)
set -o pipefail
TAG=$1; N=$2; M=$3; CNT=$4; shift 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PKG=$R/snlp---tenary-post-train-quantization_amd
cp $PKG/libpt2q.so $OUT/libpt2q_release.so || exit 1
trap 'cp $OUT/libpt2q_release.so $PKG/libpt2q.so' EXIT
cp $R/tools/_probe/libpt2q_dev.so $PKG/libpt2q.so || exit 1
cd /tmp && export TMPDIR=/tmp
k=0
for E in ${@:--}; do
  k=$((k + 1))
  timeout -k 10 120 env $([ "$E" = - ] || echo $E) rocprofv3 --kernel-trace -d $OUT/c$k -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py grams $N $M $CNT 3 > $OUT/c$k.log 2>&1 || { echo "FAIL $E"; tail -3 $OUT/c$k.log; exit 1; }
  f=$(find $OUT/c$k -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$E" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gram16b" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(f"{sys.argv[2]:28s}: {len(d)} launches, avg {sum(d[1:])/max(1,len(d)-1)/1e3:.3f} ms (first {d[0]/1e3:.3f})")
PY
  rm -rf $OUT/c$k
done
