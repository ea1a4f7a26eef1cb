#!/bin/bash
# grouped per-channel ATQ knock-outs (GPU box; results garbage): the pcr launch time of
# kern_workloads pcg 5120 16 per PT2Q_ATQ_PROBE mask (1 no code stores, 2 AGA without S1 loads,
# 4 ITF skipped), on the DEV library (tools/build_dev_lib.sh; drop ./tools/_probe from
# .gpurunignore for the run).  The release library is put back on exit.  bash tools/pc_knock.sh TAG [mask ...]
set -o pipefail
TAG=${1:-pck}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PKG=$R/snlp---tenary-post-train-quantization_amd
cp $PKG/libpt2q.so $OUT/libpt2q_release.so || exit 1
trap 'cp $OUT/libpt2q_release.so $PKG/libpt2q.so' EXIT
cp $R/tools/_probe/libpt2q_dev.so $PKG/libpt2q.so || exit 1
cd /tmp && export TMPDIR=/tmp
for M in ${@:-0 1 2 3 4 7}; do
  export PT2Q_ATQ_PROBE=$M
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/m$M -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py pcg 5120 16 3 > $OUT/m$M.log 2>&1 || { echo "FAIL $M"; tail -3 $OUT/m$M.log; exit 1; }
  f=$(find $OUT/m$M -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$M" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "atq_pcr" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(f"mask {sys.argv[2]:3s}: {len(d)} launches, avg {sum(d)/len(d):.1f} us")
PY
  rm -rf $OUT/m$M
done
