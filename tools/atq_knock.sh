#!/bin/bash
# Block-ATQ knock-outs (GPU box; results garbage): the ATQ kernel time of one grouped 7B loop (16
# fp16 4096 x 4096 linears) per PT2Q_ATQ_PROBE mask, on a DEV_PROBES library copied over the box's
# package library (tools/_probe/libpt2q_dev.so, built with make DEV_PROBES=1).
#   bash tools/atq_knock.sh TAG [mask ...]     masks: 1 no S1 wait, 2 no coefficient WGs, 4 no ITF,
#   8 no code stores, 16 no S1 workgroups, 32 no row gathers (synthetic w), 64 row workgroups idle,
#   128 no error-term stores, 256 no scale stores
set -o pipefail
TAG=${1:-atqk}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
# the DEV_PROBES library stands in for the package's release library for this script only: the
# release copy is saved first and put back on exit, so later runs on the box load the release build
PKG=$R/snlp---tenary-post-train-quantization_amd
cp $PKG/libpt2q.so $OUT/libpt2q_release.so || exit 1
trap 'cp $OUT/libpt2q_release.so $PKG/libpt2q.so' EXIT
cp $R/tools/_probe/libpt2q_dev.so $PKG/libpt2q.so || exit 1
cd /tmp && export TMPDIR=/tmp
for M in ${@:-0 1 2 4 7}; do
  export PT2Q_ATQ_PROBE=$M
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/m$M -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py group 4096 4096 16 2 > $OUT/m$M.log 2>&1 || { echo "FAIL $M"; tail -3 $OUT/m$M.log; exit 1; }
  f=$(find $OUT/m$M -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$M" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "atq_block_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(f"mask {sys.argv[2]:3s}: {len(d)} launches, avg {sum(d)/len(d):.1f} us, total {sum(d)/1e3:.2f} ms")
PY
done
