#!/bin/bash
# ef2_gemm_kernel knock-outs (GPU box): average launch time of the error feedback in one grouped
# block loop (16 fp16 4096 x 4096 linears, kern_workloads group) per PT2Q_EF2_PROBE mask
# (1 = no Wt traffic, 2 = operand DMAs from one hot chunk, 4 = no MFMAs; results garbage), and
# ef_gemm_kernel for reference.   bash tools/ef2_knock.sh TAG [mask ...]
# masks: N (ef2 knock-out N), sN (ef2, stagger N), nV (PT2Q_EF_V2=V, no w-bar)
# The knock-out masks need the development library (bash tools/build_dev_lib.sh builds
# tools/_probe/libpt2q_dev.so; the release build ignores every PT2Q_EF* variable).
set -o pipefail
TAG=${1:-ef2k}; shift
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
for M in v1 ${@:-0 1 2 4 3 7}; do
  # M: a knock-out mask, or sN = no knock-out with PT2Q_EF2_STAGGER=N
  export PT2Q_EF2_STAGGER=0 PT2Q_EF_WBAR=1
  if [ "$M" = v1 ]; then export PT2Q_EF_V2=0 PT2Q_EF2_PROBE=0;
  elif [ "${M:0:1}" = n ]; then export PT2Q_EF_V2=${M:1} PT2Q_EF2_PROBE=0 PT2Q_EF_WBAR=0;
  elif [ "${M:0:1}" = s ]; then export PT2Q_EF_V2=1 PT2Q_EF2_PROBE=0 PT2Q_EF2_STAGGER=${M:1};
  else export PT2Q_EF_V2=1 PT2Q_EF2_PROBE=$M; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/m$M -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py group 4096 4096 16 3 > $OUT/m$M.log 2>&1 || { echo "FAIL $M"; tail -3 $OUT/m$M.log; exit 1; }
  f=$(find $OUT/m$M -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$M" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ef" in r["Kernel_Name"] and "gemm_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(f"mask {sys.argv[2]:3s}: {len(d)} launches, total {sum(d)/1e3:.2f} ms, per step {sum(d)/3e3:.2f} ms")
PY
done
