#!/bin/bash
# ef2 two-team A/B (GPU box): the error feedback's total kernel time over one grouped 7B loop
# (16 fp16 4096 x 4096 linears, 3 reps) per configuration, on the DEV library tools/_probe/libpt2q_dev.so (tools/build_dev_lib.sh; drop ./tools/_probe from .gpurunignore for the run)
# (make DEV_PROBES=1; the release library ignores the PT2Q_EF2_* variables).  The release library is
# put back on exit.   bash tools/ef2_teams_ab.sh TAG [cfg ...]   cfg: t1 | t2oN (two teams, offset N)
set -o pipefail
TAG=${1:-ef2t}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PKG=$R/snlp---tenary-post-train-quantization_amd
cp $PKG/libpt2q.so $OUT/libpt2q_release.so || exit 1
trap 'cp $OUT/libpt2q_release.so $PKG/libpt2q.so' EXIT
cp $R/tools/_probe/libpt2q_dev.so $PKG/libpt2q.so || exit 1
cd /tmp && export TMPDIR=/tmp
for C in ${@:-t1 t2o5}; do
  if [ "$C" = t1 ]; then export PT2Q_EF2_TEAMS=1; else export PT2Q_EF2_TEAMS=2 PT2Q_EF2_TEAM_OFFSET=${C#t2o}; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/$C -o run --output-format csv -- \
    python3 $R/tools/kern_workloads.py group ${N:-4096} ${M:-4096} 16 3 > $OUT/$C.log 2>&1 || { echo "FAIL $C"; tail -3 $OUT/$C.log; exit 1; }
  f=$(find $OUT/$C -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$C" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ef2_gemm" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print(f"{sys.argv[2]:6s}: {len(d)} launches, per loop {sum(d)/3e3:.2f} ms")
PY
  rm -rf $OUT/$C
done
