#!/bin/bash
# Stall/conflict counters of the Gram kernel (separate passes), for kernel tuning.
# usage (on the GPU box, repo root): bash tools/pmc_gram.sh <tag> [dtype]
set -o pipefail
TAG=${1:-x}; DT=${2:-fp16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
    python3 $R/tools/bench_gram.py 262144 4096 $DT > $OUT/p$i.log 2>&1 || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "gram" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[(r["Counter_Name"], r["Dispatch_Id"])] += 1
disp = collections.Counter(k[0] for k in n)
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / disp[k]:.4g}")
PY
