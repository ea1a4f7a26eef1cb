#!/bin/bash
# EF group-0 load position in the grouped 7B block loop, by library builds (GPU box):
#   bash tools/ef2_g0_lib_ab.sh TAG "E1 E2 ..."   (PT2Q_EF2_G0_EARLY values)
set -o pipefail
TAG=$1; ES=$2
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PKG=$R/snlp---tenary-post-train-quantization_amd
for e in $ES; do
  T=$(mktemp -d /tmp/pt2q_e$e.XXXX)
  mkdir -p $T/pkg
  cp -r $PKG/csrc $PKG/Makefile $T/pkg/
  ln -s $R/include $T/include
  sed -i "s/^#define PT2Q_EF2_G0_EARLY [0-9]*$/#define PT2Q_EF2_G0_EARLY $e/" $T/pkg/csrc/ef.hip
  make -s -C $T/pkg -j16 > $OUT/build_$e.log 2>&1 || exit 1
  cp $T/pkg/libpt2q.so $OUT/lib_$e.so
done
cp $PKG/libpt2q.so $OUT/libpt2q_release.so || exit 1
trap 'cp $OUT/libpt2q_release.so $PKG/libpt2q.so' EXIT
export TMPDIR=/tmp
i=0
for rep in 1 2; do
  for e in $ES; do
    cp $OUT/lib_$e.so $PKG/libpt2q.so
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- \
      python3 tools/kern_workloads.py group 4096 4096 16 3 > $OUT/t$i.log 2>&1 || { tail -3 $OUT/t$i.log; exit 1; }
    f=$(find $OUT/t$i -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$e" >> $OUT/ab.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ef2_gemm_kernel" in r["Name"]]
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
calls = sum(int(r["Calls"]) for r in rows)
print(f"early {sys.argv[2]}: ef2 {calls} calls, {tot:.2f} ms, per 16-linear loop {tot / 3:.2f} ms")
PY
    i=$((i+1))
  done
done
cat $OUT/ab.txt
