#!/bin/bash
# Batched-inverse times of library variants (tools/_gx/lib_NAME.so, built beforehand) vs the
# release build, alternating on one box:  bash tools/inv_lib_ab.sh TAG NAME...
set -o pipefail
R=$(pwd); PKG=$R/snlp---tenary-post-train-quantization_amd; OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cp $PKG/libpt2q.so $OUT/lib_rel.so || exit 1
trap 'cp $OUT/lib_rel.so $PKG/libpt2q.so' EXIT
for round in 1 2; do
  for v in rel "$@"; do
    if [ $v = rel ]; then cp $OUT/lib_rel.so $PKG/libpt2q.so; else cp $R/tools/_gx/lib_$v.so $PKG/libpt2q.so; fi
    for shp in "11008 16" "4096 32"; do
      r=$(timeout -k 10 120 python -u tools/time_inverse.py $shp 3 2>>$OUT/err) || exit 1
      echo "$v $r" | tee -a $OUT/ab.txt
    done
  done
done
