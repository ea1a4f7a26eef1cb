#!/bin/bash
# Diagonal-factor variants (tools/_gx/lib_NAME.so, e.g. built with chol_diag.hpp DG changed): the
# inverse parity tests under each, then batched-inverse and C2 step times alternating with the
# release build:  bash tools/diag_group_ab.sh TAG NAME...
set -o pipefail
R=$(pwd); PKG=$R/snlp---tenary-post-train-quantization_amd; OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cp $PKG/libpt2q.so $OUT/lib_rel.so || exit 1
trap 'cp $OUT/lib_rel.so $PKG/libpt2q.so' EXIT
use() { if [ $1 = rel ]; then cp $OUT/lib_rel.so $PKG/libpt2q.so; else cp $R/tools/_gx/lib_$1.so $PKG/libpt2q.so; fi; }
for v in rel "$@"; do
  use $v
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "cholesky or inverse_batched or breakdown" > $OUT/pytest_$v.txt 2>&1 || { echo "$v parity FAILED"; tail -20 $OUT/pytest_$v.txt; exit 1; }
  echo "$v parity: $(tail -1 $OUT/pytest_$v.txt)" | tee -a $OUT/ab.txt
done
for round in 1 2; do
  for v in rel "$@"; do
    use $v
    for shp in "3072 12" "768 36" "4096 32"; do
      r=$(timeout -k 10 120 python -u tools/time_inverse.py $shp 5 2>>$OUT/err) || exit 1
      echo "$v $r" | tee -a $OUT/ab.txt
    done
    timeout -k 10 300 python -u bench.py --model gpt2 --steps 30 --warmup 2 --no-extra --no-cpu-baseline > $OUT/out.json 2>>$OUT/err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/out.json').read().strip().splitlines()[-1]); print(sys.argv[1], 'C2', round(d['ms_per_step'],2))" "$v" | tee -a $OUT/ab.txt
  done
done
