#!/bin/bash
# Step time of a library variant (sources edited by a sed expression) against the release build,
# alternating on one box:  bash tools/variant_ab.sh TAG FILE 'SED-EXPR' MODEL STEPS [bench args]
set -o pipefail
TAG=$1; FILE=$2; EXPR=$3; MODEL=$4; STEPS=$5; shift 5
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PKG=$R/snlp---tenary-post-train-quantization_amd
T=$(mktemp -d /tmp/pt2q_var.XXXX)
mkdir -p $T/pkg
cp -r $PKG/csrc $PKG/Makefile $T/pkg/
ln -s $R/include $T/include
sed -i "$EXPR" $T/pkg/csrc/$FILE
diff -q $PKG/csrc/$FILE $T/pkg/csrc/$FILE > /dev/null && { echo "sed changed nothing"; exit 1; }
make -s -C $T/pkg -j16 > $OUT/build.log 2>&1 || exit 1
cp $T/pkg/libpt2q.so $OUT/lib_var.so
cp $PKG/libpt2q.so $OUT/lib_rel.so || exit 1
trap 'cp $OUT/lib_rel.so $PKG/libpt2q.so' EXIT
for v in rel var rel var; do
  cp $OUT/lib_$v.so $PKG/libpt2q.so
  timeout -k 10 300 python -u bench.py --model $MODEL --steps $STEPS --warmup 1 --no-extra --no-cpu-baseline "$@" > $OUT/out.json 2> $OUT/err || { tail -3 $OUT/err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/out.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],2))" "$v" >> $OUT/ab.txt
done
cat $OUT/ab.txt
