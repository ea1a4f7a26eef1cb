#!/bin/bash
# Step time of one model workload under bench.py variants (GPU box):
#   bash tools/cfg_ab.sh TAG MODEL STEPS ["args1" ...]
set -o pipefail
TAG=$1; MODEL=$2; STEPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
[ $# -eq 0 ] && set -- ""
for v in "$@"; do
  timeout -k 10 300 python -u bench.py --model $MODEL --steps $STEPS --warmup 2 --no-extra --no-cpu-baseline $v > $OUT/out.json 2>$OUT/err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/out.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],3))" "$MODEL v=$v" >> $OUT/ab.txt
done
