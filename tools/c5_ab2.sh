#!/bin/bash
# C5 step time under bench.py variants (GPU box): bash tools/c5_ab2.sh TAG ["args1" ...]
set -o pipefail
TAG=${1:-c5ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
[ $# -eq 0 ] && set -- ""
for v in "$@"; do
  timeout -k 10 200 python -u bench.py --model llama-2-13b --steps 5 --warmup 2 --no-extra --no-cpu-baseline $v > $OUT/out.json 2>$OUT/err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/out.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],3))" "v=$v" >> $OUT/ab.txt
done
