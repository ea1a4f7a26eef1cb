#!/bin/bash
# Step times with more HIP hardware queues per process (GPU box): bash tools/hwq_ab.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-hwq}
mkdir -p $OUT
run() {  # label, env, args
  local lab=$1 q=$2; shift 2
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-extra --no-cpu-baseline "$@" > $OUT/out.json 2>$OUT/err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/out.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],3))" "$lab q=$q" >> $OUT/ab.txt
}
for q in 4 8 4 8; do run gpt2 $q --model gpt2 --steps 20; done
for q in 4 8; do run "gpt2-inv2" $q --model gpt2 --steps 20 --inv-streams 2; done
for q in 4 8 4 8; do run c5 $q --model llama-2-13b; done
for q in 4 8; do run c4 $q --steps 3 --warmup 1; done
