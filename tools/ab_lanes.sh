#!/bin/bash
# Tail lanes A/B on the default bench (GPU box)
set -o pipefail
for L in 2 4 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --steps 3 --warmup 1 --lanes $L > gpurun_out/lanes_$L.json 2> gpurun_out/lanes_$L.err || { tail gpurun_out/lanes_$L.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/lanes_$L.json'));print('lanes', $L, d['ms_per_step'], d['roofline']['phase_s'])"
done
