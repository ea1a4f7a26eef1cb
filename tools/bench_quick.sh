#!/bin/bash
# One default bench line without the CPU leg and the extra configs (GPU box): bash tools/bench_quick.sh TAG
set -o pipefail
TAG=${1:-bq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-configs "${@:2}" > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['phase_s'], r['stages']['step'])"
