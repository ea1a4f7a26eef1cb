#!/bin/bash
# Round-4 checkpoint d (GPU box): EF v1/v2 PMC passes, then 7B step variants (inverse streams /
# chunks) and the C5 step on three lanes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04d
mkdir -p $OUT
bash $R/tools/pmc_ef2.sh r04d_pmc || exit 1
cd $R
i=0
for V in "" "--inv-streams 2 --inv-chunk 11008:16" "--inv-streams 3 --inv-chunk 11008:16"; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra $V > $OUT/v$i.json 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/v$i.json'));print('variant [$V]', round(d['ms_per_step'],1), d['ranks'][0]['step_ms'])"
  i=$((i+1))
done
timeout -k 10 300 python -u bench.py --model llama-2-13b --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print('C5 3 lanes', round(d['ms_per_step'],1))"
