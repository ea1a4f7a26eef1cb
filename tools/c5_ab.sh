#!/bin/bash
# C5 (per-channel 13B, bf16) one-lane kernel traces: the streamed per-channel ATQ (atq_pc_kernel)
# against the old wide kernel (PT2Q_ATQ_PC=0), then the default 3-lane C5 step.
#   bash tools/c5_ab.sh TAG
set -o pipefail
TAG=${1:-c5ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for PC in 1 0; do
  export PT2Q_ATQ_PC=$PC
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pc$PC -o run --output-format csv -- \
    python3 $R/bench.py --model llama-2-13b --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/pc$PC.json 2> $OUT/pc$PC.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/pc$PC.json'));print('C5 1 lane PT2Q_ATQ_PC=$PC', round(d['ms_per_step'],1))"
  f=$(find $OUT/pc$PC -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/kstats.py $f > $OUT/pc${PC}_kstats.txt 2>&1 && head -8 $OUT/pc${PC}_kstats.txt
  gzip -f $f
done
unset PT2Q_ATQ_PC
cd $R && timeout -k 10 300 python3 bench.py --model llama-2-13b --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_default.json 2> $OUT/c5_default.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/c5_default.json'));print('C5 default', round(d['ms_per_step'],1), json.dumps(d['roofline'].get('stages',{}).get('atq')))"
