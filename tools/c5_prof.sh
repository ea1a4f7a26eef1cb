#!/bin/bash
# Clean per-kernel times of the C5 (per-channel 13B) step: one lane (no concurrent kernels to
# stretch a kernel's trace duration), rocprofv3 kernel trace, for each PT2Q_WIDE_WAVES value.
#   bash tools/c5_prof.sh TAG [waves ...]
set -o pipefail
TAG=${1:-c5}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for W in ${@:-4}; do
  export PT2Q_WIDE_WAVES=$W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w$W -o run --output-format csv -- \
    python3 $R/bench.py --model llama-2-13b --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/w$W.json 2> $OUT/w$W.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/w$W.json'));print('C5 1 lane waves=$W', round(d['ms_per_step'],1))"
  f=$(find $OUT/w$W -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/kstats.py $f > $OUT/w${W}_kstats.txt 2>&1 && head -12 $OUT/w${W}_kstats.txt
  gzip -f $f
done
