#!/bin/bash
# C5 (per-channel 13B, bf16) one-lane kernel traces per per-channel ATQ variant, then the default
# 3-lane C5 step.   bash tools/c5_ab.sh TAG [variants: regs stream old]
#   regs   = default (m = 5120 rows in registers, 13824 streamed: atq_pcr / atq_pc kernels)
#   stream = PT2Q_ATQ_PC_REGS=0 (every row streamed through the LDS ring)
#   old    = PT2Q_ATQ_PC=0 (atq_wide_block_kernel)
set -o pipefail
TAG=${1:-c5ab}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in ${@:-regs stream old}; do
  case $V in
    regs) export PT2Q_ATQ_PC=1 PT2Q_ATQ_PC_REGS=1;;
    stream) export PT2Q_ATQ_PC=1 PT2Q_ATQ_PC_REGS=0;;
    old) export PT2Q_ATQ_PC=0 PT2Q_ATQ_PC_REGS=0;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$V -o run --output-format csv -- \
    python3 $R/bench.py --model llama-2-13b --lanes 1 --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/$V.json 2> $OUT/$V.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$V.json'));print('C5 1 lane $V', round(d['ms_per_step'],1))"
  f=$(find $OUT/$V -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/kstats.py $f > $OUT/${V}_kstats.txt 2>&1 && head -8 $OUT/${V}_kstats.txt
  gzip -f $f
done
unset PT2Q_ATQ_PC PT2Q_ATQ_PC_REGS
cd $R && timeout -k 10 300 python3 bench.py --model llama-2-13b --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_default.json 2> $OUT/c5_default.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/c5_default.json'));print('C5 default', round(d['ms_per_step'],1), json.dumps(d['roofline'].get('stages',{}).get('atq')))"
