set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_now
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-n2048 > $OUT/bench.json 2> $OUT/err || exit 1
cat $OUT/bench.json
