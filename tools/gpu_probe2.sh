cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for t in 6 1; do PT2Q_GEMM_TILE=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lauum$t -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-n2048 > /dev/null 2>&1 || exit 1; done
