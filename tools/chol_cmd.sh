set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/bench_chol.py 4096 11008 > gpurun_out/chol_a.txt 2>&1 || exit 1
PT2Q_RANK_UPDATE=0 timeout -k 10 120 python tools/bench_chol.py 4096 11008 > gpurun_out/chol_b.txt 2>&1 || exit 1
PT2Q_CHOL_PAIR=0 timeout -k 10 120 python tools/bench_chol.py 4096 11008 > gpurun_out/chol_c.txt 2>&1 || exit 1
mkdir -p gpurun_out/chol_tr
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/chol_tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_chol.py 11008 > /dev/null 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/kstats.py $(find $GRAFT_REPO_ROOT/gpurun_out/chol_tr -name "run_kernel_trace.csv" | head -1) --after hess_fill > $GRAFT_REPO_ROOT/gpurun_out/chol_tr.txt
