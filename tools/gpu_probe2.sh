cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for it in 1 100; do timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/atqs$it -o run --output-format csv -- python3 $R/tools/atq_split.py $it > /dev/null 2>&1 || exit 1; done
