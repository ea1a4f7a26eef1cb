# One round-end measurement pass (GPU box, repo root): profiles, default bench, 7B model.
set -o pipefail
TAG=${1:-r01g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/profile_round.sh $TAG > gpurun_out/prof_$TAG.log 2>&1 || { echo "profile failed"; exit 1; }
echo "profile ok"
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; exit 1; }
echo "bench ok"
timeout -k 10 400 python -u tools/bench_model.py > gpurun_out/model_$TAG.json 2> gpurun_out/model_$TAG.err || { echo "model failed"; exit 1; }
echo "model ok"
