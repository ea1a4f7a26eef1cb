timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log; grep -E "^FAILED|^E  " gpurun_out/t.log | head -8
bash tools/gpu_trace.sh | cut -c1-200
