set -o pipefail
mkdir -p gpurun_out/r06r
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cholesky or inverse or hess" > gpurun_out/r06r/tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_inverse.py 3072 12 10 > gpurun_out/r06r/inv.txt || exit 1
timeout -k 10 120 python tools/time_inverse.py 768 36 10 >> gpurun_out/r06r/inv.txt || exit 1
timeout -k 10 120 python tools/time_inverse.py 4096 32 3 >> gpurun_out/r06r/inv.txt || exit 1
timeout -k 10 200 python tools/time_inverse.py 11008 32 2 >> gpurun_out/r06r/inv.txt || exit 1
bash tools/c2_ab.sh r06r "" ""
