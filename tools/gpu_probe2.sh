set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "concurrent" 2>&1 | tail -2
timeout -k 10 300 python -u tools/bench_model.py --layers 4 | tail -1
timeout -k 10 300 python -u tools/bench_model.py --layers 4 --serial | tail -1
