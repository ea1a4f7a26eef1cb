set -e
for nr in 3968 2048 512; do timeout -k 10 60 tools/ef_probe.bin 4096 $nr 128 20; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu 2>&1 | tail -2
timeout -k 10 300 python bench.py --no-cpu-baseline --no-n2048 | cut -c1-200
