#!/bin/bash
# gemmx check (GPU box): batched inverse timings and the inverse / GEMM parity tests
set -o pipefail
for w in "4096 32" "11008 16"; do
  timeout -k 10 120 python -u tools/time_inverse.py $w 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "inverse or cholesky or hessian or gemm or layer" --timeout 200 --timeout-method thread 2>&1 | tail -2
