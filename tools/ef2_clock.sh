#!/bin/bash
# ef2_gemm_kernel clock vs knock-outs (GPU box): bash tools/ef2_clock.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-ef2clk}
mkdir -p $OUT
bash tools/build_ef2_clock.sh > $OUT/build.log 2>&1 || exit 1
for k in 0 8 16 24 1 0; do
  timeout -k 10 60 tools/_probe/ef2clk_$k 16384 4096 128 30 1 >> $OUT/clock.txt 2>&1 || exit 1
done
