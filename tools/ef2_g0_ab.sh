#!/bin/bash
# ef2_gemm_kernel: column group 0's old values one stage earlier, A/B (GPU box): bash tools/ef2_g0_ab.sh TAG
set -o pipefail
R=$(pwd)
OUT=gpurun_out/${1:-ef2g0}
mkdir -p $OUT tools/_probe
L=$R/snlp---tenary-post-train-quantization_amd
for e in 0 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -I$R/include \
    -DPT2Q_PROBE=64 -DPT2Q_EF2_G0_EARLY=$e $R/tools/ef_probe.hip -L$L -lpt2q \
    -Wl,-rpath,'$ORIGIN/../../snlp---tenary-post-train-quantization_amd' -o tools/_probe/ef2g0_$e > $OUT/build_$e.log 2>&1 &
done
wait
for e in 0 2 3 0 2 3; do
  echo "early $e" >> $OUT/ab.txt
  timeout -k 10 60 tools/_probe/ef2g0_$e 16384 4096 128 30 1 >> $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 60 tools/_probe/ef2g0_$e 4096 4096 128 30 1 >> $OUT/ab.txt 2>&1 || exit 1
done
