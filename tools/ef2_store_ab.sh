#!/bin/bash
# ef2_gemm_kernel Wt store cache policy A/B (GPU box): bash tools/ef2_store_ab.sh TAG
set -o pipefail
R=$(pwd)
OUT=gpurun_out/${1:-ef2st}
mkdir -p $OUT tools/_probe
L=$R/snlp---tenary-post-train-quantization_amd
for aux in 0 16 2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -I$R/include \
    -DPT2Q_PROBE=64 -DPT2Q_EF2_STORE_AUX=$aux $R/tools/ef_probe.hip -L$L -lpt2q \
    -Wl,-rpath,'$ORIGIN/../../snlp---tenary-post-train-quantization_amd' -o tools/_probe/ef2st_$aux > $OUT/build_$aux.log 2>&1 &
done
wait
for aux in 0 16 2 0 16 2; do
  echo "aux $aux" >> $OUT/ab.txt
  timeout -k 10 60 tools/_probe/ef2st_$aux 16384 4096 128 30 1 >> $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 60 tools/_probe/ef2st_$aux 4096 4096 128 30 1 >> $OUT/ab.txt 2>&1 || exit 1
done
