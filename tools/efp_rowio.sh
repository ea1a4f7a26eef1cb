set -o pipefail
mkdir -p gpurun_out/efp2
for m in 64 320 64 320; do timeout -k 10 60 tools/_probe/ef_probe_$m 4096 8192 128 20 1 || exit 1; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/efp2/out.txt
