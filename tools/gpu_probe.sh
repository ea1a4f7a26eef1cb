set -e
for b in gram16_probe gram16_probe-DGX_PROBE_NO_MFMA gram16_probe-DGX_PROBE_NO_DMA; do
  for m in 4096 11008; do echo "$b m=$m"; timeout -k 10 120 tools/$b.bin 262144 $m 3; done
done
