for i in 1 2; do for b in gram16_probe gram16_probe_old; do echo -n "$b "; timeout -k 10 120 tools/$b.bin 262144 4096 5 | head -1; done; done
