timeout -k 10 60 tools/topk_probe.bin
