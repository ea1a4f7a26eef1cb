#!/bin/bash
# Gram timing under the split/grouping knobs (dev tool; run on the GPU box from the repo root)
for ng in 1 2 4 8 16; do
  PT2Q_GRAM_GROUPS=$ng timeout -k 10 120 python tools/bench_gram.py 262144 4096 fp16 2>/dev/null | sed "s/^/groups=$ng /" || exit 1
done
PT2Q_GRAM_GROUPS=8 timeout -k 10 120 python tools/bench_gram.py 262144 11008 fp16 2>/dev/null || exit 1
