#!/bin/bash
# Batched Gram super-block side A/B (GPU box)
set -o pipefail
for sj in 8 4 6 12 16 8; do
  PT2Q_GRAM_SUPER=$sj timeout -k 10 200 python -u tools/ab_gram.py 262144 2 2>&1 | grep -v amdgpu.ids | sed "s/^/super=$sj /" || exit 1
done
