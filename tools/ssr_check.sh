#!/bin/bash
# SSR check (GPU box): SSR / layer parity tests, then the single-lane phase trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "ssr or layer or group or headline" --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 300 bash $R/tools/phase_trace.sh ${1:-ssrc}_phase --lanes 1 > /dev/null 2>&1 || exit 1
grep -A8 "== tails" $R/gpurun_out/${1:-ssrc}_phase/phase_kstats.txt
