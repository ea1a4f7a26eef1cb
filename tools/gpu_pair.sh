set -e
for l in 0 2 6 12; do for m in 11008 8192; do echo -n "lead=$l "; PT2Q_GRAM_LEAD=$l timeout -k 10 120 python tools/bench_gram.py 262144 $m fp16; done; done
