set -o pipefail
for m in 4096 11008; do
  timeout -k 10 100 python tools/bench_gram.py 262144 $m fp16 || exit 1
  PT2Q_GRAM_WIDE=0 timeout -k 10 100 python tools/bench_gram.py 262144 $m fp16 || exit 1
done
