set -o pipefail
for P in 128 256 512; do echo "panel $P"; PT2Q_CHOL_PANEL=$P timeout -k 10 100 python tools/bench_chol.py 4096 || exit 1; done
for P in 256 512 1024; do echo "panel $P"; PT2Q_CHOL_PANEL=$P timeout -k 10 100 python tools/bench_chol.py 11008 || exit 1; done
