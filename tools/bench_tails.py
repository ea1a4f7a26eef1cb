"""Diagnostic (not the bench): wall time of the model step's unit TAILS alone (damping, Cholesky
inverse, block loops; Grams precomputed once per width) through engine.UnitPipeline with 1..L
lanes -- how much of the step is tail latency vs tail throughput.
python tools/bench_tails.py [lanes ...]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
from pt2q import sharding  # noqa: E402


def main():
    lanes = [int(x) for x in sys.argv[1:]] or [1, 2, 3]
    dev = torch.device("cuda", 0)
    units = sharding.llama_units(32)
    X, W, G = {}, {}, {}
    for i, (name, lins, N) in enumerate(units):
        m = lins[0][2]
        if m not in X:
            X[m] = pt2q.fill_synthetic((N, m), 2000 + m, std=1.0, outliers=True, device=dev).half()
            G[m] = pt2q.gram(X[m])
        for k, (p, n, _) in enumerate(lins):
            W[(i, p)] = pt2q.fill_synthetic((n, m), 100_000 + 16 * i + k, std=0.02, device=dev).half()
    for L in lanes:
        pipe = pt2q.UnitPipeline(dev, lanes=L)
        for m in X:
            pipe.workspace(m)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            runs = [pipe.run([W[(i, p)] for p, _, _ in lins], X[lins[0][2]], G=G[lins[0][2]])
                    for i, (name, lins, N) in enumerate(units)]
            for r in runs:
                r.finish()
            torch.cuda.synchronize()
            print(f"lanes {L} rep {rep}: tails {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
