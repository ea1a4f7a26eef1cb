"""Eager quantize_layer vs its hipGraph replay (engine.LayerGraph) on one layer (dev tool):
python tools/graph_ab.py N M TOKENS [reps] -- how much of a small layer's time is launch cost."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
n, m, N = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
W = pt2q.fill_synthetic((n, m), 5, std=0.02, device="cuda")
X = pt2q.fill_synthetic((N, m), 6, outliers=True, device="cuda")
eng = pt2q.engine
ws = eng.LayerWorkspace(n, m, 128, W.device)


def eager():
    return eng.quantize_layer(W, X, 128, True, 0.01, 100, torch.int8, workspace=ws, check_spd=False)


def timeit(f):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


g = eng.LayerGraph(W, X, 128, True)
print(f"n={n} m={m} N={N}: eager {timeit(eager):.3f} ms  graph {timeit(g.replay):.3f} ms", flush=True)
