"""Run one n x m layer eagerly (dev tool for per-shape kernel traces):
python tools/run_shape.py n m [N] [reps] -- fp16 W and X, variant M with SSR."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
n, m = int(sys.argv[1]), int(sys.argv[2])
N = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
W = pt2q.fill_synthetic((n, m), 1000, std=0.02).half()
X = pt2q.fill_synthetic((N, m), 2000 + m, std=1.0, outliers=True).half()
ws = pt2q.LayerWorkspace(n, m, 128, W.device)
for _ in range(reps):
    out = pt2q.quantize_layer(W, X, workspace=ws)
torch.cuda.synchronize()
print("spd", out.spd)
