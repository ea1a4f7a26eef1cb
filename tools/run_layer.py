"""Run the headline layer eagerly (dev tool for PMC passes, which need eager launches):
python tools/run_layer.py [reps] -- fp16 4096 x 4096, N = 262144 (bench.py's single-layer extra)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
W = pt2q.fill_synthetic((4096, 4096), 1000, std=0.02).half()
X = pt2q.fill_synthetic((262144, 4096), 2000 + 4096, std=1.0, outliers=True).half()
ws = pt2q.LayerWorkspace(4096, 4096, 128, W.device)
for _ in range(reps):
    out = pt2q.quantize_layer(W, X, workspace=ws)
torch.cuda.synchronize()
print("spd", out.spd)
