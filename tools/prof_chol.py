"""Run cholesky_inverse a few times (dev tool for rocprofv3 --kernel-trace timelines)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
m = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
X = pt2q.fill_synthetic((2048, m), 2, outliers=True)
G = pt2q.gram(X)
H, _ = pt2q.prepare_hessian(G, 2048)
for _ in range(3):
    pt2q.cholesky_inverse(H)
torch.cuda.synchronize()
