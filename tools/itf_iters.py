"""Dev tool: ITF iterations per block on the bench's synthetic layer (small N)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
W = pt2q.fill_synthetic((4096, 4096), 1000, std=0.02, device="cuda").to(torch.float16)
X = pt2q.fill_synthetic((8192, 4096), 2000, std=1.0, outliers=True, device="cuda").to(torch.float16)
out = pt2q.quantize_layer(W, X)
torch.cuda.synchronize()
print("iters per block:", out.iters.tolist())
