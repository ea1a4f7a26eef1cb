"""Dev tool: ATQ block-kernel time vs max_iter (run under rocprofv3 --kernel-trace)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
W = pt2q.fill_synthetic((4096, 4096), 1000, std=0.02, device="cuda").to(torch.float16)
X = pt2q.fill_synthetic((8192, 4096), 2000, std=1.0, outliers=True, device="cuda").to(torch.float16)
for it in (int(a) for a in sys.argv[1:]):
    out = pt2q.quantize_layer(W, X, max_iter=it)
    torch.cuda.synchronize()
