"""Power-sensitivity test (dev tool): the 16-bit Gram on random vs all-zero X of the same shape
(identical memory traffic; the MFMAs switch far less on zeros).  Large gap = clock / power bound."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader
pt2q = pt2q_loader.load()
N = 262144
for m in (11008, 4096):
    for kind in ("random", "zeros", "random"):
        X = (pt2q.fill_synthetic((N, m), 5, outliers=True).half() if kind == "random"
             else torch.zeros((N, m), dtype=torch.float16, device="cuda"))
        G = torch.empty((m, m), dtype=torch.float32, device="cuda")
        ws = torch.empty(pt2q._lib.lib().pt2q_gram_workspace_bytes(m), dtype=torch.uint8, device="cuda")
        for _ in range(3):
            pt2q.gram(X, G, workspace=ws, check=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            pt2q.gram(X, G, workspace=ws, check=False)
        e1.record()
        torch.cuda.synchronize()
        print(f"m={m} {kind:7s}: {e0.elapsed_time(e1) / 10:.2f} ms", flush=True)
        del X, G
