"""Batched 16-bit Gram timing as the 7B bench runs it (dev tool): every Gram of one input width in
one launch over the resident N x m activation.  python tools/ab_gram.py [N] [reps]
Prints ms per launch and TFLOP/s on the work done (N m (m+1) per Gram) for m = 4096 (96 Grams)
and m = 11008 (32 Grams)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for m, count in ((4096, 96), (11008, 32)):
    X = pt2q.fill_synthetic((N, m), 79, outliers=True).half()
    G = torch.empty(count, m, m, device=X.device)
    pt2q.engine.gram_batched([X] * count, G)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pt2q.engine.gram_batched([X] * count, G)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = float(N) * m * (m + 1) * count
    print(f"m={m} x{count}: {ms:.1f} ms/launch  {fl / ms / 1e9:.0f} TF/s work done", flush=True)
    del X, G
    torch.cuda.empty_cache()
