"""Batched Gram time vs CUs held (dev tool, GPU): one launch over COUNT Grams of 4 distinct
N x m fp16 activations, HIP events, for the PT2Q_GRAM_CUS value of this process.
python tools/gram_cus.py m count"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
m, count = int(sys.argv[1]), int(sys.argv[2])
Xs = [pt2q.fill_synthetic((262144, m), 79 + 7919 * k, outliers=True).half() for k in range(4)]
G = torch.empty(count, m, m, device="cuda")
items = [Xs[z % 4] for z in range(count)]
pt2q.engine.gram_batched(items, G)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(2):
    pt2q.engine.gram_batched(items, G)
e1.record()
torch.cuda.synchronize()
print(f"m={m} count={count} cus={os.environ.get('PT2Q_GRAM_CUS', 'all')}: {e0.elapsed_time(e1) / 2:.1f} ms", flush=True)
