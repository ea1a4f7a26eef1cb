"""Per-stage timing of one layer (dev tool): python tools/bench_stages.py [n] [m] [N] [fp16|fp32]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
m = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
dt = {"fp16": torch.float16, "fp32": torch.float32}[sys.argv[4] if len(sys.argv) > 4 else "fp16"]
W = pt2q.fill_synthetic((n, m), 1, std=0.02).to(dt)
X = pt2q.fill_synthetic((N, m), 2, outliers=True).to(dt)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        r = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, r


t_gram, G = timed(lambda: pt2q.gram(X))
t_prep, (H, _) = timed(lambda: pt2q.prepare_hessian(G, N))
t_chol, (Hinv, spd) = timed(lambda: pt2q.cholesky_inverse(H))
t_blk, _ = timed(lambda: pt2q.quantize_blocks(W, G, Hinv))
ws = pt2q.LayerWorkspace(n, m, 128, W.device)
t_layer, _ = timed(lambda: pt2q.quantize_layer(W, X, workspace=ws, check_spd=False))
print(f"{n}x{m} N={N} {dt}: gram {t_gram:.2f} ms | prepare {t_prep:.2f} | chol+inv {t_chol:.2f} "
      f"(spd={spd}) | blocks {t_blk:.2f} | fused layer {t_layer:.2f} ms -> {m / t_layer * 1e3:.0f} cols/s")
