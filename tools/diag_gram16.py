"""Diagnose 16-bit Gram mismatches vs the oracle (dev tool)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import pt2q_loader, synth
from oracle import oracle as orc
pt2q = pt2q_loader.load()
orc.set_threads(16)
def cmp(name, G, R):
    G = G.view(np.uint32); R = R.view(np.uint32)
    z = ((G & 0x7FFFFFFF) == 0) & ((R & 0x7FFFFFFF) == 0)
    bad = (G != R) & ~z
    print(name, "mismatches", int(bad.sum()), "of", bad.size, flush=True)
    if bad.any():
        ii, jj = np.nonzero(bad)
        print("  rows", np.unique(ii // 128)[:20], "cols", np.unique(jj // 256)[:20], "first", ii[:5], jj[:5])
        print("  upper?", np.mean(jj >= ii))
for (N, m, splits) in [(1000, 2048, None), (4000, 2048, None), (1000, 2048, (1000,)), (4000, 2048, (1000, 3000)), (20384, 2048, (1000, 3000, 16384))]:
    X = synth.activations(21 + m, N, m)
    Xd = torch.from_numpy(X).cuda().half()
    if splits is None:
        G = pt2q.gram(Xd).cpu().numpy()
        R = orc.gram16(Xd.cpu().numpy())
        cmp(f"store N={N} m={m}", G, R)
    else:
        acc = pt2q.GramAccumulator(m, "cuda"); s = 0
        for k in splits:
            acc.add(Xd[s:s + k]); s += k
        R = orc.gram16(Xd.cpu().numpy())
        cmp(f"continue {splits}", acc.G.cpu().numpy(), R)
