"""Find the first 8-row group where the device Gram chain leaves the oracle model (dev tool);
dumps (acc, a[8], b[8], hw) cases to gpurun_out/gram16_cases.npz."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import pt2q_loader, synth
from oracle import oracle as orc
pt2q = pt2q_loader.load()
orc.set_threads(16)
cases = []
for (N, m, seed) in [(4000, 2048, 21 + 2048), (16384, 2048, 13 + 2048)]:
    X = synth.activations(seed, N, m)
    Xh = X.astype(np.float16)
    Xd = torch.from_numpy(Xh).cuda()
    G = pt2q.gram(Xd).cpu().numpy()
    R = orc.gram16(Xh)
    bad = (G.view(np.uint32) != R.view(np.uint32))
    ii, jj = np.nonzero(np.triu(bad))
    print(N, m, "bad upper", len(ii), flush=True)
    for i, j in list(zip(ii, jj))[:40]:
        Xs = np.zeros((N, 8), np.float16)
        Xs[:, 0] = Xh[:, i]; Xs[:, 1] = Xh[:, j]
        Xsd = torch.from_numpy(Xs).cuda()
        acc = pt2q.GramAccumulator(8, "cuda")
        prev = 0.0
        for g in range(N // 8):
            acc.add(Xsd[8 * g: 8 * g + 8])
            hw = float(acc.G[0, 1].item())
            a = Xs[8 * g: 8 * g + 8, 0]; b = Xs[8 * g: 8 * g + 8, 1]
            A = np.zeros((1, 32, 16), np.float16); B = np.zeros((1, 16, 32), np.float16)
            C = np.zeros((1, 32, 32), np.float32)
            A[0, 0, :8] = a; B[0, :8, 0] = b; C[0, 0, 0] = prev
            mo = float(orc.mfma16_tiles(A, B, C)[0, 0, 0])
            if np.float32(mo) != np.float32(hw):
                cases.append(np.concatenate([[prev], a.astype(np.float64), b.astype(np.float64), [hw, mo]]))
                print("case", i, j, "group", g, "acc", prev, "hw", hw, "model", mo, flush=True)
                break
            prev = hw
np.save(os.path.join(ROOT, "gpurun_out", "gram16_cases.npy"), np.array(cases))
