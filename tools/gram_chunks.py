"""Drift test (dev tool): time the 16-bit Gram of N = 262144 rows as ONE launch vs as c sequential
launches over contiguous row chunks (accumulate="continue": bit-identical by the contract).  A
launch boundary re-synchronises every workgroup; if shorter launches are faster per row despite
the extra C read-modify-write, k-drift between workgroups costs L2 / MALL reuse."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader
pt2q = pt2q_loader.load()
N = 262144
for m in [int(a) for a in sys.argv[1:]] or [11008, 4096]:
    X = pt2q.fill_synthetic((N, m), 2000 + m, std=1.0, outliers=True).half()
    G = torch.empty((m, m), dtype=torch.float32, device="cuda")
    ws = torch.empty(pt2q._lib.lib().pt2q_gram_workspace_bytes(m), dtype=torch.uint8, device="cuda")
    ref = None
    for chunks in (1, 2, 4, 8, 16, 32, 64):
        rows = N // chunks
        def run():
            pt2q.gram(X[:rows], G, workspace=ws, check=False)
            for c in range(1, chunks):
                pt2q.gram(X[c * rows:(c + 1) * rows], G, accumulate="continue", workspace=ws, check=False)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        if ref is None:
            ref = G.clone()
        same = bool(torch.equal(G, ref))
        print(f"m={m} chunks={chunks:3d} rows={rows:6d}: {ms:7.2f} ms  bit-identical={same}", flush=True)
    del X, G
