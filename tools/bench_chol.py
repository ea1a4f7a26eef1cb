"""Time the Cholesky inverse of a damped Hessian (dev tool): python tools/bench_chol.py [m ...]
HIP events around pt2q_cholesky_inverse on the launch stream; prints ms and TF/s on the m^3
algorithmic flops (potrf m^3/3 + trtri m^3/3 + lauum m^3/3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
L = pt2q._lib
for m in [int(a) for a in sys.argv[1:]] or [4096, 11008]:
    X = pt2q.fill_synthetic((2048, m), 2, outliers=True).half()
    G = pt2q.gram(X)
    H, _ = pt2q.prepare_hessian(G, 2048)
    Hinv = torch.empty_like(H)
    info = torch.zeros(1, dtype=torch.int32, device=H.device)
    ws = L.workspace(L.lib().pt2q_cholesky_workspace_bytes(m), H.device)
    st = L.stream_of(H.device)

    def run():
        L.check(L.lib().pt2q_cholesky_inverse(L.ptr(H), m, m, L.ptr(Hinv), m, L.ptr(ws), ws.numel(),
                                              L.ptr(info), st), "chol")
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    assert int(info.item()) == 0
    print(f"cholesky_inverse m={m}: {ms:.3f} ms  {float(m) ** 3 / ms / 1e9:.1f} TF/s "
          f"(algorithmic m^3; f32 MFMA peak 157.3)", flush=True)
