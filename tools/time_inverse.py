"""Time engine.hessian_inverse_batched on BATCH synthetic Grams of order M (dev tool):
python tools/time_inverse.py M BATCH [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
m, batch = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
X = pt2q.fill_synthetic((4 * m, m), 77, outliers=True).half()
G = pt2q.gram(X).expand(batch, m, m).contiguous()
Hinv, info = pt2q.engine.hessian_inverse_batched(G, 4 * m, chunk=batch)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    Hinv, info = pt2q.engine.hessian_inverse_batched(G, 4 * m, chunk=batch)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"stages={os.environ.get('PT2Q_GEMMX_STAGES', '2')} m={m} x{batch}: {ms:.1f} ms  "
      f"{batch * float(m) ** 3 / ms / 1e9:.1f} TF/s on m^3", flush=True)
