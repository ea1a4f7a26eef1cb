"""Time the symmetric Gram kernel alone (dev tool): python tools/bench_gram.py [N] [m] [dtype]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
m = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dt = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3] if len(sys.argv) > 3 else "fp16"]
X = pt2q.fill_synthetic((N, m), 5, outliers=True).to(dt)
G = torch.empty((m, m), device="cuda")
pt2q.gram(X, G, check=False)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
e0.record()
for _ in range(reps):
    pt2q.gram(X, G, check=False)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
peak, pname = (157.3, "f32") if dt == torch.float32 else (2500.0, "16-bit")
fl = float(N) * m * (m + 1)
print(f"gram N={N} m={m} {dt} tile={os.environ.get('PT2Q_GEMM_TILE', 'auto')}: {ms:.2f} ms  "
      f"{fl / ms / 1e9:.1f} TFLOP/s ({fl / ms / 1e9 / peak * 100:.1f}% of {pname} MFMA peak)")
