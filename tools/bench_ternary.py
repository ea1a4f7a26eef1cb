"""Ternary inference kernel timing (dev tool): TernaryLinear (2-bit codes, f16 MFMA) vs a dense
fp16 nn.Linear (hipBLASLt) of the same shape.  python tools/bench_ternary.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


res = []
for n, m in ((4096, 4096), (11008, 4096), (4096, 11008)):
    B = m // 128
    lay = pt2q.TernaryLinear(m, n, 128, bias=False, dtype=torch.float16)
    T = torch.randint(-1, 2, (n, m), dtype=torch.int8, device="cuda")
    lay.set_quantized_params(torch.rand(n, B, device="cuda") * 0.05, torch.randn(n, B, device="cuda") * 1e-3,
                             T, torch.randperm(m, device="cuda"))
    dense = torch.nn.Linear(m, n, bias=False, device="cuda", dtype=torch.float16)
    for tokens in (1, 8, 64, 2048):
        x = torch.randn(tokens, m, device="cuda", dtype=torch.float16)
        t_t = timed(lambda: lay(x))
        t_d = timed(lambda: dense(x))
        code_bytes = n * m / 4 + 2 * n * B * 4
        res.append({"n": n, "m": m, "tokens": tokens, "ternary_us": round(t_t, 2),
                    "dense_fp16_us": round(t_d, 2),
                    "ternary_weight_GBps": round(code_bytes / t_t / 1e3, 1),
                    "ternary_TFLOPs": round(2 * n * m * tokens / t_t / 1e6, 1)})
        print(json.dumps(res[-1]), flush=True)
