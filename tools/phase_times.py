"""Phase times of one grams-first 7B step (GPU): Grams, batched Hessian inverses, block loops.
Each phase is bracketed by a device synchronisation (adds a little idle time between phases)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

a = bench.parse(sys.argv[1:] + ["--no-cpu-baseline"])
bench._load_runtime(False)
bench.resolve(a)
torch, sharding = bench.torch, bench.sharding
dev = torch.device("cuda", 0)
io = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[a.io_dtype]
work = bench.ModelStep(a, 0, 1, dev, io)
gf = work.gf
units = work.units
mine = work.mine


def step(timed):
    t = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    inputs = {i: work.provider(units[i]) for i in mine}
    gf.begin([(i, units[i][1][0][2], units[i][2]) for i in mine])
    for i in mine:
        gf.gram(i, inputs[i][0])
    gf.flush()
    torch.cuda.synchronize()
    t["gram"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    gf.inverses()
    torch.cuda.synchronize()
    t["inverse"] = time.perf_counter() - t1
    t2 = time.perf_counter()
    jobs = [(i, [inputs[i][1][p] for p, _, _ in units[i][1]], units[i][2]) for i in mine]
    runs = gf.tails(jobs) if gf.grouped else [gf.tail(i, Ws, N) for i, Ws, N in jobs]
    for r in runs:
        r.finish()
    torch.cuda.synchronize()
    t["tails"] = time.perf_counter() - t2
    gf.check()
    t["total"] = time.perf_counter() - t0
    return t


step(False)
for _ in range(2):
    t = step(True)
    print({k: round(v * 1e3, 1) for k, v in t.items()}, flush=True)
