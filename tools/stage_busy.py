"""Live per-stage busy times of one grams-first step (GPU): ModelStep.stage_busy (the library's
HIP-event brackets, block loops on one lane) after one warm step.
python tools/stage_busy.py [bench.py args]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

a = bench.parse(sys.argv[1:] + ["--no-cpu-baseline"])
bench._load_runtime(False)
bench.resolve(a)
torch = bench.torch
io = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[a.io_dtype]
w = bench.ModelStep(a, 0, 1, torch.device("cuda", 0), io)
w.step()
torch.cuda.synchronize()
b = w.stage_busy()
print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in b.items()}), flush=True)
