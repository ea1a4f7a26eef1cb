"""Reference torch path vs the C oracle on the same CPU, build container only.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_ref_vs_oracle.py

Times PT2LLMQuantizer.quantize_layer (main.py:102-230, imported from /root/reference -- it never
travels to the GPU box) and oracle.quantize_layer_m (oracle/pt2q_oracle.c, the bench's
cpu_baseline "port") on identical fp32 counter-hash inputs (tests/synth.py), SSR on, block 128,
at 8 and 1 threads, checks that both give the same codes and permutation, and writes the
ratio table to profiles/cpu_ref_vs_oracle.json.  The ratio lets the bench's cpu_baseline (the
oracle on the GPU box's host cores) be read against the reference's own CPU speed."""
import contextlib
import io
import json
import os
import platform
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402
import main as rm  # noqa: E402


def ref_layer(W, X):
    lin = torch.nn.Linear(W.shape[1], W.shape[0], bias=False)
    lin.weight.data = torch.from_numpy(W.copy())
    q = rm.PT2LLMQuantizer(model=None, tokenizer=None, device="cpu", block_size=128, use_ssr=True, percdamp=0.01)
    with contextlib.redirect_stdout(io.StringIO()):
        return q.quantize_layer(lin, "layer", torch.from_numpy(X.copy()))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    orc.build()
    rows = []
    for (n, m, N, threads) in [(1024, 1024, 2048, 8), (1024, 1024, 2048, 1), (2048, 2048, 2048, 8),
                               (2048, 2048, 2048, 1), (4096, 4096, 2048, 8)]:
        W = synth.weights(11, n, m)
        X = synth.activations(12, N, m)
        torch.set_num_threads(threads)
        t0 = time.perf_counter()
        ref = ref_layer(W, X)
        t_ref = time.perf_counter() - t0
        orc.set_threads(threads)
        t0 = time.perf_counter()
        out = orc.quantize_layer_m(W, X)
        t_orc = time.perf_counter() - t0
        T_ref = np.asarray(ref["T"] if isinstance(ref, dict) else ref[2])
        same = None
        if isinstance(ref, dict) and "perm" in ref:
            same = bool(np.array_equal(np.asarray(ref["perm"]), out["perm"]))
        row = {"n": n, "m": m, "N": N, "threads": threads, "reference_s": t_ref, "oracle_s": t_orc,
               "reference_over_oracle": t_ref / t_orc, "perm_equal": same,
               "code_agreement": float(np.mean(T_ref.astype(np.int8) == out["T"].astype(np.int8)))}
        print(row, flush=True)
        rows.append(row)
    res = {"what": "PT2LLMQuantizer.quantize_layer (torch CPU, reference) vs oracle.quantize_layer_m "
                   "(C, the bench cpu_baseline port), fp32, SSR on, block 128, same inputs",
           "cpu_model": cpu_model(), "torch": torch.__version__, "rows": rows}
    with open(os.path.join(ROOT, "profiles", "cpu_ref_vs_oracle.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
