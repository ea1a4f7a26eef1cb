"""Whole-model timing: ternary-quantise every linear of a Llama-2-7B-shaped model on one MI355X
(BASELINE.json north star: "all linear layers of a 7B-class model ... in under 60 s").

Per decoder layer the activations are synthetic (counter hash, 1 % x20 outlier channels; the
real flow would capture them with calibration.GramCapture) and the linears that share an input
share one Gram and one Cholesky inverse (q/k/v; gate/up), exactly as PT2LLMQuantizer.quantize
does.  Timed: Gram + damping + Cholesky inverse + the block loop of every linear, per layer;
the synthetic fill is timed separately and excluded.

usage: python tools/bench_model.py [--layers 32] [--tokens 262144] [--hidden 4096] [--inter 11008]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--tokens", type=int, default=262144)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=11008)
    ap.add_argument("--block-size", type=int, default=128)
    ap.add_argument("--no-ssr", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    h, f, N, bs = a.hidden, a.inter, a.tokens, a.block_size
    # (group name, input features, [(linear, out features)])
    groups = [("attn_in", h, [("q_proj", h), ("k_proj", h), ("v_proj", h)]),
              ("attn_out", h, [("o_proj", h)]),
              ("mlp_in", h, [("gate_proj", f), ("up_proj", f)]),
              ("mlp_out", f, [("down_proj", h)])]
    gram_ws = {m: torch.empty(pt2q._lib.lib().pt2q_gram_workspace_bytes(m), dtype=torch.uint8, device=dev)
               for m in {g[1] for g in groups}}
    stage = {"gram": 0.0, "hessian_inverse": 0.0, "blocks": 0.0}
    t_fill = 0.0
    t_total = 0.0
    ncols = 0
    spd_all = True
    for layer in range(a.layers):
        for gi, (gname, m, lins) in enumerate(groups):
            t0 = time.perf_counter()
            seed = 10_000 * layer + 100 * gi
            X = pt2q.fill_synthetic((N, m), seed, std=1.0, outliers=True, device=dev).to(torch.float16)
            Ws = [pt2q.fill_synthetic((n, m), seed + 1 + k, std=0.02, device=dev)
                  for k, (_, n) in enumerate(lins)]
            torch.cuda.synchronize()
            t_fill += time.perf_counter() - t0

            t0 = time.perf_counter()
            G = pt2q.gram(X, workspace=gram_ws[m])
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            Hinv, spd = pt2q.hessian_inverse(G, N)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            for W in Ws:
                pt2q.quantize_blocks(W, G, Hinv, bs, not a.no_ssr, pt2q._lib.AGA_ACT)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            stage["gram"] += t1 - t0
            stage["hessian_inverse"] += t2 - t1
            stage["blocks"] += t3 - t2
            t_total += t3 - t0
            ncols += m * len(lins)
            spd_all &= spd
            del X, Ws, G, Hinv
        print(f"layer {layer}: {t_total:.2f} s cumulative", flush=True)
    res = {"model": f"llama-2-7b shapes x{a.layers} layers (h={h}, ffn={f})", "tokens": N,
           "linears": 7 * a.layers, "weight_columns": ncols, "seconds": t_total,
           "cols_per_s": ncols / t_total, "stage_seconds": stage,
           "synthetic_fill_seconds_excluded": t_fill, "all_spd": spd_all,
           "target_seconds": 60.0, "ssr": not a.no_ssr}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
