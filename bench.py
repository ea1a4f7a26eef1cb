"""Benchmark: weight-columns quantized/s for the PT²-LLM ternary PTQ layer loop on MI355X.

Workload (BASELINE.json metric "weight-columns quantized/sec (and s/layer) at d=4096"): one
Llama-2-7B q_proj-shaped linear (4096 x 4096, fp16 weights) per GPU per step, calibrated on
N = 262144 activation rows (the reference CLI default 128 samples x 2048 tokens, fp16,
synthetic with 1 % x20 outlier channels), variant M (main.py:102-230): Gram -> damping ->
Cholesky inverse -> 32 blocks of [SSR select -> ATQ init/ITF/AGA -> error feedback].
Arithmetic: the Gram of the fp16 activations runs on the fp16 MFMA (f32 accumulate; the oracle
restates its rounding); everything after it is fp32.  Inputs are resident in HBM
before timing.

N>1 (torchrun, one rank per GPU): every rank quantises its own layer (weak scaling) and the
results (2-bit packed codes, scales, permutation) are gathered to rank 0 over RCCL inside the
timed step.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import pt2q_loader  # noqa: E402

pt2q = pt2q_loader.load()
from pt2q import sharding  # noqa: E402

MI355X_F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md:42 (dense f32 MFMA)
MI355X_F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md:43 (dense fp16/bf16 MFMA, no sparsity)
MI355X_HBM_PEAK_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--m", type=int, default=4096)
    p.add_argument("--tokens", type=int, default=262144)
    p.add_argument("--block-size", type=int, default=128)
    p.add_argument("--io-dtype", choices=["fp16", "fp32", "bf16"], default="fp16")
    p.add_argument("--no-ssr", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--eager", action="store_true", help="launch eagerly instead of hipGraph replay")
    p.add_argument("--cpu-sample-rows", type=int, default=4096)
    p.add_argument("--no-n2048", action="store_true",
                   help="skip the secondary N=2048 timing (profiling: keeps only headline launches)")
    return p.parse_args()


def cpu_baseline(n, m, tokens, sample_rows, block_size, use_ssr):
    """The CPU oracle (oracle/, C + OpenMP, kind "port") on a bounded sample of the same layer:
    Cholesky/inverse and the whole block loop timed in full; the Gram timed on `sample_rows` of
    the `tokens` activation rows and scaled linearly (its work is 2·N·m², exactly linear in N)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    orc.set_threads(threads)
    W = synth.weights(7, n, m)
    X = synth.activations(8, sample_rows, m)
    t0 = time.perf_counter()
    G = orc.gram(X)
    t_gram = time.perf_counter() - t0
    t0 = time.perf_counter()
    H, _ = orc.prepare_hessian(G, sample_rows)
    Hinv, _ = orc.cholesky_inverse(H)
    orc.quantize_blocks(W, G, Hinv, block_size, use_ssr, 1)
    t_rest = time.perf_counter() - t0
    t_layer = t_gram * (tokens / sample_rows) + t_rest
    return {"value": m / t_layer, "unit": "cols/s", "cores": orc.get_threads(), "kind": "port",
            "sample": (f"oracle/pt2q_oracle.c on one {n}x{m} layer: Gram over {sample_rows} of "
                       f"{tokens} rows ({t_gram:.2f}s, scaled x{tokens / sample_rows:.0f}), "
                       f"Cholesky-inverse + {-(-m // block_size)}-block loop in full ({t_rest:.2f}s)"),
            "s_per_layer": t_layer}


def load_traffic():
    path = os.path.join(ROOT, "profiles", "gram_pmc.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    io = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[a.io_dtype]
    n, m, N, bs = a.n, a.m, a.tokens, a.block_size
    use_ssr = not a.no_ssr

    # synthetic, resident inputs (one independent layer per rank)
    W = pt2q.fill_synthetic((n, m), 1000 + rank, std=0.02, device=dev).to(io)
    X = pt2q.fill_synthetic((N, m), 2000 + rank, std=1.0, outliers=True, device=dev).to(io)
    torch.cuda.synchronize()
    ws = pt2q.LayerWorkspace(n, m, bs, dev)
    B = -(-m // bs)
    outs = pt2q.LayerOutput(torch.empty((n, B), device=dev), torch.empty((n, B), device=dev),
                            torch.empty((n, m), dtype=torch.int8, device=dev),
                            torch.empty(m, dtype=torch.int64, device=dev),
                            torch.zeros(B, dtype=torch.int32, device=dev))
    graph = None if a.eager else pt2q.LayerGraph(W, X, bs, use_ssr)

    def step():
        if graph is not None:
            out = graph.replay()
        else:
            out = pt2q.quantize_layer(W, X, bs, use_ssr, workspace=ws, check_spd=False, outputs=outs)
        if world > 1:
            packed, _ = pt2q.pack_ternary(out.T)
            sharding.gather_to_root({"T2": packed, "alpha": out.alpha, "mu": out.mu,
                                     "perm": out.perm}, dst=0)
        return out

    for _ in range(a.warmup):
        out = step()
    torch.cuda.synchronize()
    if a.warmup and int(out.info.item()) != 0:
        raise RuntimeError("synthetic Hessian not SPD")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / max(a.steps, 1)

    # dominant kernel: the symmetric Gram XᵀX (16-bit MFMA for fp16/bf16 X, f32 MFMA for f32 X),
    # timed alone with HIP events on the stream it is launched on (torch's current stream)
    G = torch.empty((m, m), dtype=torch.float32, device=dev)
    reps = 3
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pt2q.gram(X, G)
    ev0.record()
    for _ in range(reps):
        pt2q.gram(X, G)
    ev1.record()
    torch.cuda.synchronize()
    gram_ms = ev0.elapsed_time(ev1) / reps
    gram_flops = float(N) * m * (m + 1)  # unique entries of the symmetric product, 2 flop each
    achieved = gram_flops / (gram_ms * 1e-3) / 1e12

    # secondary: s/layer at N=2048 (the survey's other d=4096 CPU reference point)
    s_layer_2048 = float("nan")
    X2 = X[:2048].contiguous() if not a.no_n2048 else None
    if X2 is not None:
        g2 = pt2q.LayerGraph(W, X2, bs, use_ssr) if not a.eager else None
        run2 = g2.replay if g2 is not None else (
            lambda: pt2q.quantize_layer(W, X2, bs, use_ssr, workspace=ws, check_spd=False, outputs=outs))
        run2()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(5):
            run2()
        torch.cuda.synchronize()
        s_layer_2048 = (time.perf_counter() - t2) / 5

    if a.io_dtype == "fp32":
        kname = "gram_streamk_kernel (symmetric Gram XᵀX, f32 MFMA 32x32x2)"
        peak = MI355X_F32_MFMA_PEAK_TFLOPS
    else:
        kname = ("gram16x_kernel (symmetric Gram XᵀX: LDS-DMA staging, ds_read_b64_tr_b16, "
                 "16-bit MFMA 32x32x16, f32 accumulate)")
        peak = MI355X_F16_MFMA_PEAK_TFLOPS
    if rank == 0:
        res = {
            "metric": "weight-columns quantized/sec (d=4096 linear, 262144 calibration rows)",
            "value": world * a.steps * m / elapsed,
            "unit": "cols/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "s_per_layer": ms_per_step / 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp16->f32" if a.io_dtype != "fp32" else "f32",
            "data": "synthetic (counter-hash weights std 0.02; unit-variance activations, 1% x20 outlier channels)",
            "config": {"workload": f"llama2-7b q_proj {n}x{m}, N={N} (CLI 128x2048), variant M, "
                                   f"{'SSR' if use_ssr else 'sequential'}+ATQ(ITF,AGA), block {bs}",
                       "n": n, "m": m, "tokens": N, "io_dtype": a.io_dtype, "block_size": bs,
                       "parallelism": f"layer-sharded x{world}" + (", rccl gather" if world > 1 else "")},
            "roofline": {"bound": "mfma", "kernel": kname,
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": None,
                         "avg_launch_ms": gram_ms, "flops_per_launch": gram_flops},
            "extra": {"s_per_layer_n2048": None if a.no_n2048 else s_layer_2048,
                      "cols_per_s_n2048": None if a.no_n2048 else m / s_layer_2048,
                      "gram_share_of_step": gram_ms / ms_per_step},
        }
        tr = load_traffic()
        if tr:
            res["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
            res["roofline"]["traffic_source"] = tr.get("source")
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(n, m, N, a.cpu_sample_rows, bs, use_ssr)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
