"""Benchmark: weight-columns quantized/s for the PT²-LLM ternary PTQ engine on MI355X.

Default workload (BASELINE.json metric "weight-columns quantized/sec (and s/layer) at d=4096;
1/2/4/8 MI355X", config C4 "Llama-2-7B fp16, full ATQ+SSR pipeline, layers sharded across
8×MI355X via RCCL/xGMI"): one step quantises EVERY linear of a Llama-2-7B-shaped model (32
decoder layers x {q,k,v,o 4096x4096; gate,up 11008x4096; down 4096x11008} = 224 linears,
1,138,688 weight columns), each calibrated on N = 262144 activation rows (the reference CLI
default 128 samples x 2048 tokens), variant M (main.py:102-230 per linear, main.py:257-304 over
the model).  Linears that read the same input (q/k/v, gate/up) form one work unit sharing one
Gram and one Cholesky inverse (128 units).  With N GPUs (torchrun, one rank per GPU) the units
are split longest-processing-time first (sharding.assign_lpt on a measured-time cost model) — the
total work is fixed, so the scaling is STRONG — and every rank's results (2-bit packed codes, scales, permutation) are
gathered to rank 0 over RCCL inside the timed step.  Per rank, every Gram of its units runs first
(one raw-Gram buffer per unit), then the units' tails on three stream lanes (sharding.GramsFirst;
`--schedule interleaved` puts each Gram on its lane before its tail instead).

Data: synthetic, resident in HBM before timing (fp16 weights, counter-hash, std 0.02; fp16
activations, unit variance with 1 % x20 outlier channels).  One activation tensor per input
width is shared by the units of that width on a rank; every unit still computes its own Gram.

`extra` carries the single-layer numbers (s/layer and cols/s of the 4096x4096 q_proj layer at
N = 262144 and N = 2048, one hipGraph replay each).  `--workload layer` times that single layer
per rank instead (weak scaling, the round-1 bench line).  `--workload split --n 4096 --m 11008`
times ONE layer whose Gram is split over the ranks' calibration rows (strong scaling, SURVEY
§8e(ii): sharding.quantize_layer_split — partial Grams, rank-ordered fold on rank 0, the rest of
the layer there).

Ranks: `python bench.py --gpus N` with no WORLD_SIZE in the environment starts the N ranks itself
(a `torch.distributed.run` child with one process per GPU, launched before this process imports
torch or touches the GPU; this process exits with the child's code).  Under an external launcher
(torchrun / `python -m torch.distributed.run ... bench.py --gpus N`) the flag must equal
WORLD_SIZE, else the run is refused; `n_gpus` in the line is `dist.get_world_size()`.
`--dry-run` exercises the same multi-rank plumbing on CPU (gloo, stub units, no libpt2q) for tests.
"""
import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Filled by _load_runtime() AFTER the launcher decision (no torch / HIP in a launching parent).
np = torch = dist = pt2q = sharding = None

MI355X_F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md (dense f32 MFMA)
MI355X_F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md (dense fp16/bf16 MFMA, no sparsity)
MI355X_HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md (HBM3E)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py starts "
                        "them itself; default: WORLD_SIZE or 1")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU plumbing check: gloo ranks, stub units (no GPU, no libpt2q)")
    p.add_argument("--share-gpu", action="store_true",
                   help="TESTING ONLY: every rank on cuda:0 with the gloo backend (the real kernels and the "
                        "sharded step's gather on a one-GPU box; not a scaling measurement)")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", choices=["model", "layer", "split", "decoder"], default="model",
                   help="model: LPT-sharded 7B step; layer: one layer per rank (weak); split: one n x m "
                        "layer, its Gram data-parallel over the ranks (strong)")
    p.add_argument("--model", choices=["llama-2-7b", "gpt2", "opt-1.3b", "llama-2-13b"], default="llama-2-7b",
                   help="model workload: the BASELINE config whose linears one step quantises (C4 default; "
                        "C2 gpt2, C3 opt-1.3b, C5 llama-2-13b) -- sets the defaults of --layers, --tokens, "
                        "--block-size and --io-dtype (sharding.MODELS)")
    p.add_argument("--layers", type=int, default=None, help="decoder layers of the model workload")
    p.add_argument("--hidden", type=int, default=None, help="llama models: override the hidden width")
    p.add_argument("--inter", type=int, default=None, help="llama models: override the MLP width")
    p.add_argument("--n", type=int, default=4096, help="layer workload: d_out")
    p.add_argument("--m", type=int, default=4096, help="layer workload: d_in")
    p.add_argument("--tokens", type=int, default=None, help="calibration rows N (default: the model's)")
    p.add_argument("--block-size", type=int, default=None)
    p.add_argument("--io-dtype", choices=["fp16", "fp32", "bf16"], default=None)
    p.add_argument("--no-ssr", action="store_true")
    p.add_argument("--lanes", type=int, default=3, help="model workload: UnitPipeline lanes")
    p.add_argument("--schedule", choices=["grams-first", "interleaved"], default="grams-first",
                   help="model workload: every Gram of the step first, then the tails on the lanes "
                        "(sharding.GramsFirst), or each unit's Gram on its lane before its tail")
    p.add_argument("--no-overlap", action="store_true",
                   help="model workload: run the units strictly one after another on one stream "
                        "(default: engine.UnitPipeline overlaps unit i+1's Gram with unit i's tail)")
    p.add_argument("--no-batched-inverse", action="store_true",
                   help="model workload, grams-first: each unit's Cholesky inverse on its lane instead of "
                        "batched per width (engine.hessian_inverse_batched)")
    p.add_argument("--no-batched-grams", action="store_true",
                   help="model workload, grams-first: one stream-K Gram launch per unit instead of one "
                        "data-parallel launch per width (pt2q_gram_batched)")
    p.add_argument("--inverse-overlap", action="store_true",
                   help="model workload: each width's block loops start once its own batched inverses "
                        "are done, beside the other widths' inverses (default: all inverses first)")
    p.add_argument("--inv-streams", type=int, default=1,
                   help="model workload, grams-first: streams the batched inverse chunks spread over "
                        "(sharding.GramsFirst inv_streams)")
    p.add_argument("--inv-chunk", type=str, default="auto",
                   help="model workload, grams-first: items per batched-inverse launch sequence, auto, N "
                        "or m:N,m:N (sharding.GramsFirst chunk)")
    p.add_argument("--group-max", action="store_true",
                   help="model workload, grams-first: shape classes cut into groups of --group linears "
                        "instead of spread over the lanes (sharding.GramsFirst spread=False)")
    p.add_argument("--group", type=int, default=16,
                   help="model workload, grams-first: same-shape linears per grouped block-loop launch "
                        "sequence (pt2q_quantize_blocks_group; 1 = per-unit loops)")
    p.add_argument("--shard", default=None,
                   help="model workload, ONE GPU: time rank r's LPT shard of a --gpus N step alone (r or 'all': "
                        "every rank's shard in turn, after the whole step on this GPU), without the gather "
                        "(its bytes are reported) -- a one-GPU projection of the N-GPU step, not a scaling "
                        "measurement")
    p.add_argument("--no-shards", action="store_true",
                   help="skip extra.shards8 (every rank's shard of an 8-GPU step timed alone on this GPU)")
    p.add_argument("--no-decoder", action="store_true",
                   help="skip extra.decoder (the layer-by-layer PT2LLMQuantizer.quantize flow, Llama-2-7B shapes)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the single-layer / Gram / per-config extras (profiling: keeps only the "
                        "step's launches)")
    p.add_argument("--no-configs", action="store_true",
                   help="skip extra.configs (one short run of each other BASELINE config)")
    p.add_argument("--no-h2d", action="store_true",
                   help="skip extra.h2d (the transfer-inclusive step: inputs from pinned host memory, "
                        "packed results back to the host)")
    return p.parse_args(argv)


def parse_chunk(v):
    """--inv-chunk: "auto" -> None (GramsFirst: 32, or one chunk for a small batch); "32" -> 32;
    "11008:16,4096:32" -> {11008: 16, 4096: 32}."""
    if v == "auto":
        return None
    if ":" not in v:
        return int(v)
    return {int(k): int(c) for k, c in (x.split(":") for x in v.split(","))}


def resolve(a):
    """Fill the model-dependent defaults from sharding.MODELS (after _load_runtime)."""
    c = sharding.MODELS[a.model]
    hidden = c["units"](1, 1)[0][1][0][2]  # the first unit's input width
    a.layers = c["layers"] if a.layers is None else a.layers
    a.tokens = c["tokens"] if a.tokens is None else a.tokens
    a.block_size = c["block_size"] if a.block_size is None else a.block_size
    a.io_dtype = c["io"] if a.io_dtype is None else a.io_dtype
    a.hidden_given = a.hidden is not None or a.inter is not None
    a.hidden = hidden if a.hidden is None else a.hidden
    a.inter = 11008 if a.inter is None else a.inter
    return a


def describe_units(units, layers):
    """'L layers x (q_proj,k_proj,v_proj,o_proj 4096x4096; ...) = K linears in U shared-input units'."""
    per = units[:len(units) // max(layers, 1)]
    shapes = {}
    for _, lins, _ in per:
        for p, n, m in lins:
            shapes.setdefault((n, m), []).append(p)
    body = "; ".join(f"{','.join(ps)} {n}x{m}" for (n, m), ps in shapes.items())
    return (f"{layers} layers x ({body}) = {sum(len(l) for _, l, _ in units)} linears in {len(units)} "
            f"shared-input units")


class no_gc:
    """Timed loops run with Python's cyclic garbage collector off (collected just before, as
    timeit does): a collection landing inside a 16 ms step (C2) once took 68 ms and moved the
    mean 20 %.  The GPU work is unchanged; the collector runs again right after the loop."""

    def __enter__(self):
        gc.collect()
        self.was = gc.isenabled()
        gc.disable()
        return self

    def __exit__(self, *exc):
        if self.was:
            gc.enable()
        return False


def config_runs(a, dev):
    """extra.configs: one short grams-first run (2 warmup + 3 timed steps -- up to 20 for a step
    under 0.1 s -- same flags) of every
    other BASELINE config's model workload on this GPU (C2 gpt2, C3 opt-1.3b, C5 llama-2-13b, or
    C4 when another model is the headline).  Two warmup steps: the second step of a fresh
    workload can still grow the caching allocator's pools (a C5 step once took 991 ms instead of
    ~120 ms right after a single warmup step)."""
    out = {}
    for name in sharding.MODELS:
        if name == a.model:
            continue
        b = resolve(parse(["--model", name, "--steps", "3", "--warmup", "2", "--group", str(a.group),
                           "--lanes", str(a.lanes), "--inv-streams", str(a.inv_streams)]))
        io = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[b.io_dtype]
        try:
            tw = time.perf_counter()
            w = ModelStep(b, 0, 1, dev, io)
            for _ in range(b.warmup):
                tws = time.perf_counter()
                w.step()
                torch.cuda.synchronize()
            # a short step (C2: ~16 ms) is timed over more steps (about 0.3 s, at most 20): the same
            # work per step, less noise in the mean
            b.steps = max(b.steps, min(20, int(0.3 / max(time.perf_counter() - tws, 1e-3))))
            with no_gc():
                t0 = time.perf_counter()
                step_ms = []
                for _ in range(b.steps):
                    ts = time.perf_counter()
                    w.step()
                    torch.cuda.synchronize()
                    step_ms.append(1e3 * (time.perf_counter() - ts))
                s = (time.perf_counter() - t0) / b.steps
            log(0, f"config {name}: setup + warmup {t0 - tw:.1f}s, steps {[round(x, 1) for x in step_ms]} ms")
            cols = sharding.units_cols(w.units)
            # live roofline of this config: phase walls + one-lane stage busy times (outside the timing)
            ph = w.phase_step()
            busy = w.stage_busy()
            peak = MI355X_F32_MFMA_PEAK_TFLOPS if b.io_dtype == "fp32" else MI355X_F16_MFMA_PEAK_TFLOPS
            st = stage_roofline(model_work(w.units, b.block_size, IO_BYTES[b.io_dtype], not b.no_ssr), ph, busy,
                                s * 1e3, 1, peak)
            del w
            gc.collect()
            torch.cuda.empty_cache()
            sh8 = None
            if name == "llama-2-13b" and not a.no_shards:  # C5 is an 8-GPU config too
                try:
                    sh8 = shard_runs(b, dev, io, 8, t1_ms=s * 1e3, t1_phase=ph)
                except Exception as e:
                    sh8 = {"error": f"{type(e).__name__}: {e}"}
            out[name] = {"config": sharding.MODELS[name]["config"], "workload": describe_units(sharding.model_units(name), b.layers),
                         "tokens": b.tokens, "block_size": b.block_size if b.block_size < (1 << 14) else "m (per-channel)",
                         "io_dtype": b.io_dtype, "weight_columns_per_step": cols, "ms_per_step": s * 1e3,
                         "cols_per_s": cols / s, "s_per_decoder_layer": s / b.layers,
                         "steps": b.steps, "warmup": b.warmup,
                         "roofline": {"dominant": st["dominant"], "floor_s": st["step"]["floor_s"],
                                      "frac_step": st["step"]["frac"], "phase_s": ph, "stages": st}}
            if sh8 is not None:
                out[name]["shards8"] = sh8
        except Exception as e:  # a config that fails is reported, not allowed to drop the line
            out[name] = {"config": sharding.MODELS[name]["config"], "error": f"{type(e).__name__}: {e}"}
        gc.collect()
        torch.cuda.empty_cache()
    return out


def shard_runs(a, dev, io, world, ranks=None, t1_ms=None, t1_phase=None, steps=3, warmup=2):
    """Every rank's LPT shard of a `world`-rank model step, timed ALONE on this one GPU (no process
    group, no gather: each shard reports the bytes its gather would send).  A shard's time is what
    its rank computes in the N-GPU step; the step itself would also wait for the gather and for
    the slowest rank.  projected_efficiency = T1 / (world x max_r T_r) with T1 the whole step on
    this GPU -- a one-GPU PROJECTION of the strong-scaling efficiency, not a measurement of it
    (the RCCL transport and the shared power / fabric of a full node are not in it).  Per phase,
    `share_ratio` = the slowest shard's phase wall / (T1's phase wall / world): the phases whose
    fixed latencies do not shrink with the shard (the batched inverse's serial panel chain, the
    per-block launch chain of the grouped loops) show up there."""
    ranks = list(range(world)) if ranks is None else list(ranks)
    out = []
    for r in ranks:
        w = ModelStep(a, r, world, dev, io, shard_only=True)
        for _ in range(warmup):
            w.step()
        torch.cuda.synchronize()
        step_ms = []
        with no_gc():
            for _ in range(steps):
                ts = time.perf_counter()
                w.step()
                torch.cuda.synchronize()
                step_ms.append(1e3 * (time.perf_counter() - ts))
        ph = w.phase_step() if w.gf is not None and a.schedule == "grams-first" else None
        units = [w.units[i] for i in w.mine]
        rec = {"rank": r, "units": len(units), "linears": sum(len(u[1]) for u in units),
               "cols": sharding.units_cols(units), "ms_per_step": float(np.median(step_ms)),
               "step_ms": {"min": min(step_ms), "median": float(np.median(step_ms)), "max": max(step_ms)},
               "phase_s": ph, "gather_send_bytes": w.gather_bytes,
               "predicted_cost_s": sum(sharding.unit_cost(u, a.block_size) for u in units),
               "predicted_shard_s": sharding.shard_cost(units, a.block_size, IO_BYTES[a.io_dtype]),
               "predicted_phase_s": sharding.shard_phases(units, a.block_size, IO_BYTES[a.io_dtype])}
        log(0, f"shard {r}/{world}: {len(units)} units, {rec['ms_per_step']:.1f} ms/step, phases "
               f"{ {k: round(v * 1e3, 1) for k, v in (ph or {}).items()} }")
        out.append(rec)
        del w
        gc.collect()
        torch.cuda.empty_cache()
    res = {"world": world, "shards": out, "steps": steps, "warmup": warmup,
           "what": "each rank's LPT shard of a world-rank step timed alone on ONE MI355X (no gather); a projection"}
    if len(out) == world:
        mx = max(x["ms_per_step"] for x in out)
        res["max_shard_ms"] = mx
        res["max_over_mean"] = mx / (sum(x["ms_per_step"] for x in out) / world)
        res["gather_bytes_to_rank0"] = sum(x["gather_send_bytes"] for x in out)
        pred = [x["predicted_shard_s"] * 1e3 for x in out]
        res["predicted_vs_measured"] = {"max_abs_rel_err": max(abs(p - x["ms_per_step"]) / x["ms_per_step"]
                                                               for p, x in zip(pred, out)),
                                        "predicted_max_over_mean": max(pred) / (sum(pred) / world),
                                        "model": "sharding.shard_cost (phase model fitted to one-GPU shard timings)"}
        if t1_ms:
            res["t1_ms"] = t1_ms
            res["projected_efficiency"] = t1_ms / (world * mx)
            res["projected_value_cols_per_s"] = sharding.units_cols(model_units(a)) / (mx * 1e-3)
        if t1_phase and all(x["phase_s"] for x in out):
            res["t1_phase_s"] = t1_phase
            res["share_ratio"] = {k: max(x["phase_s"][k] for x in out) / (t1_phase[k] / world)
                                  for k in t1_phase if t1_phase[k] > 0}
    return res


def decoder_run(a, dev, layers=None, samples=128, seq=2048):
    """extra.decoder / --workload decoder: the REAL calibration flow of a PT2LLMQuantizer.quantize
    user (main.py:232-308) on a Llama-2-7B-shaped model, one decoder layer after another: a
    random-init fp16 transformers LlamaForCausalLM (hidden 4096, MLP 11008, 32 heads; no
    checkpoint exists offline), `samples` calibration sequences of `seq` random token ids
    (N = samples x seq = 262144 rows per linear), per layer: the layer's forward over every sample
    with the capture hooks streaming each linear's input into its Gram (4 Grams: q/k/v, o,
    gate/up, down), the layer's batched inverses and grouped block loops (GramsFirst), the
    reference's write-back, the layer's forward again on the written-back weights (the next
    layer's inputs: propagate="layerwise"), the results copied to the host as the reference
    returns them.  Only the 7 linears of one layer are independent here (layer L+1's activations
    depend on layer L's write-back), unlike the headline step's 128 batched units."""
    from transformers import LlamaConfig, LlamaForCausalLM
    L = a.layers if layers is None else layers
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=11008, num_hidden_layers=L, num_attention_heads=32,
                      num_key_value_heads=32, vocab_size=32000, max_position_embeddings=4096)
    cfg._attn_implementation = "sdpa"
    t0 = time.perf_counter()
    torch.manual_seed(0)
    with torch.device(dev):
        model = LlamaForCausalLM(cfg).to(torch.float16)
    model.eval()
    g = torch.Generator(device="cpu").manual_seed(1)
    toks = [torch.randint(0, cfg.vocab_size, (1, seq), generator=g).to(dev) for _ in range(samples)]
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    q = pt2q.PT2LLMQuantizer(model, None, "llama", block_size=a.block_size, use_ssr=not a.no_ssr,
                             device=str(dev))
    timings = []
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = q.quantize(toks, writeback="reference", propagate="layerwise", timings=timings)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t1
    cols = sum(v["T"].shape[1] for v in res.values())
    steady = timings[1:] if len(timings) > 1 else timings
    per = {k: float(np.mean([t[k] for t in steady])) for k in steady[0] if k != "layer"}
    out = {"what": "PT2LLMQuantizer.quantize(propagate='layerwise', writeback='reference'): the real per-decoder-layer "
                   "flow (capture forwards + streamed Grams -> batched inverses + grouped loops -> write-back -> "
                   "forward on the written-back layer -> results to host)",
           "model": f"random-init fp16 LlamaForCausalLM, {L} layers x (q,k,v,o 4096x4096; gate,up 11008x4096; down 4096x11008)",
           "calibration": f"{samples} x {seq} random token ids (N = {samples * seq} rows per linear)",
           "layers": L, "linears": len(res), "weight_columns": cols, "total_s": tot,
           "cols_per_s": cols / tot, "s_per_decoder_layer": tot / L,
           "s_per_decoder_layer_steady": per["total_s"], "phase_s_per_layer_steady": per,
           "first_layer_s": timings[0]["total_s"], "setup_s": t_setup,
           "projected_32_layers_s": per["total_s"] * 31 + timings[0]["total_s"] if L < 32 else tot}
    del q, model, res, toks
    gc.collect()
    torch.cuda.empty_cache()
    return out


def model_units(a):
    """The model workload's units: sharding.MODELS[a.model], or llama shapes with --hidden/--inter."""
    if a.hidden_given and a.model.startswith("llama"):
        return sharding.llama_units(a.layers, a.hidden, a.inter, a.tokens)
    return sharding.model_units(a.model, a.layers, a.tokens)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_or_check(a, argv):
    """Rank plumbing, decided before torch is imported.  Returns None to run in this process, or
    the exit code of the rank launcher this process started (the caller exits with it).

    * WORLD_SIZE unset and --gpus N > 1: start `python -m torch.distributed.run` with N processes
      on 127.0.0.1 as a CHILD process (this process has not touched the GPU and never execs).
    * WORLD_SIZE set (torchrun / the driver's launcher): --gpus, when given, must equal it."""
    env_world = os.environ.get("WORLD_SIZE")
    if a.shard is not None:  # one process on one GPU times the shards of a --gpus N step
        if env_world is not None and int(env_world) > 1:
            print("[bench] refusing: --shard runs in ONE process (no launcher)", file=sys.stderr)
            return 2
        return None
    if env_world is not None:
        if a.gpus is not None and a.gpus != int(env_world):
            print(f"[bench] refusing: --gpus {a.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
            return 2
        return None
    if a.gpus is None or a.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    print(f"[bench] starting {a.gpus} ranks: {' '.join(cmd[1:5])} ...", file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "16")
    return subprocess.call(cmd, env=env)


def _load_runtime(dry):
    """Heavy imports, after the launcher decision.  --dry-run loads sharding.py alone (no
    libpt2q, no HIP)."""
    global np, torch, dist, pt2q, sharding
    import numpy
    import torch as _torch
    import torch.distributed as _dist
    np, torch, dist = numpy, _torch, _dist
    if dry:
        import importlib.util
        path = os.path.join(ROOT, "snlp---tenary-post-train-quantization_amd", "sharding.py")
        spec = importlib.util.spec_from_file_location("pt2q_sharding_dry", path)
        sharding = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(sharding)
        return
    import pt2q_loader
    pt2q = pt2q_loader.load()
    from pt2q import sharding as _sh
    sharding = _sh


def log(rank, msg):
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota if one is
    set (a GPU box's share of a large host).  Returns (cores, how it was found)."""
    aff = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
            if quota < aff:
                return quota, f"cgroup cpu.max quota {quota} of {aff} in the affinity mask"
    except (OSError, ValueError):
        pass
    return aff, f"sched_getaffinity: {aff} CPUs"


# ------------------------------------------------------------------ CPU baseline (oracle, "port")

def cpu_baseline(units, N, block_size, use_ssr, hidden):
    """The CPU oracle (oracle/pt2q_oracle.c, plain C + OpenMP, kind "port") timed on bounded
    samples of the d x d layer and scaled to the workload by each stage's exact work law (Gram
    ∝ N·m², Cholesky inverse ∝ m³, block loop ∝ n·m² at a fixed block size — SSR, ATQ and the
    error feedback are all row-local): on all host cores, and on one core with smaller samples."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    from oracle import oracle as orc
    d = hidden
    cores, cores_how = host_cores()
    cols = sharding.units_cols(units)

    def scaled(tg, rows, tc, cm, tb, brow):
        tot = 0.0
        for _, lins, Nu in units:
            m = lins[0][2]
            tot += tg * (Nu / rows) * (m / d) ** 2 + tc * (m / cm) ** 3
            tot += sum(tb * (n / brow) * (m / d) ** 2 for _, n, _ in lins)
        return tot, tg * (N / rows) + tc * (d / cm) ** 3 + tb * (d / brow)

    def timed(threads, fn, reps=2):
        # best of `reps` runs: the host is shared, a single sub-second sample drifts run to run
        orc.set_threads(threads)
        dt = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            dt = min(dt, time.perf_counter() - t0)
        orc.set_threads(cores)
        return r, dt

    # all cores: Gram over 8192 rows, the full Cholesky inverse, the full block loop (best of 2)
    rows = 8192
    X = synth.activations(8, rows, d)
    W = synth.weights(7, d, d)
    G, tg = timed(cores, lambda: orc.gram(X))
    H, _ = orc.prepare_hessian(G, rows)
    (Hinv, _), tc = timed(cores, lambda: orc.cholesky_inverse(H))
    _, tb = timed(cores, lambda: orc.quantize_blocks(W, G, Hinv, block_size, use_ssr, 1))
    tot, layer = scaled(tg, rows, tc, d, tb, d)
    res = {"value": cols / tot, "unit": "cols/s", "cores": cores, "kind": "port",
           "sample": (f"oracle/pt2q_oracle.c, {cores} threads, on the {d}x{d} layer, best of 2 runs each: "
                      f"Gram over {rows} of {N} rows ({tg:.2f}s), Cholesky inverse ({tc:.2f}s), "
                      f"{-(-d // block_size)}-block loop in full ({tb:.2f}s); the workload's "
                      f"{len(units)} units = these stages scaled by N*m^2, m^3, n*m^2"),
           "s_per_layer": layer, "s_workload": tot, "cpu_model": cpu_model_name(),
           "cores_source": cores_how}
    # one core: smaller samples of the same stages
    rows1, cm1, br1 = 128, 2048, 256
    _, tg1 = timed(1, lambda: orc.gram(X[:rows1]))
    Hs = np.ascontiguousarray(H[:cm1, :cm1])  # a leading principal block of an SPD matrix is SPD
    _, tc1 = timed(1, lambda: orc.cholesky_inverse(Hs))
    _, tb1 = timed(1, lambda: orc.quantize_blocks(W[:br1], G, Hinv, block_size, use_ssr, 1))
    tot1, layer1 = scaled(tg1, rows1, tc1, cm1, tb1, br1)
    res["one_core"] = {"value": cols / tot1, "unit": "cols/s", "cores": 1, "kind": "port",
                       "s_per_layer": layer1, "s_workload": tot1,
                       "sample": (f"1 thread: Gram over {rows1} rows ({tg1:.2f}s), Cholesky inverse "
                                  f"of order {cm1} ({tc1:.2f}s, x(m/{cm1})^3), block loop on {br1} "
                                  f"of {d} rows ({tb1:.2f}s, x n/{br1}); same work-law scaling")}
    # The reference's own CPU path is faster than this port: its Gram and Cholesky are torch /
    # MKL calls (main.py:128, 136-139), and its block loop ran in 0.47-0.61x the port's time on
    # identical layers (profiles/cpu_ref_vs_oracle.json, build container).  So a GPU / port ratio
    # overstates GPU / reference: estimate the reference on this host from the same torch ops,
    # timed live on the same samples, and the measured block-loop ratio.
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_ref_vs_oracle.json")) as f:
            rows_ref = json.load(f)["rows"]
        r44 = [r for r in rows_ref if r["m"] == 4096 and r["threads"] == 8]
        ratio = float(r44[0]["reference_over_oracle"]) if r44 else None
    except (OSError, KeyError, ValueError):
        ratio = None
    if ratio is not None:
        torch.set_num_threads(cores)
        Xt, Ht = torch.from_numpy(X), torch.from_numpy(H)

        def tbest(fn):
            dt = float("inf")
            for _ in range(2):
                t0 = time.perf_counter()
                fn()
                dt = min(dt, time.perf_counter() - t0)
            return dt
        tgt = tbest(lambda: Xt.T @ Xt)
        tct = tbest(lambda: torch.cholesky_inverse(torch.linalg.cholesky(Ht)))
        tot_t, _ = scaled(tgt, rows, tct, d, tb * ratio, d)
        res["torch_ref_over_port"] = ratio
        res["reference_estimate"] = {
            "value": cols / tot_t, "unit": "cols/s", "cores": cores, "s_workload": tot_t,
            "how": (f"the reference's CPU ops timed live with torch on {cores} threads: X.T @ X over {rows} rows "
                    f"({tgt:.3f}s, main.py:128), cholesky + cholesky_inverse at {d} ({tct:.3f}s, main.py:136-139); "
                    f"the block loop = the port's x {ratio:.3f} (reference / port time on a {d}x{d} layer, "
                    "profiles/cpu_ref_vs_oracle.json); same work-law scaling")}
    return res


# ------------------------------------------------------------------ helpers

def gram_time_ms(X, m, reps=3):
    """Average launch time of the symmetric Gram on X, HIP events on the launch stream (torch's
    current stream, which pt2q_gram uses)."""
    G = torch.empty((m, m), dtype=torch.float32, device=X.device)
    ws = torch.empty(pt2q._lib.lib().pt2q_gram_workspace_bytes(m), dtype=torch.uint8, device=X.device)
    pt2q.gram(X, G, workspace=ws, check=False)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        pt2q.gram(X, G, workspace=ws, check=False)
    ev1.record()
    torch.cuda.synchronize()
    pt2q._lib.check_status(ws, "gram timing")
    return ev0.elapsed_time(ev1) / reps


def gram_batched_time_ms(Xl, m, count, reps=2):
    """Average time of ONE batched Gram launch over `count` Grams (pt2q_gram_batched, as the
    step issues it) of the activation tensors Xl rotated over the items (item z reads
    Xl[z % len(Xl)], as ModelStep's units do), HIP events on torch's current stream (the launch
    stream)."""
    G = torch.empty((count, m, m), dtype=torch.float32, device=Xl[0].device)
    Xs = [Xl[z % len(Xl)] for z in range(count)]
    pt2q.engine.gram_batched(Xs, G)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        pt2q.engine.gram_batched(Xs, G)
    ev1.record()
    torch.cuda.synchronize()
    del G
    return ev0.elapsed_time(ev1) / reps


def load_traffic():
    path = os.path.join(ROOT, "profiles", "gram_pmc.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


X_DISTINCT = 4  # distinct resident activation tensors per input width, rotated over its units


class ModelStep:
    """This rank's share of the model: resident inputs, per-width workspaces, one step.

    Activations: X_DISTINCT distinct tensors per input width, rotated over that width's units
    (unit j of a width reads tensor j % X_DISTINCT), so the items of one batched Gram launch
    stream different rows -- a real model's layers have their own activations, and a single
    shared tensor would let concurrent items hit each other's X lines in L2 / MALL."""

    def __init__(self, a, rank, world, dev, io, shard_only=False):
        self.units = model_units(a)
        self.shards = sharding.assign_lpt([sharding.unit_cost(u, a.block_size) for u in self.units], world)
        self.mine = self.shards[rank]
        # shard_only: rank `rank`'s shard of a `world`-rank step on this one GPU (no process
        # group): the step skips the gather and keeps the bytes it would have sent (bench --shard)
        self.shard_only, self.rank = shard_only, rank
        self.gather_bytes = 0
        self.bs, self.ssr = a.block_size, not a.no_ssr
        self.pipe = None if a.no_overlap else pt2q.UnitPipeline(dev, self.bs, self.ssr, lanes=a.lanes)
        self.schedule = a.schedule
        self.gf = (sharding.GramsFirst(self.pipe, dev, batched=not a.no_batched_inverse, group=a.group,
                                       overlap=a.inverse_overlap, batch_grams=not a.no_batched_grams,
                                       inv_streams=a.inv_streams, chunk=parse_chunk(a.inv_chunk),
                                       spread=not a.group_max)
                   if self.pipe is not None else None)
        self.X, self.W, self.ws = {}, {}, {}
        self.xi = {}  # unit -> which of this rank's activation tensors of its width it reads
        self.index = {u[0]: i for i, u in enumerate(self.units)}
        # unit i reads activation slot (its position among the model's units of its width) %
        # X_DISTINCT, seeded by the slot alone: the same tensor on whichever rank runs the unit,
        # so every shard of a sharded step quantises exactly the whole step's inputs
        pos, slot = {}, {}
        for j, (_, lins, _) in enumerate(self.units):
            m = lins[0][2]
            slot[j] = pos.get(m, 0) % X_DISTINCT
            pos[m] = pos.get(m, 0) + 1
        have = {}
        for i in self.mine:
            name, lins, N = self.units[i]
            m = lins[0][2]
            if m not in self.X:
                self.X[m] = []
                self.ws[m] = self.pipe.workspace(m) if self.pipe else pt2q.UnitWorkspace(m, dev, self.bs)
            if (m, slot[i]) not in have:
                have[(m, slot[i])] = len(self.X[m])
                self.X[m].append(pt2q.fill_synthetic((N, m), 2000 + m + 7919 * slot[i], std=1.0,
                                                     outliers=True, device=dev).to(io))
            self.xi[i] = have[(m, slot[i])]
            for k, (p, n, _) in enumerate(lins):
                self.W[(i, p)] = pt2q.fill_synthetic((n, m), 100_000 + 16 * i + k, std=0.02,
                                                     device=dev).to(io)
        torch.cuda.synchronize()

    def provider(self, unit):
        i = self.index[unit[0]]
        _, lins, _ = unit
        return self.X[lins[0][2]][self.xi[i]], {p: self.W[(i, p)] for p, _, _ in lins}

    def run_unit(self, Ws, X):
        if self.pipe is not None:
            return self.pipe.run(Ws, X)
        return pt2q.quantize_unit(Ws, X, block_size=self.bs, use_ssr=self.ssr,
                                  workspace=self.ws[X.shape[1]], defer=True)

    def step(self):
        gf = self.gf if self.schedule == "grams-first" and self.pipe is not None else None
        res, _ = sharding.quantize_units_sharded(self.units, self.provider, run_unit=self.run_unit,
                                                 pack=True, dst=0, grams_first=gf, mine=self.mine,
                                                 gather=not self.shard_only, block_size=self.bs)
        if self.shard_only:
            # the bytes this rank's packed results would put on its xGMI link (rank 0 keeps its own)
            self.gather_bytes = 0 if self.rank == 0 else sum(e[4] for e in sharding._manifest(res))
            self.gathered = None
            return res
        self.gathered = None if res is None else len(res)  # linears whose results reached rank 0
        return res

    def phase_step(self):
        """One grams-first step of this rank's units with a device synchronisation between the
        three phases (Grams; batched Hessian inverses; block loops) -> wall seconds of each.
        Outside the timed region (the syncs add a little idle time)."""
        gf, units = self.gf, self.units
        t = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        inputs = {i: self.provider(units[i]) for i in self.mine}
        gf.begin([(i, units[i][1][0][2], units[i][2]) for i in self.mine])
        for i in self.mine:
            gf.gram(i, inputs[i][0])
        gf.flush()
        torch.cuda.synchronize()
        t["gram"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        gf.inverses()
        torch.cuda.synchronize()
        t["inverse"] = time.perf_counter() - t1
        t2 = time.perf_counter()
        jobs = [(i, [inputs[i][1][p] for p, _, _ in units[i][1]], units[i][2]) for i in self.mine]
        runs = gf.tails(jobs) if gf.grouped else [gf.tail(i, Ws, N) for i, Ws, N in jobs]
        for r in runs:
            r.finish()
        torch.cuda.synchronize()
        t["tails"] = time.perf_counter() - t2
        gf.check()
        return t

    def stage_busy(self):
        """Per-stage busy milliseconds of one grams-first step with the block loops on ONE lane
        (every launch of the step on one stream at a time), from the library's HIP-event
        brackets (pt2q_stage_timing: Gram, inverse, setup, SSR, ATQ, EF, outputs).  Outside the
        timed region."""
        lib = pt2q._lib
        lanes = self.gf.pipe.lanes
        self.gf.pipe.lanes = lanes[:1]
        try:
            torch.cuda.synchronize()
            lib.stage_timing(True)
            wall = self.phase_step()
        finally:
            lib.stage_timing(False)
            self.gf.pipe.lanes = lanes
        busy = lib.stage_timing_read()
        busy["phase_wall_ms"] = {k: v * 1e3 for k, v in wall.items()}
        return busy


# ------------------------------------------------------------------ stage rooflines

IO_BYTES = {"fp16": 2, "bf16": 2, "fp32": 4}


def model_work(units, bs, io_bytes=2, ssr=True):
    """Algorithmic work of one model step per stage: flops and HBM bytes.
    Per-channel units (bs >= m: one block) have no inverse, no error feedback and no SSR pass."""
    w = {k: 0.0 for k in ("gram_fl_2nm2", "gram_fl_done", "gram_bytes", "chol_fl", "ef_fl", "ef_bytes",
                          "ssr_bytes", "atq_bytes", "atq_valu", "setup_bytes", "out_bytes")}
    for _, lins, N in units:
        m = lins[0][2]
        w["gram_fl_2nm2"] += 2.0 * N * m * m          # §8(d) basis: the full product
        w["gram_fl_done"] += float(N) * m * (m + 1)    # the symmetric half actually formed
        w["gram_bytes"] += float(io_bytes) * N * m     # X read once
        nblk = -(-m // bs) if bs < m else 1
        if nblk > 1:
            w["chol_fl"] += float(m) ** 3              # potrf + trtri + lauum, m^3/3 each
        rsum = sum(max(m - (k + 1) * bs, 0) for k in range(nblk))
        for _, n, _ in lins:
            w["ef_fl"] += 2.0 * n * bs * rsum          # W[:, rem] -= E C, K = b
            w["ef_bytes"] += 8.0 * n * rsum            # read + write of W[:, rem] (fp32)
            if ssr and nblk > 1:
                # similarity pass over W[:, rem] of every SSR block (r = m, m - b, ...: m + rsum
                # columns) plus block 0's stand-alone w-bar pass (m columns); later blocks' w-bar
                # partials come out of the error feedback (no pass over W, DESIGN.md §3 CHUNK128)
                w["ssr_bytes"] += 4.0 * n * (2 * m + rsum)
            if nblk > 1:
                # every block's W columns read (fp32) and codes written; the error term E written
                # for every block that leaves columns behind
                w["atq_bytes"] += 5.0 * n * m + 4.0 * n * (m - (m - (nblk - 1) * bs))
                w["setup_bytes"] += (io_bytes + 4.0) * n * m  # W in, feature-major fp32 copy out
                w["out_bytes"] += 2.0 * n * m              # codes transposed back (int8 in + out)
            else:
                # per-channel: the caller's W read in place (io_bytes) and int8 codes written, no
                # layout copies (api.hip run_blocks); the ITF passes are VALU work (atq_pc.hip)
                w["atq_bytes"] += (io_bytes + 1.0) * n * m
                w["atq_valu"] += PC_VALU_PER_ELEM * n * m
        if nblk == 1:
            w["atq_bytes"] += 4.0 * m * m                  # S1 = S·1 over the unit's Gram, once per unit
    return w


# VALU lane-operations per element of a per-channel ATQ row (atq_pc.hip, counted from the
# register kernel's ISA: sum w 2, sum |w - mu| 3, init 10, one ITF pass 10-11 x ~7 passes (the
# wave's slowest row, tools/itf_dist), AGA + codes 14), and the chip's VALU rate: 256 CUs x 4
# SIMDs x 32 lanes per cycle at 2.4 GHz (MI355X_MICROARCH.md: a wave64 VALU op issues over 2
# cycles on a SIMD-32).
PC_VALU_PER_ELEM = 106.0
MI355X_VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


STAGE_KERNELS = {"gram": "gram16b_kernel / gram_streamk_kernel", "inverse": "chol_* + rank_update2 + gemmx_kernel",
                 "setup": "transpose_to_f32 + group_init", "ssr": "ssr_wbar_* + ssr_sim* + ssr_topk",
                 "atq": "atq_block_kernel + atq_finish_kernel", "ef": "ef2_gemm_kernel<4, true>",
                 "out": "transpose_i8 / transpose_f32"}


def stage_roofline(work, phase_s, busy, ms_per_step, world, gram_peak_tf, committed=None):
    """roofline.stages: every stage's algorithmic work per step against its peak.  Phase walls
    (gram / inverse / tails) are live (ModelStep.phase_step); every `kernel_busy_s` is live too:
    the library's HIP-event brackets around each stage's launches in one grams-first step with
    the block loops on ONE lane (ModelStep.stage_busy), so a stage's time is its own.  `committed`
    (profiles/stage_kernels.json, a rocprof trace of the same one-lane step) rides along as a
    cross-check only."""
    F32, HBM = MI355X_F32_MFMA_PEAK_TFLOPS * 1e12, MI355X_HBM_PEAK_GBS * 1e9
    GP = gram_peak_tf * 1e12
    b = {k: busy.get(k, 0.0) / 1e3 for k in ("gram", "inverse", "setup", "ssr", "atq", "ef", "out")}
    src = "live: pt2q_stage_timing HIP-event brackets, one-lane grams-first step (bench.py ModelStep.stage_busy)"
    st = {}
    g = b["gram"] or phase_s["gram"]
    st["gram"] = {"bound": "mfma", "seconds": phase_s["gram"], "kernel_busy_s": b["gram"], "source": src,
                  "flops_2nm2": work["gram_fl_2nm2"], "frac_2nm2": work["gram_fl_2nm2"] / g / GP,
                  "flops_done": work["gram_fl_done"], "frac_done": work["gram_fl_done"] / g / GP,
                  "hbm_frac": work["gram_bytes"] / g / HBM, "peak_tflops": gram_peak_tf}
    if work["chol_fl"] > 0:
        c = b["inverse"] or phase_s["inverse"]
        st["cholesky_inverse"] = {"bound": "mfma", "seconds": phase_s["inverse"], "kernel_busy_s": b["inverse"],
                                  "source": src, "flops": work["chol_fl"], "frac": work["chol_fl"] / c / F32}
    else:
        st["cholesky_inverse"] = {"seconds": phase_s["inverse"], "kernel_busy_s": b["inverse"], "flops": 0.0,
                                  "note": "per-channel: no inverse (H^-1 feeds only the error feedback)"}
    st["tails"] = {"seconds": phase_s["tails"], "source": "live phase wall (block loops on the lanes)"}
    if b["ef"] > 0 and work["ef_fl"] > 0:
        st["ef"] = {"bound": "mfma+hbm", "kernel_busy_s": b["ef"], "flops": work["ef_fl"],
                    "frac_mfma": work["ef_fl"] / b["ef"] / F32, "bytes": work["ef_bytes"],
                    "frac_hbm": work["ef_bytes"] / b["ef"] / HBM, "source": src}
    if b["ssr"] > 0:
        st["ssr"] = {"bound": "hbm", "kernel_busy_s": b["ssr"], "bytes": work["ssr_bytes"],
                     "frac_hbm": work["ssr_bytes"] / b["ssr"] / HBM, "source": src}
    if b["atq"] > 0:
        st["atq"] = {"bound": "hbm/latency", "kernel_busy_s": b["atq"], "bytes": work["atq_bytes"],
                     "frac_hbm": work["atq_bytes"] / b["atq"] / HBM, "source": src}
        if work["atq_valu"] > 0:  # per-channel rows: HBM fraction headline, the ITF passes' VALU beside it
            st["atq"].update(kernels="atq_pcr_kernel / atq_pc_kernel (pt2q_quantize_perchannel_group)",
                             valu_lane_ops=work["atq_valu"],
                             frac_valu=work["atq_valu"] / b["atq"] / (MI355X_VALU_PEAK_TOPS * 1e12),
                             valu_peak_tops=MI355X_VALU_PEAK_TOPS)
    io = b["setup"] + b["out"]
    if io > 0:
        st["layout"] = {"bound": "hbm", "kernel_busy_s": io, "bytes": work["setup_bytes"] + work["out_bytes"],
                        "frac_hbm": (work["setup_bytes"] + work["out_bytes"]) / io / HBM, "source": src,
                        "what": "W -> feature-major fp32 copies and the result transposes"}
    if committed and "tails" in committed:
        cc = {"ef": 0.0, "ssr": 0.0, "atq": 0.0}
        for name, (ms, _) in committed["tails"]["kernels"].items():
            for pre, stage in TAIL_STAGE:
                if name.startswith(pre):
                    cc[stage] += ms / 1e3
        st["cross_check"] = {"kernel_busy_s": cc, "source": "committed:profiles/stage_kernels.json "
                                                            "(rocprof kernel trace of a one-lane step)"}
    atq_floor = max(work["atq_bytes"] / HBM, work["atq_valu"] / (MI355X_VALU_PEAK_TOPS * 1e12))
    floor = (work["gram_fl_done"] / GP + work["chol_fl"] / F32 + work["ef_fl"] / F32 + atq_floor +
             (work["ef_bytes"] + work["ssr_bytes"] + work["setup_bytes"] + work["out_bytes"]) / HBM
             ) / max(world, 1)
    st["step"] = {"floor_s": floor, "frac": floor / (ms_per_step * 1e-3),
                  "floor": "Gram work done at the MFMA peak of its input type + Cholesky inverse and EF flops at "
                           "the f32 MFMA peak + EF/SSR/layout bytes at HBM peak + ATQ at the larger of its bytes at "
                           "HBM peak and (per-channel) its VALU work at the VALU peak, stages back to back, / ranks"}
    # the dominant stage: the largest live busy time, against the roofline that bounds it
    dom = max(("gram", "inverse", "ssr", "atq", "ef"), key=lambda k: b[k])
    d = {"stage": dom, "kernels": STAGE_KERNELS[dom], "busy_s": b[dom]}
    if dom == "gram":
        d.update(bound="mfma", unit="TFLOP/s", achieved=work["gram_fl_done"] / b[dom] / 1e12, peak=gram_peak_tf,
                 basis="work done N*m*(m+1)")
    elif dom == "inverse" or dom == "ef":
        fl = work["chol_fl"] if dom == "inverse" else work["ef_fl"]
        d.update(bound="mfma", unit="TFLOP/s", achieved=fl / b[dom] / 1e12, peak=MI355X_F32_MFMA_PEAK_TFLOPS)
    elif dom == "atq" and work["atq_valu"] > 0:
        # per-channel rows: the headline is the HBM fraction of the bytes the stage must move (W
        # read once, codes written, the Gram read once for S1); its VALU work rides beside it
        d.update(kernels="atq_pcr_kernel / atq_pc_kernel (pt2q_quantize_perchannel_group)", bound="hbm",
                 unit="GB/s", achieved=work["atq_bytes"] / b[dom] / 1e9, peak=MI355X_HBM_PEAK_GBS,
                 valu_achieved_tlane_ops=work["atq_valu"] / b[dom] / 1e12, valu_peak_tlane_ops=MI355X_VALU_PEAK_TOPS,
                 frac_valu=work["atq_valu"] / b[dom] / (MI355X_VALU_PEAK_TOPS * 1e12))
    else:
        by = work["ssr_bytes"] if dom == "ssr" else work["atq_bytes"]
        d.update(bound="hbm", unit="GB/s", achieved=by / b[dom] / 1e9, peak=MI355X_HBM_PEAK_GBS)
    d["frac"] = d["achieved"] / d["peak"]
    st["dominant"] = d
    return st


# kernel-name prefixes of the tail stages (ef_gemm_kernel, ef2_gemm_kernel<4>, ...)
TAIL_STAGE = (("ef_gemm", "ef"), ("ef2_gemm", "ef"), ("ef3_gemm", "ef"), ("ssr_", "ssr"), ("atq_", "atq"))


def load_committed_stages():
    kp = os.path.join(ROOT, "profiles", "stage_kernels.json")
    if os.path.exists(kp):
        with open(kp) as f:
            return json.load(f)
    return None


class H2DStep:
    """extra.h2d: SURVEY §8(d)'s whole window, "from H2D of inputs to results resident on rank 0":
    the step of `ms` (a grams-first ModelStep) with every input starting in PINNED HOST memory and
    the results ending there, as the reference's flow hands them over (main.py:225-230 returns
    `.cpu()` tensors).

    Per step: every linear's fp16 W is uploaded on a copy stream; every unit's activations
    (the same X_DISTINCT tensors per width as the resident line, each unit's own copy) are
    uploaded in chunks of `chunk` units into two device staging buffers per width, each chunk's
    batched Gram starting as soon as its copy lands while the next chunk copies; then the batched
    inverses and grouped block loops as usual; then every result (2-bit codes, alpha, mu, perm)
    is packed into one flat device buffer and copied into a pinned host buffer.  The staging
    replaces the resident activations, so the device holds 2 x chunk activation tensors per width
    instead of all of them."""

    def __init__(self, ms, chunk=2):
        self.ms, self.chunk = ms, chunk
        dev = ms.gf.dev
        self.copy = torch.cuda.Stream(dev)
        self.Xh = {m: [x.cpu().pin_memory() for x in xs] for m, xs in ms.X.items()}
        self.Wh = {k: w.cpu().pin_memory() for k, w in ms.W.items()}
        self.stage = {}
        for m, xs in ms.X.items():
            N = xs[0].shape[0]
            self.stage[m] = [torch.empty((chunk, N, m), dtype=xs[0].dtype, device=dev) for _ in range(2)]
        self.h2d_bytes = (sum(t.numel() * t.element_size() for t in self.Wh.values()) +
                          sum(self.Xh[u[1][0][2]][ms.xi[i]].numel() * 2 for i, u in
                              ((i, ms.units[i]) for i in ms.mine)))
        self.host_res = None
        self.d2h_bytes = 0

    def step(self):
        ms = self.ms
        gf, units, mine = ms.gf, ms.units, ms.mine
        eng = pt2q.engine
        comp = torch.cuda.current_stream(gf.dev)
        gf.begin([(i, units[i][1][0][2], units[i][2]) for i in mine])
        self.copy.wait_stream(comp)
        with torch.cuda.stream(self.copy):
            for k, Wd in ms.W.items():
                Wd.copy_(self.Wh[k], non_blocking=True)
        w_done = torch.cuda.Event()
        w_done.record(self.copy)
        # Grams: per width, units in slot order, chunk by chunk through the staging buffers
        by_group = {}
        for i in mine:
            by_group.setdefault(gf.slot[i][0], []).append(i)
        freed = {}
        for g, items in sorted(by_group.items()):
            m = g[0]
            G = gf.groups[g]["G"]
            for c, c0 in enumerate(range(0, len(items), self.chunk)):
                part = items[c0:c0 + self.chunk]
                buf = self.stage[m][c % 2]
                ev = freed.get((m, c % 2))
                if ev is not None:
                    self.copy.wait_event(ev)  # the Gram that last read this buffer is done
                with torch.cuda.stream(self.copy):
                    for j, i in enumerate(part):
                        buf[j].copy_(self.Xh[m][ms.xi[i]], non_blocking=True)
                landed = torch.cuda.Event()
                landed.record(self.copy)
                comp.wait_event(landed)
                z0 = gf.slot[part[0]][1]
                assert [gf.slot[i][1] for i in part] == list(range(z0, z0 + len(part)))
                eng.gram_batched([buf[j] for j in range(len(part))], G[z0:z0 + len(part)])
                done = torch.cuda.Event()
                done.record(comp)
                freed[(m, c % 2)] = done
        comp.wait_event(w_done)
        gf.inverses()
        jobs = [(i, [ms.W[(i, p)] for p, _, _ in units[i][1]], units[i][2]) for i in mine]
        runs = gf.tails(jobs)
        results = {}
        for i, run in zip(mine, runs):
            name, lins, _ = units[i]
            for (p, _, _), out in zip(lins, run.finish()):
                results[f"{name}.{p}"] = {"T2": eng.pack_ternary(out.T)[0], "alpha": out.alpha, "mu": out.mu,
                                          "perm": out.perm}
        gf.check()
        manifest, flat = sharding._flatten(results)
        if self.host_res is None or self.host_res.numel() < flat.numel():
            self.host_res = torch.empty(flat.numel(), dtype=torch.uint8).pin_memory()
        self.host_res[:flat.numel()].copy_(flat, non_blocking=True)
        self.d2h_bytes = flat.numel()
        torch.cuda.synchronize(gf.dev)
        return manifest


def h2d_run(ms, steps=2, warmup=1):
    """extra.h2d: H2DStep timed like the main line (warmup, then `steps` steps, synchronised)."""
    h = H2DStep(ms)
    for _ in range(warmup):
        h.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        h.step()
    torch.cuda.synchronize()
    s = (time.perf_counter() - t0) / steps
    cols = sharding.units_cols([ms.units[i] for i in ms.mine])
    out = {"ms_per_step": s * 1e3, "cols_per_s": cols / s, "steps": steps, "warmup": warmup,
           "h2d_bytes_per_step": h.h2d_bytes, "d2h_bytes_per_step": h.d2h_bytes,
           "pcie_gbs_if_transfer_bound": (h.h2d_bytes + h.d2h_bytes) / s / 1e9,
           "window": "from pinned-host fp16 W and X to packed results in pinned host memory (SURVEY §8(d))",
           "chunk_units": h.chunk}
    del h
    return out


class LayerStep:
    """One n x m layer per rank (weak scaling), a hipGraph replay; results gathered at N > 1."""

    def __init__(self, a, rank, world, dev, io):
        self.world = world
        self.Wl = pt2q.fill_synthetic((a.n, a.m), 1000 + rank, std=0.02, device=dev).to(io)
        self.Xl = pt2q.fill_synthetic((a.tokens, a.m), 2000 + rank, std=1.0, outliers=True, device=dev).to(io)
        self.graph = pt2q.LayerGraph(self.Wl, self.Xl, a.block_size, not a.no_ssr)
        self.units = [("layer", [("proj", a.n, a.m)], a.tokens)] * world

    def step(self):
        out = self.graph.replay()
        if self.world > 1:
            packed, _ = pt2q.pack_ternary(out.T)
            sharding.gather_results({f"rank{dist.get_rank()}": {"T2": packed, "alpha": out.alpha,
                                                                "mu": out.mu, "perm": out.perm}})
        return out


class SplitStep:
    """One n x m layer whose Gram is split over the ranks' calibration rows:
    partial Grams -> rank-ordered fold on rank 0 -> Cholesky inverse and block loop there."""

    def __init__(self, a, rank, world, dev, io):
        lo, hi = sharding.row_slice(a.tokens, rank, world)
        self.X = pt2q.fill_synthetic((hi - lo, a.m), 3000 + rank, std=1.0, outliers=True, device=dev).to(io)
        self.W = pt2q.fill_synthetic((a.n, a.m), 1000, std=0.02, device=dev).to(io) if rank == 0 else None
        self.bs, self.ssr = a.block_size, not a.no_ssr
        self.units = [("layer", [("proj", a.n, a.m)], a.tokens)]

    def step(self):
        outs = sharding.quantize_layer_split([self.W], self.X, dst=0, block_size=self.bs,
                                             use_ssr=self.ssr)
        if outs is not None and not outs[0].spd:
            raise RuntimeError("synthetic Hessian not SPD")
        return outs


class DryStep:
    """--dry-run: the model workload's rank plumbing on CPU (gloo) -- the same unit list, LPT
    shards, sharding.quantize_units_sharded and gather as ModelStep, with a stub run_unit that
    returns small deterministic outputs instead of launching kernels."""

    def __init__(self, a, rank, world, dev, io, shard_only=False):
        self.units = model_units(a)
        self.shards = sharding.assign_lpt([sharding.unit_cost(u, a.block_size) for u in self.units], world)
        self.mine = self.shards[rank]
        # shard_only: rank `rank`'s shard of a `world`-rank step on this one GPU (no process
        # group): the step skips the gather and keeps the bytes it would have sent (bench --shard)
        self.shard_only, self.rank = shard_only, rank
        self.gather_bytes = 0
        self.bs = a.block_size
        self.ran = []

    def provider(self, unit):
        name, lins, _ = unit
        return None, {p: (name, p, n, m) for p, n, m in lins}

    def run_unit(self, Ws, X):
        import zlib
        from types import SimpleNamespace
        outs = []
        for name, p, n, m in Ws:
            self.ran.append(f"{name}.{p}")
            g = torch.Generator().manual_seed(zlib.crc32(f"{name}.{p}".encode()))
            B = -(-m // self.bs)
            n = min(n, 8)  # 8-row stand-ins: full-size shapes (a 7B / 13B unit list) stay cheap on gloo
            outs.append(SimpleNamespace(alpha=torch.rand((n, B), generator=g), mu=torch.rand((n, B), generator=g),
                                        T=(torch.randint(0, 3, (n, m), generator=g) - 1).to(torch.int8),
                                        perm=torch.randperm(m, generator=g)))
        return outs

    def step(self):
        res, _ = sharding.quantize_units_sharded(self.units, self.provider, run_unit=self.run_unit,
                                                 pack=False, dst=0)
        self.last = res
        return res


def shard_main(a, dev, io):
    """bench.py --gpus N --shard r|all (one process, one GPU): rank r's LPT shard of an N-rank
    model step timed alone ('all': the whole step on this GPU first -- T1 and its phases -- then
    every rank's shard); one JSON line with the per-shard times and the projection."""
    world = a.gpus or 1
    if a.workload != "model" or world < 2 or a.dry_run:
        raise SystemExit("--shard needs the model workload and --gpus N >= 2")
    ranks = list(range(world)) if a.shard == "all" else [int(a.shard)]
    t1 = t1p = None
    if a.shard == "all":
        w = ModelStep(a, 0, 1, dev, io)
        for _ in range(a.warmup):
            w.step()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            w.step()
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
        t1 = float(np.median(ts))
        t1p = w.phase_step()
        log(0, f"whole step on one GPU: {t1:.1f} ms, phases { {k: round(v * 1e3, 1) for k, v in t1p.items()} }")
        del w
        gc.collect()
        torch.cuda.empty_cache()
    res = shard_runs(a, dev, io, world, ranks, t1, t1p, steps=a.steps, warmup=max(a.warmup, 2))
    res.update({"metric": "one-GPU shard timing (projection; no RCCL, no scaling measurement)",
                "model": a.model, "config": sharding.MODELS[a.model]["config"],
                "workload": describe_units(model_units(a), a.layers), "tokens": a.tokens,
                "block_size": a.block_size, "io_dtype": a.io_dtype})
    print(json.dumps(res), flush=True)
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    rc = launch_or_check(a, argv)
    if rc is not None:
        return rc
    _load_runtime(a.dry_run)
    resolve(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        if a.workload != "model":
            raise SystemExit("--dry-run covers the model workload only")
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if a.share_gpu:
            local = 0
        elif world > torch.cuda.device_count():
            print(f"[bench] refusing: {world} ranks but {torch.cuda.device_count()} visible GPUs", file=sys.stderr)
            return 2
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
        if world > 1:
            if a.share_gpu:
                dist.init_process_group("gloo")  # RCCL refuses two ranks on one device
            else:
                dist.init_process_group("nccl", device_id=dev)
    if world > 1:
        world, rank = dist.get_world_size(), dist.get_rank()
    io = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[a.io_dtype]
    if a.shard is not None:
        return shard_main(a, dev, io)
    if a.workload == "decoder":  # one line: the layer-by-layer flow (see decoder_run)
        if world > 1:
            raise SystemExit("--workload decoder runs on one GPU")
        r = decoder_run(a, dev)
        print(json.dumps({"metric": "weight-columns quantized/sec (and s/layer) at d=4096 [real calibration flow, "
                                    "decoder layer by decoder layer]", "value": r["cols_per_s"], "unit": "cols/s",
                          "n_gpus": 1, "higher_is_better": True, "dtype": "fp16->f32",
                          "data": "synthetic (random-init model, random token ids)", "decoder": r}), flush=True)
        return 0
    N, bs, d = a.tokens, a.block_size, a.hidden
    use_ssr = not a.no_ssr

    t_setup = time.perf_counter()
    kind = DryStep if a.dry_run else {"model": ModelStep, "layer": LayerStep, "split": SplitStep}[a.workload]
    work = kind(a, rank, world, dev, io)
    log(rank, f"{a.workload} inputs resident ({time.perf_counter() - t_setup:.1f}s); warmup {a.warmup}")
    for i in range(a.warmup):
        work.step()
        sync()
        log(rank, f"warmup step {i + 1}/{a.warmup} done")
    if a.workload == "layer" and not work.graph.spd():
        raise RuntimeError("synthetic Hessian not SPD")
    if world > 1:
        dist.barrier()
    sync()
    with no_gc():
        t0 = time.perf_counter()
        step_ms = []
        for i in range(a.steps):
            ts = time.perf_counter()
            work.step()
            sync()  # per-step wall (box-to-box and step-to-step spread); the step ends in host reads anyway
            step_ms.append(1e3 * (time.perf_counter() - ts))
            if a.steps > 3:
                log(rank, f"step {i + 1}/{a.steps}")
        sync()
        t_rank = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ranks = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if a.workload == "model":
        # per-rank shard and its own compute time (before the closing barrier): load balance
        mine = getattr(work, "mine", [])
        me = {"rank": rank, "units": len(mine),
              "linears": sum(len(work.units[i][1]) for i in mine),
              "cols": sharding.units_cols([work.units[i] for i in mine]),
              "ms_per_step": 1e3 * t_rank / max(a.steps, 1),
              "step_ms": {"min": min(step_ms), "median": float(np.median(step_ms)), "max": max(step_ms)}
              if step_ms else None}
        if a.dry_run:
            me["ran"] = sorted(set(work.ran))
        # the LPT cost model's seconds for this shard (sharding.unit_cost), beside the measured ms,
        # so a first multi-GPU run shows a modelled-vs-measured imbalance at once
        me["predicted_cost_s"] = sum(sharding.unit_cost(work.units[i], a.block_size) for i in mine)
        # the phase model of this rank's step (fixed latencies included, sharding.shard_phases)
        me["predicted_shard_s"] = sharding.shard_cost([work.units[i] for i in mine], a.block_size,
                                                      IO_BYTES[a.io_dtype])
        if world > 1:
            ranks = [None] * world
            dist.all_gather_object(ranks, me)
        else:
            ranks = [me]
    ms_per_step = 1e3 * elapsed / max(a.steps, 1)
    cols = {"model": sharding.units_cols(work.units), "layer": world * a.m, "split": a.m}[a.workload]
    balance = None
    if ranks:
        pc = [r["predicted_cost_s"] for r in ranks]
        mc = [r["ms_per_step"] for r in ranks]
        ps = [r["predicted_shard_s"] for r in ranks]
        balance = {"predicted_max_over_mean": max(pc) / (sum(pc) / len(pc)) if sum(pc) > 0 else None,
                   "shard_model_max_over_mean": max(ps) / (sum(ps) / len(ps)) if sum(ps) > 0 else None,
                   "measured_max_over_mean": max(mc) / (sum(mc) / len(mc)) if sum(mc) > 0 else None,
                   "model": "sharding.unit_cost (per-unit shares of the fitted phase model), LPT over the ranks; "
                            "sharding.shard_cost: the phase model of each rank's step"}
    log(rank, f"timed {a.steps} steps: {ms_per_step:.1f} ms/step")
    if a.dry_run:
        if rank == 0:
            got = work.last
            res = {"metric": "weight-columns quantized/sec (and s/layer) at d=4096 [DRY RUN: CPU stub units]",
                   "value": cols / (ms_per_step * 1e-3), "unit": "cols/s", "n_gpus": world,
                   "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms_per_step,
                   "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "none",
                   "data": "dry run (no kernels)", "ranks": ranks, "lpt_balance": balance,
                   "gathered_linears": sorted(got) if got is not None else None,
                   "config": {"workload": "dry run", "weight_columns_per_step": cols}}
            print(json.dumps(res), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0

    extra = {}
    roof = None
    if rank == 0 and not a.no_extra and a.workload != "split":
        # the d=4096 q_proj layer alone (s/layer at d=4096): one hipGraph replay per layer
        if a.workload == "model":
            Wl = pt2q.fill_synthetic((d, d), 1000, std=0.02, device=dev).to(io)
            Xl = work.X[d][0] if d in work.X else None
            if Xl is None:
                Xl = pt2q.fill_synthetic((N, d), 2000 + d, std=1.0, outliers=True, device=dev).to(io)
            g = pt2q.LayerGraph(Wl, Xl, bs, use_ssr)
        else:
            Wl, Xl, g = work.Wl, work.Xl, work.graph
        g.replay()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        s_layer = (time.perf_counter() - t1) / 5
        if not g.spd():
            raise RuntimeError("synthetic Hessian not SPD")
        X2 = Xl[:2048].contiguous()
        g2 = pt2q.LayerGraph(Wl, X2, bs, use_ssr)
        g2.replay()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(5):
            g2.replay()
        torch.cuda.synchronize()
        s_layer_2048 = (time.perf_counter() - t2) / 5
        g2.spd()
        extra.update({"s_per_layer_d4096": s_layer, "cols_per_s_layer_d4096": d / s_layer,
                      "s_per_layer_d4096_n2048": s_layer_2048, "cols_per_s_layer_d4096_n2048": d / s_layer_2048})
        del g, g2
        # dominant kernel: the symmetric Gram XᵀX (16-bit MFMA for fp16/bf16 X), timed alone with
        # HIP events per input width, averaged over the step's mix of Gram launches
        mix = {}
        for _, lins, Nu in work.units:
            mix[lins[0][2]] = mix.get(lins[0][2], 0) + 1
        # the step's Gram launches: one pt2q_gram_batched launch per input width (<= 128 Grams
        # each) with batched Grams, else one pt2q_gram launch per unit
        gb = (a.workload == "model" and work.gf is not None and work.gf.batch_grams and a.io_dtype != "fp32"
              and all(m % 256 == 0 for m in mix))
        per_launch = {m: (min(cnt, pt2q.engine.GRAM_BATCH_MAX) if gb else 1) for m, cnt in mix.items()}
        nl = {m: -(-cnt // per_launch[m]) for m, cnt in mix.items()}
        launches = sum(nl.values())
        tot_ms = tot_fl = 0.0
        per_m = {}
        for m, cnt in sorted(mix.items()):
            Xm = work.X.get(m) if a.workload == "model" else [work.Xl]
            if Xm is None:
                Xm = [pt2q.fill_synthetic((N, m), 2000 + m, std=1.0, outliers=True, device=dev).to(io)]
            # the step's own activations (X_DISTINCT distinct tensors rotated over the items) set
            # the line; one tensor shared by every item is timed beside it (cross-item L2 / MALL hits)
            ms = gram_batched_time_ms(Xm, m, per_launch[m]) if gb else gram_time_ms(Xm[0], m)
            fl = float(N) * m * (m + 1) * per_launch[m]  # unique entries of each symmetric product, 2 flop each
            per_m[str(m)] = {"launches_per_step": nl[m], "grams_per_launch": per_launch[m], "avg_launch_ms": ms,
                             "ms_per_gram": ms / per_launch[m], "tflops": fl / ms / 1e9,
                             "distinct_x": len(Xm) if gb else 1}
            if gb:
                ms1 = gram_batched_time_ms(Xm[:1], m, per_launch[m])
                per_m[str(m)]["shared_x"] = {"avg_launch_ms": ms1, "tflops": fl / ms1 / 1e9,
                                             "note": "every item reads ONE activation tensor"}
            tot_ms += nl[m] * ms
            tot_fl += nl[m] * fl
        avg_ms, avg_fl = tot_ms / launches, tot_fl / launches
        achieved = avg_fl / (avg_ms * 1e-3) / 1e12
        peak = MI355X_F32_MFMA_PEAK_TFLOPS if a.io_dtype == "fp32" else MI355X_F16_MFMA_PEAK_TFLOPS
        kname = ("gram_streamk_kernel (symmetric Gram XᵀX, f32 MFMA 32x32x2)" if a.io_dtype == "fp32" else
                 "gram16b_kernel: every Gram of one input width in one data-parallel launch (256x256 tiles, "
                 "LDS-DMA ring, ds_read_b64_tr_b16, hand-interleaved 16-bit MFMA 32x32x16, f32 accumulate)"
                 if gb else
                 "gram16x_kernel (m=4096: 128x256 tiles) / gram16w_kernel (m=11008: 256x256 tiles): "
                 "symmetric Gram XᵀX, LDS-DMA ring, ds_read_b64_tr_b16, hand-interleaved 16-bit MFMA "
                 "32x32x16, f32 accumulate")
        fl_2nm2 = sum(nl[m] * per_launch[m] * 2.0 * N * m * m for m in mix) / launches
        roof = {"bound": "mfma", "kernel": kname, "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                "frac": achieved / peak, "frac_basis": "work done: N*m*(m+1) flops per Gram (the symmetric "
                                                      "half the kernel forms) x Grams per launch",
                "frac_2nm2": fl_2nm2 / (avg_ms * 1e-3) / 1e12 / peak,
                "traffic": None, "avg_launch_ms": avg_ms,
                "flops_per_launch": avg_fl, "flops_per_launch_2nm2": fl_2nm2, "per_width": per_m,
                "gram_share_of_step": tot_ms / (ms_per_step * max(world, 1)) if a.workload == "model" else
                avg_ms / ms_per_step}
        if a.workload == "model" and work.gf is not None and a.schedule == "grams-first" and world == 1:
            work.phase_step()
            ph = work.phase_step()
            busy = work.stage_busy()
            roof["phase_s"] = ph
            roof["stage_busy_ms"] = busy
            roof["stages"] = stage_roofline(model_work(work.units, bs, IO_BYTES[a.io_dtype], use_ssr), ph, busy,
                                            ms_per_step, world, peak, load_committed_stages())
        tr = load_traffic()
        key = "batched" if gb else "per_item"
        if tr and key in tr and all(str(m) in tr[key]["per_width"] for m in mix):
            # PMC fabric bytes per Gram of each width (same kernel, same launch shape), times the
            # Grams of the step, over its launches
            pw = tr[key]["per_width"]
            roof["traffic"] = sum(cnt * pw[str(m)]["fabric_bytes_per_gram"] for m, cnt in mix.items()) / launches
            roof["traffic_algorithmic"] = sum(cnt * 2.0 * N * m for m, cnt in mix.items()) / launches
            roof["traffic_source"] = "committed:profiles/gram_pmc.json (" + str(tr[key].get("source")) + ")"

    if rank == 0:
        model_desc = (f"{a.model} shapes: {describe_units(work.units, a.layers)}" if a.workload == "model" else
                      f"one {a.n}x{a.m} linear per rank" if a.workload == "layer" else
                      f"one {a.n}x{a.m} linear, its Gram split over {world} ranks' calibration rows")
        res = {
            "metric": "weight-columns quantized/sec (and s/layer) at d=4096",
            "value": cols / (ms_per_step * 1e-3),
            "unit": "cols/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak" if a.workload == "layer" else "strong",
            "vs_baseline": None,
            "dtype": f"{a.io_dtype}->f32" if a.io_dtype != "fp32" else "f32",
            "data": (f"synthetic (counter-hash {a.io_dtype} weights std 0.02; {a.io_dtype} activations, unit "
                     f"variance, 1% x20 outlier channels; {X_DISTINCT} distinct resident activation tensors per "
                     "input width per rank, rotated over that width's units)"),
            "config": {"workload": f"{model_desc}, N={N} calibration rows, variant M, "
                                   f"{'SSR' if use_ssr else 'sequential'}+ATQ(ITF,AGA), block {bs}",
                       "weight_columns_per_step": cols, "tokens": N, "io_dtype": a.io_dtype,
                       "block_size": bs,
                       "parallelism": ({"model": f"LPT unit sharding x{world}", "layer": f"layer per rank x{world}",
                                        "split": f"Gram rows x{world}, rank-ordered fold on rank 0"}[a.workload])
                                  + ((", gloo gather, TEST ONLY: every rank shares cuda:0" if a.share_gpu else
                                      ", rccl gather") if world > 1 else "")
                                  + ((f", every Gram first then the tails on {a.lanes} unit lanes"
                                      if a.schedule == "grams-first" else
                                      f", {a.lanes} unit lanes (Grams chained, tails overlapped)")
                                     if a.workload == "model" and not a.no_overlap else "")},
        }
        if a.workload == "model":
            res["s_model"] = ms_per_step / 1e3
            res["ranks"] = ranks
            res["lpt_balance"] = balance
            res["gathered_linears"] = getattr(work, "gathered", None)
        if roof is not None:
            res["roofline"] = roof
        if (a.workload == "model" and world == 1 and not a.no_extra and not a.no_h2d and work.gf is not None
                and a.schedule == "grams-first" and all(len(v) > 0 for v in work.X.values())):
            log(rank, "h2d (transfer-inclusive) run ...")
            try:
                extra["h2d"] = h2d_run(work)
            except Exception as e:  # reported, never allowed to drop the line
                extra["h2d"] = {"error": f"{type(e).__name__}: {e}"}
            gc.collect()
            torch.cuda.empty_cache()
        full_model = (a.workload == "model" and world == 1 and not a.no_extra and not a.hidden_given
                      and a.layers == sharding.MODELS[a.model]["layers"])
        if full_model and (not a.no_configs or not a.no_shards or not a.no_decoder):
            units_main = work.units
            del work  # the headline model's resident inputs and buffers (~150 GB) make room
            gc.collect()
            torch.cuda.empty_cache()
            if not a.no_shards and a.schedule == "grams-first":
                log(rank, "8-rank shards, one at a time on this GPU (projection) ...")
                try:
                    extra["shards8"] = shard_runs(a, dev, io, 8, t1_ms=ms_per_step,
                                                  t1_phase=roof.get("phase_s") if roof else None)
                except Exception as e:  # reported, never allowed to drop the line
                    extra["shards8"] = {"error": f"{type(e).__name__}: {e}"}
                gc.collect()
                torch.cuda.empty_cache()
            if not a.no_decoder and a.model == "llama-2-7b":
                log(rank, "decoder flow (PT2LLMQuantizer.quantize, layer by layer) ...")
                try:
                    extra["decoder"] = decoder_run(a, dev)
                except Exception as e:  # reported, never allowed to drop the line
                    extra["decoder"] = {"error": f"{type(e).__name__}: {e}"}
                gc.collect()
                torch.cuda.empty_cache()
            if not a.no_configs:
                log(rank, "per-config runs ...")
                extra["configs"] = config_runs(a, dev)
            work = argparse.Namespace(units=units_main)
        res["extra"] = extra
        if world == 1 and not a.no_cpu_baseline and a.workload != "split":
            log(rank, "cpu baseline (oracle) ...")
            units = work.units if a.workload == "model" else [("layer", [("proj", a.n, a.m)], N)]
            res["cpu_baseline"] = cpu_baseline(units, N, bs, use_ssr, d if a.workload == "model" else a.m)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
