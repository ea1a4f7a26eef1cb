"""Multi-GPU layer sharding: one process per GPU, independent linears per rank, one gather.

The per-layer loop has no cross-layer dependency once activations are captured, so linears are
independent work units.  Units are assigned longest-processing-time first; linears
that share an input (q/k/v, gate/up) form ONE unit so they share a Gram and a Cholesky.  The only
collective is a gather of the quantised results to the root rank over RCCL/xGMI (backend "nccl"
is RCCL on ROCm) — 2-bit packed codes (utils.py:189-219 layout) plus scales and permutation.

Reference flow replaced: main.py:257-304 (every linear of every decoder layer, one after the
other, on the devices HF/accelerate `device_map="auto"` placed the layers on, model.py:257).

Units are (name, [(proj, n, m)], N) tuples.  This module imports no device code at load time, so
the assignment and the gather are testable on CPU with gloo.
"""
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def assign_lpt(costs: Sequence[float], world_size: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of work units to ranks (deterministic)."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    loads = [0.0] * world_size
    shards: List[List[int]] = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (loads[k], k))
        shards[r].append(i)
        loads[r] += costs[i]
    for s in shards:
        s.sort()
    return shards


def llama_units(num_layers: int, hidden: int = 4096, inter: int = 11008, tokens: int = 262144):
    """Work units of a Llama-2-style decoder stack: (name, [(proj, n, m)], N)."""
    units = []
    for l in range(num_layers):
        units.append((f"layer_{l}.qkv", [("q_proj", hidden, hidden), ("k_proj", hidden, hidden),
                                         ("v_proj", hidden, hidden)], tokens))
        units.append((f"layer_{l}.o", [("o_proj", hidden, hidden)], tokens))
        units.append((f"layer_{l}.gate_up", [("gate_proj", inter, hidden), ("up_proj", inter, hidden)],
                      tokens))
        units.append((f"layer_{l}.down", [("down_proj", hidden, inter)], tokens))
    return units


def gpt2_units(num_layers: int = 12, hidden: int = 768, inter: int = 3072, tokens: int = 2048):
    """GPT-2 decoder stack (HF Conv1D weights taken transposed): c_attn is already
    the fused q/k/v projection, so every linear is its own unit."""
    units = []
    for l in range(num_layers):
        units.append((f"h_{l}.c_attn", [("c_attn", 3 * hidden, hidden)], tokens))
        units.append((f"h_{l}.attn_c_proj", [("attn.c_proj", hidden, hidden)], tokens))
        units.append((f"h_{l}.c_fc", [("c_fc", inter, hidden)], tokens))
        units.append((f"h_{l}.mlp_c_proj", [("mlp.c_proj", hidden, inter)], tokens))
    return units


def opt_units(num_layers: int = 24, hidden: int = 2048, ffn: int = 8192, tokens: int = 2048):
    """OPT decoder stack (model.py:139-171 finds q/k/v/out_proj, fc1, fc2): q/k/v share one input."""
    units = []
    for l in range(num_layers):
        units.append((f"layer_{l}.qkv", [("q_proj", hidden, hidden), ("k_proj", hidden, hidden),
                                         ("v_proj", hidden, hidden)], tokens))
        units.append((f"layer_{l}.out", [("out_proj", hidden, hidden)], tokens))
        units.append((f"layer_{l}.fc1", [("fc1", ffn, hidden)], tokens))
        units.append((f"layer_{l}.fc2", [("fc2", hidden, ffn)], tokens))
    return units


# The BASELINE.json configs C2-C5 as model workloads: unit list, calibration
# rows N, block size (C5 per-channel: one block per linear, b >= every m) and activation dtype.
MODELS = {
    "gpt2": dict(config="C2 GPT-2-small all linears, ITF + SSR", layers=12,
                 units=lambda L, N: gpt2_units(L, 768, 3072, N), tokens=2048, block_size=128, io="fp32"),
    "opt-1.3b": dict(config="C3 OPT-1.3B fp16, AGA + GPTQ error feedback", layers=24,
                     units=lambda L, N: opt_units(L, 2048, 8192, N), tokens=2048, block_size=128, io="fp16"),
    "llama-2-7b": dict(config="C4 Llama-2-7B fp16, full ATQ + SSR", layers=32,
                       units=lambda L, N: llama_units(L, 4096, 11008, N), tokens=262144, block_size=128,
                       io="fp16"),
    "llama-2-13b": dict(config="C5 Llama-2-13B bf16, per-channel, 4096-row Hessian", layers=40,
                        units=lambda L, N: llama_units(L, 5120, 13824, N), tokens=4096, block_size=1 << 14,
                        io="bf16"),
}


def model_units(model: str, layers: Optional[int] = None, tokens: Optional[int] = None):
    """Work units of one of MODELS (layers / tokens override the config's)."""
    c = MODELS[model]
    return c["units"](c["layers"] if layers is None else layers, c["tokens"] if tokens is None else tokens)


# ----------------------------------------------------------------- cost model
# One rank's grams-first step (GramsFirst: every Gram, then the batched inverses -- or, for
# per-channel units, S1 / d -- then the grouped block loops on the lanes), phase by phase, with the
# fixed latencies that do NOT shrink with a shard written out.  Constants fitted (round 6) to the
# phase walls of the whole 7B / 13B steps and of their 8-rank shards timed alone on one MI355X
# (bench.py --gpus 8 --shard all; profiles/r06a_shards_c4.json, and r06i_shards_c5.json after the
# S1 ring kernel and the upper-only per-channel Grams): the model reproduces all four within 6 %
# (C4 2236 vs 2232 ms, its shards 302 vs 298-306 ms; C5 105 vs 105 ms, its shards 14.6-15.4 ms).
#   Gram: the batched 16-bit Gram runs 256 x 256 tiles in waves of one tile per CU; a wave costs
#     N * 2 * 256^2 / GRAM_TILE_RATE (a CU's MFMA rate under the power limit) + GRAM_TILE_FIXED
#     (the tile's ramp and its 512 KiB mirrored epilogue: 54 us, which dominates at N = 4096; 36 us
#     for a per-channel unit's upper-only Gram, pt2q_gram_batched_upper).
#   Inverse: per chunk of <= 32 items, m / 64 serial panel steps of INV_STEP each, plus the
#     trailing updates at INV_RATE m^3 per second.
#   S1 / d (per-channel units): S1_FIXED + the Grams' bytes at S1_BW.
#   Tails: the block loops' work LOOP_NR per n * r (error feedback + SSR passes over the remaining
#     columns) plus LOOP_BLOCK per block of each group (its launch chain), the latter spread over
#     the lanes; per-channel groups LOOP_PC per element plus LOOP_PC_GROUP per group (its last,
#     slowest wave).
SHARD_MODEL = dict(
    cus=256,
    gram_tile_rate=4.887e12, gram_tile_fixed=5.43e-5, gram_tile_fixed_upper=3.6e-5, gram_batch=128,
    inv_step=4.53e-5, inv_rate=1.134e14, chunk=32,
    s1_fixed=5.4e-4, s1_bw=7.2e12,
    loop_nr=4.056e-12, loop_block=8.53e-5, loop_pc=3.28e-12, loop_pc_group=9.0e-4,
    lanes=3, group=16, pc_group=16,
)


def _rsum(m: int, block_size: int) -> int:
    nblk = -(-m // block_size) if block_size < m else 1
    return sum(max(m - (k + 1) * block_size, 0) for k in range(nblk))


def block_loop_cost(n: int, m: int, block_size: int = 128) -> float:
    """Modelled busy seconds of one n x m linear's block loop inside a full group (SHARD_MODEL)."""
    c = SHARD_MODEL
    if block_size >= m:
        return float(n) * m * c["loop_pc"] + c["loop_pc_group"] / (c["pc_group"] * c["lanes"])
    nblk = -(-m // block_size)
    return float(n) * _rsum(m, block_size) * c["loop_nr"] + nblk * c["loop_block"] / (c["group"] * c["lanes"])


def _gram_tiles(m: int) -> int:
    t = -(-m // 256)
    return t * (t + 1) // 2


def unit_cost(unit, block_size: int = 128) -> float:
    """Modelled seconds of one work unit (its Gram, Cholesky inverse or S1 / d, and every
    linear's block loop) as its share of a full step (SHARD_MODEL, per-item shares of the
    per-launch latencies).  LPT balances ranks on this; a pure flop count (N·m² dominates) would
    put a q/k/v unit level with an o unit although its three block loops make it ~1.6x longer."""
    c = SHARD_MODEL
    _, linears, N = unit
    m = linears[0][2]
    fixed = c["gram_tile_fixed_upper"] if block_size >= m else c["gram_tile_fixed"]
    t = _gram_tiles(m) * (float(N) * 2 * 256 * 256 / c["gram_tile_rate"] + fixed) / c["cus"]
    if block_size < m:
        t += float(m) ** 3 / c["inv_rate"] + (m / 64.0) * c["inv_step"] / c["chunk"]
    else:
        t += float(m) * m * 4 / c["s1_bw"]
    for _, n, _ in linears:
        t += block_loop_cost(n, m, block_size)
    return t


def _groups(count: int, cap: int, lanes: int):
    """GramsFirst.tails' group sizes for `count` same-class linears (spread policy)."""
    size = max(1, count if count <= cap else min(cap, -(-count // lanes)))
    return [min(size, count - g0) for g0 in range(0, count, size)]


def shard_phases(units, block_size: int = 128, io_bytes: int = 2, model=None):
    """{gram, inverse, tails} modelled seconds of ONE rank's grams-first step over `units`."""
    c = dict(SHARD_MODEL, **(model or {}))
    by_w, lins = {}, []
    for _, ls, N in units:
        m = ls[0][2]
        by_w[(m, int(N))] = by_w.get((m, int(N)), 0) + 1
        lins += [(n, m) for _, n, _ in ls]
    f32 = 16.0 if io_bytes == 4 else 1.0  # f32 MFMA: 1/16 of the 16-bit rate
    gram = 0.0
    for (m, N), cnt in by_w.items():
        for z0 in range(0, cnt, c["gram_batch"]):
            k = min(c["gram_batch"], cnt - z0)
            waves = -(-k * _gram_tiles(m) // c["cus"])
            fixed = c["gram_tile_fixed_upper"] if block_size >= m and io_bytes == 2 else c["gram_tile_fixed"]
            gram += waves * (f32 * N * 2 * 256 * 256 / c["gram_tile_rate"] + fixed)
    inv, s1_bytes = 0.0, 0.0
    for (m, N), cnt in by_w.items():
        if block_size >= m:
            s1_bytes += cnt * 4.0 * m * m
            continue
        inv += -(-cnt // c["chunk"]) * (m / 64.0) * c["inv_step"] + cnt * float(m) ** 3 / c["inv_rate"]
    if s1_bytes:
        inv += c["s1_fixed"] + s1_bytes / c["s1_bw"]
    shapes = {}
    for n, m in lins:
        shapes[(n, m)] = shapes.get((n, m), 0) + 1
    tails, pc_count = 0.0, {}
    for (n, m), cnt in shapes.items():
        if block_size >= m:
            tails += cnt * float(n) * m * c["loop_pc"]
            pc_count[m] = pc_count.get(m, 0) + cnt  # per-channel groups: by width, any row count
            continue
        nblk = -(-m // block_size)
        tails += cnt * float(n) * _rsum(m, block_size) * c["loop_nr"]
        tails += len(_groups(cnt, c["group"], c["lanes"])) * nblk * c["loop_block"] / c["lanes"]
    for m, cnt in pc_count.items():
        tails += len(_groups(cnt, c["pc_group"], c["lanes"])) * c["loop_pc_group"] / c["lanes"]
    return {"gram": gram, "inverse": inv, "tails": tails}


def shard_cost(units, block_size: int = 128, io_bytes: int = 2, model=None) -> float:
    """Modelled seconds of ONE rank's grams-first step over `units` (shard_phases summed)."""
    return sum(shard_phases(units, block_size, io_bytes, model).values())


# ----------------------------------------------------------------- heterogeneous result gather

_ALIGN = 16  # every entry starts 16-byte aligned, so the receiver views the bytes in place


def _manifest(results: Dict[str, Dict[str, torch.Tensor]]):
    """[(name, key, dtype, shape, padded nbytes)] of {name: {key: tensor}} in sorted (name, key)
    order: the layout _flatten gives the bytes (each entry padded to 16 bytes)."""
    out = []
    for name in sorted(results):
        for key in sorted(results[name]):
            t = results[name][key]
            nb = t.numel() * t.element_size()
            out.append((name, key, str(t.dtype).replace("torch.", ""), tuple(t.shape), nb + (-nb) % _ALIGN))
    return out


def _flatten(results: Dict[str, Dict[str, torch.Tensor]]):
    """(manifest, flat uint8 tensor) of {name: {key: tensor}}: every tensor's bytes back to back
    (each padded to 16 bytes) in _manifest's order -- the send buffer of a non-destination rank."""
    manifest, parts = _manifest(results), []
    for name, key, _, _, nb in manifest:
        t = results[name][key].contiguous()
        b = t.reshape(-1).view(torch.uint8) if t.numel() else torch.empty(0, dtype=torch.uint8, device=t.device)
        if nb > b.numel():
            b = torch.cat([b, torch.zeros(nb - b.numel(), dtype=torch.uint8, device=b.device)])
        parts.append(b)
    if parts:
        flat = torch.cat(parts)
    else:
        flat = torch.empty(0, dtype=torch.uint8)
    return manifest, flat


def _unflatten(manifest, flat: torch.Tensor) -> Dict[str, Dict[str, torch.Tensor]]:
    out: Dict[str, Dict[str, torch.Tensor]] = {}
    o = 0
    for name, key, dt, shape, nb in manifest:
        dtype = getattr(torch, dt)
        cnt = 1
        for d in shape:
            cnt *= d
        used = cnt * torch.empty(0, dtype=dtype).element_size()
        t = flat[o:o + used].view(dtype).reshape(shape)
        out.setdefault(name, {})[key] = t
        o += nb
    return out


def gather_results(results: Dict[str, Dict[str, torch.Tensor]], dst: int = 0, group=None,
                   device=None):
    """Gather heterogeneous per-rank results ({unit.linear: {key: tensor}}, any shapes/dtypes) to
    `dst`: one small object gather of the shape manifests, then ONE size-exact byte buffer per
    rank point-to-point (send/recv; RCCL over xGMI on GPUs, gloo on CPU).  Returns the merged dict
    on dst, None elsewhere.  The receive buffers go on `device`, else on the device of dst's own
    results, else (dst holds none) the current HIP device under RCCL / the CPU under gloo.
    Only the senders pack their bytes: dst keeps its own tensors as they are (one rank: no copy
    at all -- packing a 13B step's 1,400 result tensors cost as many device copies), so dst's own
    entries in the returned dict ALIAS the caller's tensors (they may be non-contiguous views;
    clone before modifying them in place); received entries are views into one receive buffer
    per sender."""
    own = {name: dict(entry) for name, entry in results.items()}
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return own
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank != dst:
        manifest, flat = _flatten(results)
    else:
        manifest = _manifest(results)
    manifests = [None] * world if rank == dst else None
    dist.gather_object(manifest, manifests, dst=dst, group=group)
    host = dist.get_backend(group) == "gloo"  # gloo moves host memory only: device bytes go via the CPU
    if rank != dst:
        if flat.numel():
            dist.send(flat.cpu() if host else flat, dst=dst, group=group)
        return None
    merged = own
    dev = device
    if dev is None:
        if manifest:  # the first manifest entry's tensor (a name may map to an empty dict)
            dev = results[manifest[0][0]][manifest[0][1]].device
        elif dist.get_backend(group) == "nccl":
            dev = torch.device("cuda", torch.cuda.current_device())
        else:
            dev = torch.device("cpu")
    ops, bufs = [], {}
    for r in range(world):
        if r == dst:
            continue
        nbytes = sum(e[4] for e in manifests[r])
        if nbytes:
            bufs[r] = torch.empty(nbytes, dtype=torch.uint8, device="cpu" if host else dev)
            ops.append(dist.P2POp(dist.irecv, bufs[r], r, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for r, buf in bufs.items():
        merged.update(_unflatten(manifests[r], buf.to(dev) if host else buf))
    return merged


# ----------------------------------------------------------------- sharded model quantisation

def units_cols(units) -> int:
    """Weight columns (the metric's unit) of a list of units: Σ m over their linears."""
    return sum(m for _, lins, _ in units for _, _, m in lins)


def quantize_units_sharded(units, provider: Callable, run_unit: Optional[Callable] = None,
                           block_size: int = 128, use_ssr: bool = True, percdamp: float = 0.01,
                           pack: bool = True, dst: int = 0, group=None, gather: bool = True,
                           grams_first: Optional["GramsFirst"] = None, mine: Optional[Sequence[int]] = None):
    """Quantise a list of independent work units across the ranks of `group` (LPT shards), then
    gather every linear's result to `dst`.

    provider(unit) -> (X, {proj: W}) gives a unit's activations and weights on this rank's device
    (called only for this rank's units).  run_unit(Ws, X) -> [LayerOutput] defaults to
    engine.UnitPipeline.run (Gram -> damping -> Cholesky inverse -> block loops, shared per unit,
    the next unit's Gram overlapping this unit's tail on a second stream).
    grams_first (a GramsFirst) replaces run_unit: every Gram of this rank's units first, then
    their tails.
    mine: this rank's unit indices, overriding the LPT assignment (the caller's own shards, e.g.
    one rank's shard of a larger world timed alone on one GPU, bench.py --shard).
    Results are {f"{unit}.{proj}": {"T2" (2-bit packed, utils.py:189-219) or "T", "alpha", "mu",
    "perm", "shape"}}; every "shape" entry (int64 (2,): T's n, m) is a row of ONE device table
    per step (a single host-to-device copy), i.e. a read-only view -- clone it before writing to
    it or saving it alone.  Returns (results on dst or None, this rank's unit indices)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if mine is None:
        mine = assign_lpt([unit_cost(u, block_size) for u in units], world)[rank]
    mine = list(mine)
    if run_unit is None and grams_first is None:
        from . import engine  # noqa: WPS433 (device code only when quantising for real)

        pipes = {}

        def run_unit(Ws, X):  # unit i+1's Gram overlaps unit i's tail (engine.UnitPipeline)
            dev = Ws[0].device
            if dev not in pipes:
                pipes[dev] = engine.UnitPipeline(dev, block_size, use_ssr, percdamp)
            return pipes[dev].run(Ws, X)
    runs = []
    if grams_first is not None:  # every Gram of this rank first, then the tails (GramsFirst)
        inputs = {i: provider(units[i]) for i in mine}
        if hasattr(grams_first, "begin"):
            grams_first.begin([(i, units[i][1][0][2], units[i][2]) for i in mine])
        for i in mine:
            grams_first.gram(i, inputs[i][0])
        if hasattr(grams_first, "flush"):
            grams_first.flush()  # batched Grams issued here
        if hasattr(grams_first, "inverses"):
            grams_first.inverses()
        jobs = [(i, [inputs[i][1][p] for p, _, _ in units[i][1]], units[i][2]) for i in mine]
        if getattr(grams_first, "grouped", False):
            tails = grams_first.tails(jobs)  # block loops grouped across units by shape
        else:
            tails = [grams_first.tail(i, Ws, N) for i, Ws, N in jobs]
        for i, run in zip(mine, tails):
            name, lins, _ = units[i]
            runs.append((name, [p for p, _, _ in lins], run))
    for i in ([] if grams_first is not None else mine):
        name, lins, _ = units[i]
        X, Wd = provider(units[i])
        runs.append((name, [p for p, _, _ in lins], run_unit([Wd[p] for p, _, _ in lins], X)))
    finished = [(name, projs, run.finish() if hasattr(run, "finish") else run) for name, projs, run in runs]
    if grams_first is not None and hasattr(grams_first, "check"):
        grams_first.check()  # every Gram's stall bits of the step, one host read
    results = {}
    # every linear's "shape" entry: one host-to-device copy for the step, not one blocking copy each
    outs_all = [out for _, _, outs in finished for out in outs]
    shapes = {}
    for dev in {o.T.device for o in outs_all}:
        mine_d = [o for o in outs_all if o.T.device == dev]
        tab = torch.tensor([list(o.T.shape) for o in mine_d], dtype=torch.int64).to(dev, non_blocking=False)
        shapes.update({id(o): tab[j] for j, o in enumerate(mine_d)})
    for name, projs, outs in finished:
        for p, out in zip(projs, outs):
            r = {"alpha": out.alpha, "mu": out.mu, "perm": out.perm, "shape": shapes[id(out)]}
            if pack:
                from . import engine
                r["T2"] = engine.pack_ternary(out.T)[0]
            else:
                r["T"] = out.T
            results[f"{name}.{p}"] = r
    if not gather:
        return results, mine
    return gather_results(results, dst=dst, group=group), mine


# ----------------------------------------------------------------- intra-layer split (§8e(ii))

def row_slice(N: int, rank: int, world: int):
    """Calibration rows [lo, hi) of `rank` in the intra-layer split (contiguous, balanced)."""
    return rank * N // world, (rank + 1) * N // world


def quantize_layer_split(Ws, X_local: torch.Tensor, dst: int = 0, group=None, block_size: int = 128,
                         use_ssr: bool = True, percdamp: float = 0.01, max_iter: int = 100,
                         gram_fn: Optional[Callable] = None, sum_fn: Optional[Callable] = None,
                         layer_fn: Optional[Callable] = None):
    """One layer (or a unit of linears sharing an input) too big for one GPU's share of the
    step, its Gram data-parallel over the ranks (main.py:128-230).

    Every rank holds its slice of the N calibration rows (row_slice) and forms its partial Gram
    Xᵣᵀ Xᵣ (a chain from +0, engine.gram).  The partials go point-to-point to `dst`, which folds
    them in rank order (engine.sum_partials: ((G₀ + G₁) + G₂) + …, deterministic -- an RCCL
    all-reduce would leave the summation order to the ring schedule) and runs the rest of the
    layer there: damping with nsamples = Σ rows, Cholesky inverse, block loops of every W in Ws.
    The result is bit-identical to oracle.quantize_layer_split for the same row split.

    gram_fn(X) -> G, sum_fn(parts (P, m, m)) -> G and layer_fn(Ws, G, nsamples) -> outputs
    default to the libpt2q kernels (engine.gram / sum_partials / quantize_shared); tests on CPU
    (gloo) substitute their own.  Returns layer_fn's outputs on dst, None elsewhere."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if gram_fn is None or sum_fn is None or layer_fn is None:
        from . import engine
        gram_fn = gram_fn or engine.gram
        sum_fn = sum_fn or engine.sum_partials

        def _layer(Ws_, G, nsamples):
            return engine.quantize_shared(Ws_, G, nsamples, block_size, use_ssr, percdamp, max_iter)
        layer_fn = layer_fn or _layer
    X2 = X_local.reshape(-1, X_local.shape[-1])
    m = X2.shape[1]
    dev = X2.device
    rows = torch.tensor([X2.shape[0]], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(rows, group=group)  # exact integer sum: nsamples of main.py:129
    nsamples = int(rows.item())
    if rank != dst:
        G = gram_fn(X2).contiguous()
        dist.send(G, dst=dst, group=group)
        return None
    parts = torch.empty((world, m, m), dtype=torch.float32, device=dev)
    ops = [dist.P2POp(dist.irecv, parts[r], r, group) for r in range(world) if r != dst]
    reqs = dist.batch_isend_irecv(ops) if ops else []
    parts[dst].copy_(gram_fn(X2))
    for req in reqs:
        req.wait()
    G = sum_fn(parts)
    return layer_fn(list(Ws), G, nsamples)


class GramsFirst:
    """The step schedule for independent units whose activations are all at hand (synthetic or
    pre-captured; within one decoder layer of the real flow, calibration.quantize_decoder_layer):

    1. every unit's Gram back to back on the caller's stream, each into its slot of a packed
       (units, m, m) raw-Gram buffer per (width, rows) group (Σ m² fp32: 21.7 GB for Llama-2-7B);
    2. (batched=True) every group's damped Hessian inverses by engine.hessian_inverse_batched:
       each step of the blocked Cholesky factorisation serves all units of a chunk in one launch,
       instead of 64-172 latency-bound steps per unit;
    3. the units' block loops on the lanes of an engine.UnitPipeline (with batched=False the
       lanes also run each unit's own damping and Cholesky inverse).

    A Gram holds every CU for its whole duration, so interleaving the Grams with other units'
    tails only stalls those tails; keeping the phases apart measured 2.80 s against 2.95 s per 7B
    step.  Results are bit-identical to any other order.

    Stall reporting: the Grams of one width share a workspace, and every pt2q_gram call zeroes
    its status word first, so after each Gram its word is OR-ed (on the stream) into one
    per-step device word; check() reads that word once and clears it.

    Per-channel groups (block size >= m: one block per linear) get no inverse at all -- H⁻¹
    feeds only the error feedback (main.py:198-214), which a single block never reaches -- so
    neither the Hinv buffer nor the batched factorisation exists for them (as pt2q_quantize_layer).

    The damping is the pipeline's (pipe.percdamp) everywhere: batched inverses, the per-lane
    inverses of batched=False and the pinv fallback, so no path damps differently."""

    def __init__(self, pipe, device, batched: bool = True, chunk=None, group: int = 16,
                 overlap: bool = False, batch_grams: bool = True, inv_streams: int = 1, spread: bool = True):
        from . import engine, _lib
        self.engine, self.lib, self.pipe, self.dev = engine, _lib, pipe, torch.device(device)
        # step 1 batched: the Grams of each (m, N) group in data-parallel launches
        # (pt2q_gram_batched) instead of one stream-K launch per unit
        self.batch_grams, self.pending = batch_grams, {}
        # chunk: items per batched-inverse launch sequence, an int or {m: items} (others: 32), or
        # None: 32, or the whole batch when small (_chunk)
        self.batched, self.chunk = batched, chunk
        # step 3 grouped: the block loops of up to `group` same-shape linears (across units) per
        # pt2q_quantize_blocks_group launch sequence, groups spread over the pipeline's lanes
        self.group = group if batched else 0
        self.grouped = self.group > 1
        # spread: a shape class of k linears that fits one group (k <= group) is ONE group -- its
        # block chain is latency-bound, and one launch sequence over k linears costs little more
        # than one over k / lanes (GPT-2: 15.9 -> 15.3 ms) -- and a larger class is cut into groups
        # of ceil(k / lanes) (at most `group`) so every lane gets an even share (C5's 40 down_proj:
        # 14 / 14 / 12, not 16 / 16 / 8: 107.7 -> 106.0 ms).  False: groups of `group`.
        self.spread = spread
        self.gws = {}
        # overlap=True: the batched inverses run on a stream of their own, one event per (m, N)
        # group, and a unit's block loops wait only for its own width's inverses, so the narrow
        # units' loops overlap the wide units' inverses (measured slower on the 7B step, 2.816
        # vs 2.771 s: both phases fill the CUs)
        self.inv_stream = (torch.cuda.Stream(self.dev, priority=-1) if batched and overlap and self.dev.type == "cuda"
                           else None)
        self.inv_done = {}
        # inv_streams > 1 (without overlap): the batched inverse chunks of all widths spread over
        # that many streams (longest first, least-loaded stream), so one chunk's latency-bound
        # panel steps run beside another chunk's MFMA-bound trailing updates; each stream has its
        # own scratch, and the caller's stream joins them all before any tail
        self.inv_streams = max(1, int(inv_streams))
        self._istreams, self._iscratch = [], []
        self.G, self.ws = {}, {}
        self.slot = {}       # key -> (group, index)
        self.groups = {}     # (m, N) -> {"G", "Hinv", "info"} packed over the group's units
        self.scratch = {}
        self.ows = {}        # per-lane workspaces of the per-linear ("one") block loops
        self.stall = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._s1_streams = []  # per-channel S1 / d, one stream per width (inverses())
        self.s1_done = {}      # per-channel group -> event: its S1 / d formed

    @property
    def percdamp(self):
        return self.pipe.percdamp

    # a width whose whole batch of H copies fits in this many bytes is factorised as ONE chunk:
    # each chunk walks the full m / 64-step panel chain, so a short remainder chunk (GPT-2's 36
    # m = 768 items: 32 + 4) costs a second chain for little work
    ONE_CHUNK_BYTES = 4 << 30

    def _chunk(self, m: int, count: int = 0) -> int:
        """Items per batched-inverse launch sequence: chunk as given (int or {m: items}), or with
        chunk=None ("auto") 32 -- the whole batch as one chunk when its H copies fit
        ONE_CHUNK_BYTES."""
        if isinstance(self.chunk, dict):
            return int(self.chunk.get(m, 32))
        if self.chunk is not None:
            return int(self.chunk)
        if count > 32 and count * m * m * 4 <= self.ONE_CHUNK_BYTES:
            return count
        return 32

    def needs_inverse(self, m: int) -> bool:
        return self.engine.needs_inverse(m, self.pipe.bs)

    def begin(self, units):
        """Slots for this step's units [(key, m, N)]: one packed buffer per (m, N) group,
        reused while the step's shape does not change."""
        count = {}
        self.slot = {}
        if self.dev.type == "cuda":
            self.join_side()  # a previous step's S1 / d still reading the buffers reused below
        for key, m, N in units:
            g = (m, int(N))
            self.slot[key] = (g, count.get(g, 0))
            count[g] = count.get(g, 0) + 1
        for g, c in count.items():
            have = self.groups.get(g)
            m = g[0]
            inv = self.batched and self.needs_inverse(m)
            # per-channel groups (no inverse): S1 / d of every Gram, formed once in inverses()
            # and shared by the unit's linears (pt2q_s1_from_gram_batched, PT2Q_FLAG_S1_GIVEN)
            s1 = self.batched and not self.needs_inverse(m) and m > 512
            if have is None or have["G"].shape[0] != c or (have["Hinv"] is not None) != inv or \
                    (have.get("S1d") is not None) != s1:
                self.groups[g] = {"G": torch.empty((c, m, m), dtype=torch.float32, device=self.dev),
                                  "Hinv": torch.empty((c, m, m), dtype=torch.float32, device=self.dev)
                                  if inv else None,
                                  "S1d": torch.empty((c, m + 1), dtype=torch.float32, device=self.dev)
                                  if s1 else None,
                                  "info": torch.zeros(c, dtype=torch.int32, device=self.dev), "upper": False}
        for g in [g for g in self.groups if g not in count]:
            del self.groups[g]
        self.G = {}

    def _gbuf(self, key, m):
        if key in self.slot:
            g, z = self.slot[key]
            return self.groups[g]["G"][z]
        if key not in self.G or self.G[key].shape[0] != m:  # no begin(): a buffer of its own
            self.G[key] = torch.empty((m, m), dtype=torch.float32, device=self.dev)
        return self.G[key]

    def gram(self, key, X):
        X2 = X.reshape(-1, X.shape[-1])
        m = X2.shape[1]
        if self.batch_grams and key in self.slot and self.engine.gram_batched_supported(X2):
            g, z = self.slot[key]
            self.pending.setdefault(g, []).append((z, X2))  # issued by flush()
            return
        if m not in self.ws:
            self.ws[m] = self.lib.workspace(self.lib.lib().pt2q_gram_workspace_bytes(m), self.dev)
        self.engine.gram(X2, G=self._gbuf(key, m), workspace=self.ws[m], check=False)
        torch.bitwise_or(self.stall, self.lib.status_view(self.ws[m]), out=self.stall)

    def set_gram(self, key, G: torch.Tensor):
        """A unit's raw Gram formed elsewhere (calibration.GramAccumulator): copied into its slot
        on the current stream (begin() first)."""
        g, z = self.slot[key]
        self.groups[g]["G"][z].copy_(G)

    def flush(self):
        """Issue the batched Grams gram() collected: one pt2q_gram_batched sequence per group
        whose every slot is pending (else per item)."""
        for g, items in self.pending.items():
            items.sort(key=lambda t: t[0])
            grp = self.groups[g]
            if [z for z, _ in items] == list(range(grp["G"].shape[0])) and \
                    len({(X.shape, X.dtype) for _, X in items}) == 1:
                # a per-channel group's Grams feed only S1 / d: their upper triangles suffice
                # (pt2q_gram_batched_upper; inverses() then reads them with s1 upper_only)
                X0 = items[0][1]
                grp["upper"] = (grp.get("S1d") is not None and X0.dtype in (torch.float16, torch.bfloat16)
                                and X0.shape[1] % 4 == 0)
                self.engine.gram_batched([X for _, X in items], grp["G"], upper_only=grp["upper"])
            else:
                grp["upper"] = False
                m = grp["G"].shape[1]
                if m not in self.ws:
                    self.ws[m] = self.lib.workspace(self.lib.lib().pt2q_gram_workspace_bytes(m), self.dev)
                for z, X in items:
                    self.engine.gram(X, G=grp["G"][z], workspace=self.ws[m], check=False)
                    torch.bitwise_or(self.stall, self.lib.status_view(self.ws[m]), out=self.stall)
        self.pending = {}

    def inverses(self):
        """Step 2: every group's Hessian inverses, batched (no-op with batched=False), narrowest
        width first, on the inverse stream; each group records its event.  Per-channel groups
        (no Hinv buffer, see needs_inverse) are skipped: their info words stay 0."""
        if not self.batched:
            return
        caller = torch.cuda.current_stream(self.dev)
        # per-channel groups: S1 / d once per Gram, each width's launch pair on a side stream of its
        # own with an event (s1_done): a lane's per-channel block loops wait for their width's S1 /
        # d only (_wait_inverse), so the narrow widths' loops start while a wider width's S1 runs --
        # each pair ends in serial d chains and a partial last wave.  Bit-identical either way.
        s1g = [g for g in sorted(self.groups) if self.groups[g].get("S1d") is not None]
        self.s1_done = {}
        if s1g and self.dev.type == "cuda":
            while len(self._s1_streams) < len(s1g):
                self._s1_streams.append(torch.cuda.Stream(self.dev))
            for k, g in enumerate(s1g):
                grp = self.groups[g]
                st = self._s1_streams[k]
                st.wait_stream(caller)  # the Grams
                with torch.cuda.stream(st):
                    self.engine.s1_from_gram_batched(grp["G"], out=grp["S1d"], upper_only=grp.get("upper", False))
                ev = torch.cuda.Event()
                ev.record(st)
                self.s1_done[g] = ev
        else:
            for g in s1g:
                grp = self.groups[g]
                self.engine.s1_from_gram_batched(grp["G"], out=grp["S1d"], upper_only=grp.get("upper", False))
        self.inv_done = {}
        live = [g for g in sorted(self.groups) if self.groups[g]["Hinv"] is not None]
        if self.inv_stream is None and self.inv_streams > 1 and self.dev.type == "cuda":
            jobs = []
            for g in live:
                c = self.groups[g]["G"].shape[0]
                ch = self._chunk(g[0], c)
                jobs += [(float(g[0]) ** 3 * min(ch, c - z0), g, z0, min(ch, c - z0)) for z0 in range(0, c, ch)]
            jobs.sort(key=lambda j: (-j[0], j[1], j[2]))
            while len(self._istreams) < min(self.inv_streams, len(jobs)):
                self._istreams.append(torch.cuda.Stream(self.dev))
                self._iscratch.append({})
            load = [0.0] * len(self._istreams)
            for cost, g, z0, k in jobs:
                si = min(range(len(load)), key=lambda i: (load[i], i))
                load[si] += cost
                st = self._istreams[si]
                st.wait_stream(caller)  # the Grams
                grp = self.groups[g]
                with torch.cuda.stream(st):
                    self.engine.hessian_inverse_batched(grp["G"][z0:z0 + k], g[1], self.percdamp,
                                                        Hinv=grp["Hinv"][z0:z0 + k], info=grp["info"][z0:z0 + k],
                                                        scratch=self._iscratch[si], chunk=k)
            for st in self._istreams:
                caller.wait_stream(st)
            return
        if self.inv_stream is None:  # no overlap: on the caller's stream, before any tail
            for g in live:
                grp = self.groups[g]
                self.engine.hessian_inverse_batched(grp["G"], g[1], self.percdamp, Hinv=grp["Hinv"],
                                                    info=grp["info"], scratch=self.scratch,
                                                    chunk=self._chunk(g[0], grp["G"].shape[0]))
            return
        self.inv_stream.wait_stream(caller)  # the Grams
        with torch.cuda.stream(self.inv_stream):
            for g in live:
                grp = self.groups[g]
                self.engine.hessian_inverse_batched(grp["G"], g[1], self.percdamp, Hinv=grp["Hinv"],
                                                    info=grp["info"], scratch=self.scratch,
                                                    chunk=self._chunk(g[0], grp["G"].shape[0]))
                ev = torch.cuda.Event()
                ev.record(self.inv_stream)
                self.inv_done[g] = ev

    def _wait_inverse(self, stream, key):
        """`stream` waits for the inverses -- or the per-channel S1 / d -- of `key`'s group."""
        if self.batched and key in self.slot:
            g = self.slot[key][0]
            for ev in (self.inv_done.get(g), self.s1_done.get(g)):
                if ev is not None:
                    stream.wait_event(ev)

    def join_side(self):
        """The caller's stream waits for the side streams (per-channel S1 / d)."""
        caller = torch.cuda.current_stream(self.dev)
        for st in self._s1_streams:
            caller.wait_stream(st)

    def tail(self, key, Ws, nsamples):
        if key in self.slot:
            g, z = self.slot[key]
            grp = self.groups[g]
            if self.batched and grp["Hinv"] is not None:
                self._wait_inverse(torch.cuda.current_stream(self.dev), key)
                return self.pipe.run(Ws, G=grp["G"][z], nsamples=nsamples, Hinv=grp["Hinv"][z],
                                     info=grp["info"][z:z + 1])
            return self.pipe.run(Ws, G=grp["G"][z], nsamples=nsamples)
        return self.pipe.run(Ws, G=self.G[key], nsamples=nsamples)

    def tails(self, jobs):
        """Step 3, grouped: jobs [(key, [W], nsamples)] in unit order.  Every linear whose shape
        the grouped entry takes joins a group of same-shape, same-dtype linears (in job order, at
        most `group` per group); groups go round-robin onto the pipeline's lanes.  Returns one
        run per job (finish() -> [LayerOutput]); results are bit-identical to tail()."""
        eng, lib = self.engine, self.lib
        bs, ssr, mi = self.pipe.bs, self.pipe.use_ssr, self.pipe.max_iter
        flags = (lib.FLAG_SSR if ssr else 0) | lib.AGA_ACT
        state = _GroupState(self)
        runs = []
        classes = {}
        for j, (key, Ws, N) in enumerate(jobs):
            g, z = self.slot[key]
            grp = self.groups[g]
            Ws = [eng._float_input(W) for W in Ws]
            run = _GroupedRun(state, key, Ws, grp["G"][z], N, grp["info"][z:z + 1])
            runs.append(run)
            state.runs.append(run)
            Hz = grp["Hinv"][z] if grp["Hinv"] is not None else None  # None: per-channel, never read
            S1z = grp["S1d"][z] if grp.get("S1d") is not None else None  # per-channel: S1 / d formed
            for k, W in enumerate(Ws):
                n, m = W.shape
                if eng.group_supported(n, m, bs, flags):
                    classes.setdefault((n, m, W.dtype), []).append((run, k, W, grp["G"][z], Hz))
                elif S1z is not None and eng.perchannel_group_supported(m):
                    # per-channel (one block) with its Gram's S1 / d formed: grouped by width and
                    # dtype whatever the row count (pt2q_quantize_perchannel_group)
                    classes.setdefault(("pc", m, W.dtype), []).append((run, k, W, grp["G"][z], Hz, S1z))
                else:  # a lone linear of an unsupported shape: its own loop on the next lane
                    classes.setdefault(("one", j, k), []).append((run, k, W, grp["G"][z], Hz, S1z))
        caller = torch.cuda.current_stream(self.dev)
        lanes = self.pipe.lanes
        # groups: at most `group` linears, and small enough that every lane gets work; issued
        # longest first onto the least-loaded lane (LPT on the block-loop cost model)
        plan = []
        for ckey, items in classes.items():
            cap = eng.PC_GROUP_MAX if ckey[0] == "pc" else self.group
            k = len(items)
            size = max(1, k if k <= cap else (min(cap, -(-k // len(lanes))) if self.spread else cap))
            for c0 in range(0, len(items), size):
                chunk = items[c0:c0 + size]
                cost = sum(block_loop_cost(c[2].shape[0], c[2].shape[1], bs) if ckey[0] != "pc"
                           else c[2].shape[0] * c[2].shape[1] * SHARD_MODEL["loop_pc"] for c in chunk)
                plan.append((cost, ckey, chunk))
        plan.sort(key=lambda x: -x[0])
        load = [0.0] * len(lanes)
        for cost, ckey, chunk in plan:
            li = min(range(len(lanes)), key=lambda i: (load[i], i))
            load[li] += cost
            ln = lanes[li]
            ln.stream.wait_stream(caller)
            for key in {c[0].key for c in chunk}:
                self._wait_inverse(ln.stream, key)
            with torch.cuda.stream(ln.stream):
                if ckey[0] == "pc":  # one launch sequence over the chunk's rows (lane workspace)
                    nbytes = lib.lib().pt2q_quantize_perchannel_group_workspace_bytes(eng.PC_GROUP_MAX)
                    okey = ("pc", id(ln))
                    if okey not in self.ows:
                        self.ows[okey] = lib.workspace(nbytes, self.dev)
                    ws = self.ows[okey]
                    outs = eng.quantize_perchannel_group([c[2] for c in chunk], [c[5] for c in chunk], mi,
                                                         workspace=ws, check=False)
                    state.statuses.append(lib.status_view(ws).clone())
                    for (run, k, _, _, _, _), out in zip(chunk, outs):
                        run.outs[k] = out
                    continue
                if ckey[0] == "one":  # stream-ordered like a group: lane workspace, status read in finish()
                    run, k, W, G, H, S1z = chunk[0]
                    n, m = W.shape
                    nbytes = eng.blocks_workspace_bytes(n, m, bs, flags)
                    okey = (id(ln), W.device)
                    if okey not in self.ows or self.ows[okey].numel() < nbytes:
                        self.ows[okey] = lib.workspace(nbytes, self.dev)
                    ws = self.ows[okey]
                    run.outs[k] = eng.quantize_blocks(W, G, H, bs, ssr, lib.AGA_ACT, mi, workspace=ws, check=False,
                                                      s1d=S1z)
                    state.statuses.append(lib.status_view(ws).clone())
                    continue
                n, m, _ = ckey
                wkey = (id(ln), n, m)
                nbytes = lib.lib().pt2q_quantize_blocks_group_workspace_bytes(len(chunk), n, m, bs, flags)
                if wkey not in self.gws or self.gws[wkey].numel() < nbytes:
                    self.gws[wkey] = lib.workspace(
                        lib.lib().pt2q_quantize_blocks_group_workspace_bytes(self.group, n, m, bs, flags), self.dev)
                ws = self.gws[wkey]
                outs = eng.quantize_blocks_group([c[2] for c in chunk], [c[3] for c in chunk],
                                                 [c[4] for c in chunk], bs, ssr, lib.AGA_ACT, mi,
                                                 workspace=ws, check=False)
                state.statuses.append(lib.status_view(ws).clone())
                for (run, k, _, _, _), out in zip(chunk, outs):
                    run.outs[k] = out
        state.join = lambda: [caller.wait_stream(x) for x in [ln.stream for ln in lanes] + self._s1_streams +
                              ([self.inv_stream] if self.inv_stream is not None else [])]
        return runs

    def check(self):
        """Raise if any Gram since the last check stalled in a stream-K hand-off (one host read)."""
        status = int(self.stall.item())
        self.stall.zero_()
        self.lib.raise_stall(status, "pt2q_gram")


class _GroupState:
    """The device words of one grouped tail phase -- every block-loop stall word and every
    unit's Cholesky info word -- read in ONE host read by the first finish()."""

    def __init__(self, gf):
        self.gf, self.statuses, self.runs, self.join, self.read = gf, [], [], None, None

    def read_once(self):
        if self.read is not None:
            return
        if self.join is not None:
            self.join()
        words = torch.cat([s.reshape(1) for s in self.statuses] +
                          [r.info.reshape(1) for r in self.runs]).cpu().tolist()
        ns = len(self.statuses)
        for v in words[:ns]:
            self.gf.lib.raise_stall(int(v), "pt2q_quantize_blocks_group")
        for r, v in zip(self.runs, words[ns:]):
            r.info_val = int(v)
        self.read = True


class _GroupedRun:
    """One unit's outputs from GramsFirst.tails: finish() joins the lanes, reads every group's
    stall word and every unit's Cholesky status once (the first call, _GroupState.read_once),
    and re-runs this unit with pinv (main.py:140-141) if its Hessian was not positive definite
    (never for per-channel units: they have no inverse, and nothing would read one)."""

    def __init__(self, state, key, Ws, G, nsamples, info):
        self.state, self.key, self.Ws, self.G, self.N, self.info = state, key, Ws, G, nsamples, info
        self.outs = [None] * len(Ws)
        self.spd = None
        self.info_val = None

    def finish(self):
        if self.spd is not None:
            return self.outs
        self.state.read_once()
        self.spd = self.info_val == 0
        if not self.spd:
            gf = self.state.gf
            eng, pipe = gf.engine, gf.pipe
            H, _ = eng.prepare_hessian(self.G, self.N, gf.percdamp)
            Hinv = torch.linalg.pinv(H)
            self.outs = [eng.quantize_blocks(W, self.G, Hinv, pipe.bs, pipe.use_ssr, eng._lib.AGA_ACT,
                                             pipe.max_iter) for W in self.Ws]
        for o in self.outs:
            o.spd = self.spd
        return self.outs
