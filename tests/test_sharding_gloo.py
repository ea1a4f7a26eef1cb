"""Multi-process (world_size 2, gloo on CPU) coverage of the layer-sharded path: LPT assignment
and the gather of per-rank results to rank 0 (bench.py's N>1 step uses the same helpers over
RCCL)."""
import os
import socket
import zlib

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (path setup)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharding():
    import importlib.util
    path = os.path.join(ROOT, "snlp---tenary-post-train-quantization_amd", "sharding.py")
    spec = importlib.util.spec_from_file_location("pt2q_sharding_cpu", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_lpt_assignment_balances_llama_units():
    sh = _sharding()
    units = sh.llama_units(32)
    costs = [sh.unit_cost(u) for u in units]
    for world in (1, 2, 4, 8):
        shards = sh.assign_lpt(costs, world)
        assert sorted(i for s in shards for i in s) == list(range(len(units)))
        loads = [sum(costs[i] for i in s) for s in shards]
        assert max(loads) <= 1.05 * (sum(costs) / world) + max(costs)
        # deterministic
        assert shards == sh.assign_lpt(costs, world)
    # linears sharing an input are one unit (one Gram / Cholesky)
    assert [p for p, _, _ in units[0][1]] == ["q_proj", "k_proj", "v_proj"]


def _worker_empty_dst(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = _sharding()
    res = {}
    if rank == 1:  # only the sender holds results: dst must still size its receive buffers
        gen = torch.Generator().manual_seed(5)
        res = {"u.p": {"alpha": torch.rand((16, 2), generator=gen), "perm": torch.randperm(40, generator=gen)}}
    out = sh.gather_results(res, dst=0)
    if rank == 0:
        q.put({k: {f: t.numpy().copy() for f, t in v.items()} for k, v in out.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_results_dst_without_results_world2():
    """dst holding no results of its own receives into buffers on a valid device
    (gloo: CPU) instead of on the device of an empty flat tensor."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_empty_dst, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=90)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    gen = torch.Generator().manual_seed(5)
    assert torch.equal(torch.from_numpy(got["u.p"]["alpha"]), torch.rand((16, 2), generator=gen))
    assert torch.equal(torch.from_numpy(got["u.p"]["perm"]), torch.randperm(40, generator=gen))


class _FakeOut:
    """A LayerOutput stand-in (CPU): deterministic from (n, m, seed)."""

    def __init__(self, n, m, seed, bs=128):
        g = torch.Generator().manual_seed(seed)
        B = -(-m // bs)
        self.alpha = torch.rand((n, B), generator=g)
        self.mu = torch.rand((n, B), generator=g)
        self.T = (torch.randint(0, 3, (n, m), generator=g) - 1).to(torch.int8)
        self.perm = torch.randperm(m, generator=g)


def _mixed_units():
    # qkv-like (3 x 64x48), o-like, gate/up-like (2 x 96x48) and down-like (48x96) units:
    # heterogeneous shapes and linear counts per unit
    return [("l0.qkv", [("q_proj", 64, 48), ("k_proj", 64, 48), ("v_proj", 64, 48)], 256),
            ("l0.o", [("o_proj", 64, 48)], 256),
            ("l0.gate_up", [("gate_proj", 96, 48), ("up_proj", 96, 48)], 256),
            ("l0.down", [("down_proj", 48, 96)], 256),
            ("l1.down", [("down_proj", 48, 96)], 256)]


def _fake_run(units):

    def provider(unit):
        name, lins, _ = unit
        return None, {p: (name, p, n, m) for p, n, m in lins}

    def run_unit(Ws, X):
        return [_FakeOut(n, m, zlib.crc32(f"{name}.{p}".encode()) % 10007) for (name, p, n, m) in Ws]
    return provider, run_unit


def _worker_mixed(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = _sharding()
    units = _mixed_units()
    provider, run_unit = _fake_run(units)
    res, mine = sh.quantize_units_sharded(units, provider, run_unit=run_unit, pack=False, dst=0)
    q.put(("mine", rank, mine))
    if rank == 0:
        # numpy copies: tensors shared through the queue would need this process alive
        q.put(("res", 0, {k: {f: t.numpy().copy() for f, t in v.items()} for k, v in res.items()}))
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_sharded_units_heterogeneous_gather_world2():
    """quantize_units_sharded over 2 gloo ranks with mixed unit shapes (qkv-like 3 x 64x48,
    gate/up-like, down-like 48x96): every linear's result reaches rank 0 intact, each unit runs
    on exactly one rank (the LPT shard), and the shapes ride along in the manifest."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_mixed, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    mine = {}
    for _ in range(3):
        kind, r, v = q.get(timeout=90)
        if kind == "res":
            got = v
        else:
            mine[r] = v
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    units = _mixed_units()
    sh = _sharding()
    assert sorted(mine[0] + mine[1]) == list(range(len(units)))
    assert mine == {r: s for r, s in enumerate(sh.assign_lpt([sh.unit_cost(u) for u in units], 2))}
    want_names = {f"{name}.{p}" for name, lins, _ in units for p, _, _ in lins}
    assert set(got) == want_names
    for name, lins, _ in units:
        for p, n, m in lins:
            ref = _FakeOut(n, m, zlib.crc32(f"{name}.{p}".encode()) % 10007)
            r = {f: torch.from_numpy(a) for f, a in got[f"{name}.{p}"].items()}
            assert r["T"].dtype == torch.int8 and tuple(r["T"].shape) == (n, m)
            assert torch.equal(r["T"], ref.T) and torch.equal(r["perm"], ref.perm)
            assert torch.equal(r["alpha"], ref.alpha) and torch.equal(r["mu"], ref.mu)
            assert r["shape"].tolist() == [n, m]
    assert sh.units_cols(units) == 3 * 48 + 48 + 2 * 48 + 96 + 96


def test_flatten_roundtrip_cpu():
    sh = _sharding()
    res = {"b": {"x": torch.arange(6, dtype=torch.int64).reshape(2, 3), "e": torch.empty(0)},
           "a": {"y": torch.tensor([1.5, -2.0]), "z": torch.tensor([[1, -1]], dtype=torch.int8)}}
    man, flat = sh._flatten(res)
    back = sh._unflatten(man, flat)
    for k, v in res.items():
        for f, t in v.items():
            assert back[k][f].dtype == t.dtype and torch.equal(back[k][f], t)


# ----------------------------------------------------------------- intra-layer split (§8e(ii))

def _worker_split(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import numpy as np
    import synth
    from oracle import oracle as orc
    sh = _sharding()
    N, m = 203, 48  # ragged row split: 67 / 68 / 68
    X = synth.activations(77, N, m).astype(np.float16)
    lo, hi = sh.row_slice(N, rank, world)
    calls = []

    def gram_fn(Xr):
        calls.append(Xr.shape[0])
        return torch.from_numpy(orc.gram16(Xr.numpy()))

    def sum_fn(parts):
        return torch.from_numpy(orc.sum_partials([p.numpy() for p in parts]))

    def layer_fn(Ws, G, nsamples):
        return {"G": G.numpy().copy(), "nsamples": nsamples, "Ws": Ws}

    out = sh.quantize_layer_split(["w"], torch.from_numpy(X[lo:hi]), dst=0, gram_fn=gram_fn,
                                  sum_fn=sum_fn, layer_fn=layer_fn)
    q.put(("rows", rank, calls))
    if rank == 0:
        q.put(("out", 0, out))
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_layer_split_rank_ordered_gram_world3():
    """Each rank forms the Gram of its calibration rows; dst folds the partials in rank order and
    runs the layer with nsamples = all rows (oracle.quantize_layer_split's G)."""
    import numpy as np
    import synth
    from oracle import oracle as orc
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_split, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=90) for _ in range(world + 1)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rows = {r: c for k, r, c in got if k == "rows"}
    out = [v for k, _, v in got if k == "out"][0]
    N, m = 203, 48
    assert rows == {r: [hi - lo] for r, (lo, hi) in enumerate(orc.row_slices(N, world))}
    assert out["nsamples"] == N and out["Ws"] == ["w"]
    X = synth.activations(77, N, m).astype(np.float16)
    ref = orc.sum_partials([orc.gram16(X[a:b]) for a, b in orc.row_slices(N, world)])
    assert np.array_equal(out["G"], ref)


def test_oracle_split_one_rank_is_the_layer():
    """oracle.quantize_layer_split with one rank is quantize_layer_m; with several ranks its G is
    the rank-ordered fold of the slices' Grams (a different rounding, same matrix to ~1e-6)."""
    import numpy as np
    import synth
    from oracle import oracle as orc
    W = synth.weights(31, 64, 96)
    X = synth.activations(32, 300, 96)
    a, b = orc.quantize_layer_split(W, X, 1), orc.quantize_layer_m(W, X)
    for k in ("T", "perm", "alpha", "mu"):
        assert np.array_equal(a[k], b[k])
    G3 = orc.quantize_layer_split(W, X, 3)["G"]
    G1 = orc.gram(X)
    assert np.allclose(G3, G1, rtol=1e-5, atol=1e-3)


def test_grams_first_orders_phases_single_process():
    """quantize_units_sharded(grams_first=...) forms every unit's Gram before any tail, keeps
    the per-unit pairing, and returns the same result dict as the per-unit path."""
    sh = _sharding()
    units = _mixed_units()
    provider, run_unit = _fake_run(units)
    log = []

    class FakeGF:
        def gram(self, key, X):
            log.append(("gram", key))

        def tail(self, key, Ws, N):
            log.append(("tail", key))
            return run_unit(Ws, None)

    got, mine = sh.quantize_units_sharded(units, provider, pack=False, grams_first=FakeGF())
    want, _ = sh.quantize_units_sharded(units, provider, run_unit=run_unit, pack=False)
    kinds = [k for k, _ in log]
    assert kinds == ["gram"] * len(mine) + ["tail"] * len(mine)
    assert [i for _, i in log[:len(mine)]] == [i for _, i in log[len(mine):]] == mine
    assert got.keys() == want.keys()
    for k in got:
        for f in got[k]:
            assert torch.equal(got[k][f], want[k][f])


# ----------------------------------------------------------------- bench.py rank plumbing

def _last_json(text):
    import json
    for line in reversed(text.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError("no JSON line in bench output:\n" + text[-2000:])


@pytest.mark.timeout(180)
def test_bench_gpus2_launches_two_ranks_dry_run():
    """`python bench.py --gpus 2` (no WORLD_SIZE) starts two ranks itself; each runs exactly its
    LPT shard of the model's units, rank 0 gathers every linear and prints ONE JSON line with
    n_gpus from the process group (--dry-run: gloo, stub units)."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    args = ["--layers", "2", "--hidden", "64", "--inter", "96", "--tokens", "256", "--steps", "2",
            "--warmup", "1", "--dry-run"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args,
                       capture_output=True, text=True, timeout=170, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    assert sum(1 for l in p.stdout.splitlines() if l.startswith("{")) == 1
    d = _last_json(p.stdout)
    sh = _sharding()
    units = sh.llama_units(2, 64, 96, 256)
    shards = sh.assign_lpt([sh.unit_cost(u) for u in units], 2)
    assert d["n_gpus"] == 2 and len(d["ranks"]) == 2
    for r in d["ranks"]:
        want = sorted(f"{units[i][0]}.{p}" for i in shards[r["rank"]] for p, _, _ in units[i][1])
        assert r["ran"] == want and r["units"] == len(shards[r["rank"]])
    assert d["gathered_linears"] == sorted(f"{n}.{p}" for n, lins, _ in units for p, _, _ in lins)
    assert d["config"]["weight_columns_per_step"] == sh.units_cols(units)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,linears", [("llama-2-7b", 224), ("llama-2-13b", 280)])
def test_bench_gpus8_dry_run_full_models(model, linears):
    """The driver's 8-GPU run, rehearsed on CPU: `bench.py --gpus 8 --model M --dry-run` with the
    model's full unit list (C4: 128 units / 224 linears; C5: 160 / 280).  Every rank runs its LPT
    shard, rank 0 gathers every linear, and the modelled makespan (max / mean rank cost) is <= 1.10."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    args = ["--model", model, "--steps", "1", "--warmup", "0", "--dry-run"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"] + args,
                       capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _last_json(p.stdout)
    sh = _sharding()
    units = sh.model_units(model)
    bs = sh.MODELS[model]["block_size"]
    assert d["n_gpus"] == 8 and len(d["ranks"]) == 8
    assert len(d["gathered_linears"]) == linears == sum(len(u[1]) for u in units)
    assert d["gathered_linears"] == sorted(f"{n}.{p}" for n, lins, _ in units for p, _, _ in lins)
    shards = sh.assign_lpt([sh.unit_cost(u, bs) for u in units], 8)
    for r in d["ranks"]:
        assert r["units"] == len(shards[r["rank"]])
        want = sum(sh.unit_cost(units[i], bs) for i in shards[r["rank"]])
        assert abs(r["predicted_cost_s"] - want) <= 1e-9 * want
    assert d["lpt_balance"]["predicted_max_over_mean"] <= 1.10
    # the refitted phase model of every rank's step (fixed per-launch latencies included)
    assert d["lpt_balance"]["shard_model_max_over_mean"] <= 1.10
    for r in d["ranks"]:
        want = sh.shard_cost([units[i] for i in shards[r["rank"]]], bs, 2)
        assert abs(r["predicted_shard_s"] - want) <= 1e-9 * want


def test_bench_refuses_gpus_world_size_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run"],
                       capture_output=True, text=True, timeout=60, env=env, cwd=ROOT)
    assert p.returncode == 2 and "refusing" in p.stderr


# ----------------------------------------------------------------- GramsFirst stall reporting

def test_grams_first_keeps_an_early_stall():
    """Grams of one width share a workspace whose status word every pt2q_gram zeroes
    first; a stall in an EARLY Gram must survive the later Grams and raise once at check()."""
    import types

    import pt2q_loader
    pt2q = pt2q_loader.load()  # ctypes load of libpt2q.so works without a GPU
    from pt2q import sharding as sh
    gf = sh.GramsFirst(pipe=None, device="cpu")
    stalls = iter([1, 0, 0])  # the first Gram of the width stalls, the next two do not

    def fake_gram(X, G=None, workspace=None, check=False):
        pt2q._lib.status_view(workspace).fill_(next(stalls))  # take_status zeroes, kernel may set
        return G

    gf.engine = types.SimpleNamespace(gram=fake_gram)
    for k in range(3):
        gf.gram(k, torch.zeros(8, 16))
    with pytest.raises(pt2q._lib.Pt2qError, match="Gram partial-tile"):
        gf.check()
    gf.check()  # cleared after the read


@pytest.mark.parametrize("model,bs,prof", [("llama-2-7b", 128, "r06zi_shards_c4.json"),
                                           ("llama-2-13b", 1 << 14, "r06zi_shards_c5.json")])
def test_shard_model_matches_measured_shards(model, bs, prof):
    """sharding.shard_cost / shard_phases against the one-GPU shard timings of C4 and C5 committed
    under profiles/ (bench.py --gpus 8 --shard all): every shard's step and the whole step within
    10 %, and each modelled phase of the whole step within 10 % of its measured wall."""
    import json
    sh = _sharding()
    with open(os.path.join(ROOT, "profiles", prof)) as f:
        d = json.load(f)
    units = sh.model_units(model)
    shards = sh.assign_lpt([sh.unit_cost(u, bs) for u in units], 8)
    for rec in d["shards"]:
        mine = [units[i] for i in shards[rec["rank"]]]
        assert len(mine) == rec["units"]
        pred = sh.shard_cost(mine, bs) * 1e3
        assert abs(pred - rec["ms_per_step"]) <= 0.10 * rec["ms_per_step"], (rec["rank"], pred, rec["ms_per_step"])
    whole = sh.shard_phases(units, bs)
    assert abs(sum(whole.values()) * 1e3 - d["t1_ms"]) <= 0.10 * d["t1_ms"]
    for k, v in d["t1_phase_s"].items():
        assert abs(whole[k] - v) <= 0.10 * v, (k, whole[k], v)


def test_grams_first_inverse_chunking_policy():
    """GramsFirst._chunk: an explicit chunk (int or {m: items}) is used as given; chunk=None
    (bench --inv-chunk auto) takes 32 items per batched-inverse launch sequence, or the whole
    batch when its H copies fit ONE_CHUNK_BYTES (GPT-2's 36 m = 768 items: one chunk, not 32 + 4;
    the 7B's 96 m = 4096 items: 6.4 GB, three chunks).  Chunking never changes a bit
    (test_hessian_inverse_batched_equals_per_item); this is the schedule only."""
    import pt2q_loader
    pt2q_loader.load()
    from pt2q import sharding as sh
    auto = sh.GramsFirst(pipe=None, device="cpu")
    assert auto._chunk(768, 36) == 36 and auto._chunk(3072, 12) == 32 and auto._chunk(2048, 72) == 72
    assert auto._chunk(4096, 96) == 32 and auto._chunk(11008, 32) == 32 and auto._chunk(768, 0) == 32
    assert sh.GramsFirst(pipe=None, device="cpu", chunk=16)._chunk(768, 36) == 16
    assert sh.GramsFirst(pipe=None, device="cpu", chunk={768: 8})._chunk(768, 36) == 8
