"""Multi-process (world_size 2, gloo on CPU) coverage of the layer-sharded path: LPT assignment
and the gather of per-rank results to rank 0 (bench.py's N>1 step uses the same helpers over
RCCL)."""
import os
import socket

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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = _sharding()
    n, m, B = 16, 40, 2
    gen = torch.Generator().manual_seed(rank)
    T = (torch.randint(0, 3, (n, m), generator=gen) - 1).to(torch.int8)
    flat = (T.flatten() + 1).to(torch.uint8)
    pad = (-flat.numel()) % 4
    flat = torch.cat([flat, torch.zeros(pad, dtype=torch.uint8)]).reshape(-1, 4)
    packed = flat[:, 0] | (flat[:, 1] << 2) | (flat[:, 2] << 4) | (flat[:, 3] << 6)
    res = {"T2": packed, "alpha": torch.full((n, B), float(rank)), "mu": torch.zeros(n, B),
           "perm": torch.randperm(m, generator=gen)}
    out = sh.gather_to_root(res, dst=0)
    if rank == 0:
        q.put({k: [t.clone() for t in v] for k, v in out.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_to_root_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=90)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert len(got["alpha"]) == world
    for r in range(world):
        assert torch.all(got["alpha"][r] == float(r))
        gen = torch.Generator().manual_seed(r)
        torch.randint(0, 3, (16, 40), generator=gen)
        assert torch.equal(got["perm"][r], torch.randperm(40, generator=gen))
