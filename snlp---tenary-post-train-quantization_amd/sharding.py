"""Multi-GPU layer sharding: one process per GPU, independent linears per rank, one gather.

The per-layer loop has no cross-layer dependency once activations are captured, so linears are
independent work units.  Units are assigned longest-processing-time first; linears
that share an input (q/k/v, gate/up) form ONE unit so they share a Gram and a Cholesky.  The only
collective is a gather of the quantised results to the root rank over RCCL/xGMI (backend "nccl"
is RCCL on ROCm) — 2-bit packed codes (utils.py:189-219 layout) plus scales and permutation.
"""
from typing import Dict, List, Sequence

import torch
import torch.distributed as dist


def layer_cost(n: int, m: int, N: int, block_size: int = 128) -> float:
    """Relative cost of one linear: symmetric Gram N·m² + Cholesky/inverse m³ + block loop n·m²."""
    return float(N) * m * m + float(m) ** 3 + float(n) * m * m


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


def unit_cost(unit) -> float:
    _, linears, N = unit
    m = linears[0][2]
    return float(N) * m * m + float(m) ** 3 + sum(float(n) * m * m for _, n, _ in linears)


def gather_to_root(tensors: Dict[str, torch.Tensor], dst: int = 0, group=None):
    """Gather same-shaped tensors from every rank to `dst` (one dist.gather per entry).
    Returns {name: [tensor from rank 0, 1, ...]} on dst, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    out = {} if rank == dst else None
    for name in sorted(tensors):
        t = tensors[name].contiguous()
        bucket = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, bucket, dst=dst, group=group)
        if rank == dst:
            out[name] = bucket
    return out
