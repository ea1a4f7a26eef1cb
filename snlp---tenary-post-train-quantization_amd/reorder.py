"""SSR dynamic block selection on MI355X — reference reorder.py:36-61 and :107-143.

One call = the similarity of every remaining column to the remaining-column mean plus the
ordered top-k (ssr.hip).  Ties (equal similarity) resolve to the lower position in
`remaining_indices`; torch.topk leaves that order unspecified.  CPU inputs (the reference's call
shape) are computed on the current HIP device and returned on the CPU.
"""
from typing import Tuple

import torch

from . import _lib


def _ssr_call(W, remaining_indices, block_size, want_sim):
    dev = _lib.compute_device(W, remaining_indices)  # CPU callers: computed on the GPU
    Wf = W.to(dev).contiguous().float()
    n, m = Wf.shape
    rem = remaining_indices.to(device=dev, dtype=torch.int64).contiguous()
    r = rem.numel()
    bs = min(block_size, r)
    blk = torch.empty(max(bs, 1), dtype=torch.int64, device=dev)
    newrem = torch.empty(max(r - bs, 1), dtype=torch.int64, device=dev)
    sim = torch.empty(r, dtype=torch.float32, device=dev) if want_sim else None
    ws = _lib.workspace(_lib.lib().pt2q_ssr_workspace_bytes(n, m), dev)
    rc = _lib.lib().pt2q_ssr_select(_lib.ptr(Wf), m, n, m, _lib.ptr(rem), r, int(block_size),
                                    _lib.ptr(blk), _lib.ptr(newrem), _lib.ptr(sim), _lib.ptr(ws),
                                    ws.numel(), _lib.stream_of(dev))
    _lib.check(rc, "pt2q_ssr_select")
    return blk[:bs], newrem[: r - bs], sim


def compute_column_similarity_to_mean(W: torch.Tensor, indices: torch.Tensor) -> torch.Tensor:
    """reorder.py:36-61: cosine similarity of each W[:, indices] column to their mean."""
    _, _, sim = _ssr_call(W, indices, 1, True)
    return sim.to(W.device, W.dtype)


def select_next_block_ssr(W: torch.Tensor, remaining_indices: torch.Tensor,
                          block_size: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """reorder.py:107-143: (block_indices in similarity order, new_remaining ascending)."""
    if len(remaining_indices) <= block_size:
        return remaining_indices, torch.tensor([], dtype=remaining_indices.dtype,
                                               device=remaining_indices.device)
    blk, newrem, _ = _ssr_call(W, remaining_indices, block_size, False)
    dt, dv = remaining_indices.dtype, remaining_indices.device
    return blk.to(dv, dt), newrem.to(dv, dt)
