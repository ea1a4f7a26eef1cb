"""Per-layer engine: the GPTQ-style ternary block loop on one MI355X.

Reference: main.py:102-230 (PT2LLMQuantizer.quantize_layer, variant M) and gptq.py:78-199
(GPTQ.quantize, variant G).  The whole layer is one stream-ordered sequence of libpt2q kernels
(Gram -> damping -> Cholesky/inverse -> per block [SSR select -> ATQ -> error feedback]) with no
host synchronisation inside; the host reads one status word at the end to apply the reference's
pinv fallback (main.py:140-141) when the Hessian is not positive definite.
"""
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib


def num_blocks(m: int, block_size: int) -> int:
    return -(-m // block_size) if block_size < m else 1


def _float_input(t):
    _lib.require_device(t)
    t = t.contiguous()
    if t.dtype not in (torch.float32, torch.float16, torch.bfloat16):
        t = t.float()
    return t


@dataclass
class LayerOutput:
    alpha: torch.Tensor   # n x B fp32
    mu: torch.Tensor      # n x B fp32
    T: torch.Tensor       # n x m int8 (or fp32), original column order
    perm: torch.Tensor    # m int64
    iters: torch.Tensor   # B int32 (ITF iterations per block)
    spd: bool = True


def gram(X: torch.Tensor, G: Optional[torch.Tensor] = None, accumulate=False,
         workspace: Optional[torch.Tensor] = None, check: bool = True) -> torch.Tensor:
    """XᵀX (main.py:128), X (N, m) or (B, L, m).

    accumulate=False: G = XᵀX.  True: G = G + XᵀX (gptq.py:75 add_batch).  "continue": every
    entry's fp32 chain resumes from G, so a Gram streamed batch by batch is bit-identical to one
    Gram of the concatenated rows (the captured-and-concatenated X of main.py:293) — for fp16 /
    bf16 activations, whose 16-bit MFMA chain advances in groups of 8 rows, when every batch
    but the last has a multiple of 8 rows (calibration.GramAccumulator carries the remainder
    rows itself, so ragged batches keep the guarantee).

    check=True reads the workspace status word afterwards (one host synchronisation) and raises
    Pt2qError if a stream-K hand-off timed out; check=False leaves that to the caller
    (`_lib.check_status(workspace)`)."""
    X = _float_input(X.reshape(-1, X.shape[-1]))
    N, m = X.shape
    if G is None:
        G = torch.empty((m, m), dtype=torch.float32, device=X.device)
        accumulate = False
    mode = 2 if accumulate == "continue" else int(bool(accumulate))
    ws = workspace
    if ws is None or ws.numel() < _lib.lib().pt2q_gram_workspace_bytes(m):
        ws = _lib.workspace(_lib.lib().pt2q_gram_workspace_bytes(m), X.device)
    _lib.check(_lib.lib().pt2q_gram(_lib.ptr(X), _lib.dtype_code(X), N, m, m, _lib.ptr(G), m,
                                    mode, _lib.ptr(ws), ws.numel(),
                                    _lib.stream_of(X.device)), "pt2q_gram")
    if check:
        _lib.check_status(ws, "pt2q_gram")
    return G


GRAM_BATCH_MAX = 128  # items per pt2q_gram_batched launch


def gram_batched_supported(X: torch.Tensor) -> bool:
    """Whether pt2q_gram_batched takes activations like X (2-D view N x m)."""
    m = X.shape[-1]
    if X.dtype == torch.float32:  # any m: the batched f32 GEMM (gemm.hip gram_f32_batched_kernel)
        return X.is_contiguous()
    return (X.dtype in (torch.float16, torch.bfloat16) and m % 256 == 0 and X.is_contiguous()
            and X.data_ptr() % 16 == 0 and m % 8 == 0)


def gram_batched(Xs, G: torch.Tensor, upper_only: bool = False) -> torch.Tensor:
    """G[z] = Xs[z]ᵀ Xs[z] for every item (main.py:128 per unit) in data-parallel launches of up to
    GRAM_BATCH_MAX items (pt2q_gram_batched): G is a contiguous fp32 (batch, m, m) tensor, the Xs
    fp16 / bf16 (m % 256 == 0) or fp32 (N, m) of one shape.  Each G[z] is bit-identical to
    gram(Xs[z]).  upper_only (16-bit Xs): only the upper triangle (c >= r) is written, the rest of
    G is left as it was (pt2q_gram_batched_upper; for Grams that feed only S1 / d,
    s1_from_gram_batched(upper_only=True))."""
    Xs = [X.reshape(-1, X.shape[-1]) for X in Xs]
    N, m = Xs[0].shape
    if G.shape != (len(Xs), m, m) or G.dtype != torch.float32 or not G.is_contiguous():
        raise ValueError("gram_batched: G must be a contiguous fp32 (batch, m, m) tensor")
    if any(X.shape != (N, m) or X.dtype != Xs[0].dtype or not gram_batched_supported(X) for X in Xs):
        raise _lib.Pt2qError("gram_batched: every X must be a contiguous (N, m) tensor of one dtype "
                             "(16-bit: m % 256 == 0)")
    for z0 in range(0, len(Xs), GRAM_BATCH_MAX):
        chunk = Xs[z0:z0 + GRAM_BATCH_MAX]
        arr, keep = _lib.ptr_array(chunk)
        fn = _lib.lib().pt2q_gram_batched_upper if upper_only else _lib.lib().pt2q_gram_batched
        _lib.check(fn(len(chunk), arr, _lib.dtype_code(chunk[0]), N, m, m, _lib.ptr(G[z0]), _lib.stream_of(G.device)),
                   "pt2q_gram_batched" + ("_upper" if upper_only else ""))
    return G


def sum_partials(parts: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """((parts[0] + parts[1]) + parts[2]) + ... elementwise in fp32, in index order (the
    deterministic rank-ordered reduction of the intra-layer split; out may alias parts[0]).
    parts: (P, ...) fp32, contiguous, on a HIP device."""
    _lib.require_device(parts)
    if parts.dtype != torch.float32 or not parts.is_contiguous():
        raise _lib.Pt2qError("sum_partials: parts must be a contiguous fp32 (P, ...) device tensor")
    P = parts.shape[0]
    count = parts[0].numel()
    if out is None:
        out = torch.empty(parts.shape[1:], dtype=torch.float32, device=parts.device)
    _lib.check(_lib.lib().pt2q_sum_partials(_lib.ptr(parts), count, P, count, _lib.ptr(out),
                                            _lib.stream_of(parts.device)), "pt2q_sum_partials")
    return out


def prepare_hessian(G: torch.Tensor, nsamples: int, percdamp: float = 0.01):
    """H = G / nsamples + percdamp * mean(diag) * I (main.py:129-133, gptq.py:94-98)."""
    m = G.shape[0]
    H = torch.empty_like(G)
    damp = torch.empty(1, dtype=torch.float32, device=G.device)
    _lib.check(_lib.lib().pt2q_prepare_hessian(_lib.ptr(G), m, m, int(nsamples), float(percdamp),
                                               _lib.ptr(H), m, _lib.ptr(damp),
                                               _lib.stream_of(G.device)), "pt2q_prepare_hessian")
    return H, damp


def cholesky_inverse(H: torch.Tensor):
    """cholesky_inverse(cholesky(H)), falling back to pinv like main.py:137-141. -> (Hinv, spd)."""
    m = H.shape[0]
    dev = H.device
    Hinv = torch.empty_like(H)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = _lib.workspace(_lib.lib().pt2q_cholesky_workspace_bytes(m), dev)
    _lib.check(_lib.lib().pt2q_cholesky_inverse(_lib.ptr(H), m, m, _lib.ptr(Hinv), m, _lib.ptr(ws),
                                                ws.numel(), _lib.ptr(info), _lib.stream_of(dev)),
               "pt2q_cholesky_inverse")
    if int(info.item()) != 0:
        return torch.linalg.pinv(H), False
    return Hinv, True


def needs_inverse(m: int, block_size: int) -> bool:
    """Whether the block loop reads H⁻¹: only the error feedback does (main.py:198-214), and a
    single block (per-channel, block_size >= m) leaves no columns to feed back into."""
    return block_size < m


def blocks_workspace_bytes(n: int, m: int, block_size: int, flags: int) -> int:
    return int(_lib.lib().pt2q_blocks_workspace_bytes(n, m, int(block_size), flags))


def quantize_blocks(W: torch.Tensor, A: Optional[torch.Tensor], Hinv: Optional[torch.Tensor],
                    block_size: int = 128, use_ssr: bool = True, aga: int = _lib.AGA_ACT,
                    max_iter: int = 100, t_dtype=torch.int8, workspace: Optional[torch.Tensor] = None,
                    check: bool = True, s1d: Optional[torch.Tensor] = None) -> LayerOutput:
    """The block loop given the AGA matrix A (raw Gram for variant M, damped H for variant G).
    Hinv may be None for a single block (block_size >= m: it is never read).  workspace: reused
    when large enough (pt2q_blocks_workspace_bytes); check=False leaves the status word to the
    caller (`_lib.check_status(workspace)`; no host read here).  s1d: per-channel only (one block,
    m > 512, variant M) -- S1 then d of A from s1_from_gram_batched, formed once per Gram; A is
    then not read (PT2Q_FLAG_S1_GIVEN)."""
    W = _float_input(W)
    n, m = W.shape
    dev = W.device
    B = num_blocks(m, block_size)
    alpha = torch.empty((n, B), dtype=torch.float32, device=dev)
    mu = torch.empty((n, B), dtype=torch.float32, device=dev)
    T = torch.empty((n, m), dtype=t_dtype, device=dev)
    perm = torch.empty(m, dtype=torch.int64, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)  # zeroed by the call (run_blocks)
    flags = (_lib.FLAG_SSR if use_ssr else 0) | aga
    nbytes = blocks_workspace_bytes(n, m, block_size, flags)
    if s1d is not None:
        if aga != _lib.AGA_ACT or block_size < m or m <= 512 or s1d.numel() != m + 1:
            raise ValueError("quantize_blocks: s1d is for one-block (per-channel) variant-M loops, m + 1 floats")
        # the library reads it as m + 1 raw fp32 values on W's device
        if s1d.dtype != torch.float32 or not s1d.is_contiguous() or s1d.device != dev:
            raise ValueError("quantize_blocks: s1d must be a contiguous fp32 tensor on W's device")
        A, flags = s1d, flags | _lib.FLAG_S1_GIVEN
    ws = workspace if workspace is not None and workspace.numel() >= nbytes else _lib.workspace(nbytes, dev)
    if Hinv is None:
        if needs_inverse(m, block_size):
            raise ValueError("quantize_blocks: Hinv is required when block_size < m (error feedback)")
    else:
        Hinv = Hinv.contiguous().float()
    rc = _lib.lib().pt2q_quantize_blocks(
        _lib.ptr(W), _lib.dtype_code(W), m, n, m, int(block_size), flags,
        _lib.ptr(A), m, _lib.ptr(Hinv), m, int(max_iter), _lib.ptr(alpha), _lib.ptr(mu), _lib.ptr(T),
        _lib.dtype_code(T), _lib.ptr(perm), _lib.ptr(iters), _lib.ptr(ws), ws.numel(),
        _lib.stream_of(dev))
    _lib.check(rc, "pt2q_quantize_blocks")
    if check:
        _lib.check_status(ws, "pt2q_quantize_blocks")
    return LayerOutput(alpha, mu, T, perm, iters)


def s1_from_gram_batched(G: torch.Tensor, out: Optional[torch.Tensor] = None, upper_only: bool = False) -> torch.Tensor:
    """S1 = S·1 and d = 1ᵀS1 (quantizer.py:215-218) of every m x m raw Gram in G (batch, m, m) in
    one launch pair: row z of the (batch, m + 1) result is S1 then d of item z, bit-identical to
    pt2q_s1_from_gram per item (quantize_blocks(..., s1d=row) consumes it).  upper_only: read only
    the upper triangle (c >= r) of each Gram -- gram_batched(upper_only=True)'s output -- with the
    same bits (pt2q_s1_from_upper_batched; m > 512, m % 4 == 0)."""
    _lib.require_device(G)
    if G.dim() != 3 or G.shape[1] != G.shape[2] or G.dtype != torch.float32 or not G.is_contiguous():
        raise ValueError("s1_from_gram_batched: G must be a contiguous fp32 (batch, m, m) device tensor")
    b, m = G.shape[0], G.shape[-1]
    if out is None:
        out = torch.empty((b, m + 1), dtype=torch.float32, device=G.device)
    elif (out.shape != (b, m + 1) or out.dtype != torch.float32 or not out.is_contiguous()
          or out.device != G.device):
        raise ValueError("s1_from_gram_batched: out must be a contiguous fp32 (batch, m + 1) tensor on G's device")
    fn = _lib.lib().pt2q_s1_from_upper_batched if upper_only else _lib.lib().pt2q_s1_from_gram_batched
    _lib.check(fn(_lib.ptr(G), G.stride(1), m, b, G.stride(0) if b > 1 else m * m, _lib.ptr(out),
                  _lib.stream_of(G.device)), "pt2q_s1_from_" + ("upper" if upper_only else "gram") + "_batched")
    return out


GROUP_MAX = 16  # linears per pt2q_quantize_blocks_group call (PT2Q_GROUP_MAX)


def group_supported(n: int, m: int, block_size: int, flags: int = _lib.FLAG_SSR | _lib.AGA_ACT) -> bool:
    """Whether pt2q_quantize_blocks_group takes linears of this shape (else per-linear loops):
    the library's own answer (pt2q_quantize_blocks_group_supported), so shape limits, tuning
    overrides and the error feedback's buffer limits are never restated here."""
    return bool(_lib.lib().pt2q_quantize_blocks_group_supported(int(n), int(m), int(block_size), int(flags)))


def quantize_blocks_group(Ws, As, Hinvs, block_size: int = 128, use_ssr: bool = True,
                          aga: int = _lib.AGA_ACT, max_iter: int = 100, t_dtype=torch.int8,
                          workspace: Optional[torch.Tensor] = None, outs=None, check: bool = True):
    """The block loops of several linears of one shape (n x m) in one launch sequence
    (pt2q_quantize_blocks_group): linear z is W = Ws[z] with AGA matrix As[z] (raw Gram, variant
    M) and inverse Hessian Hinvs[z]; each result is bit-identical to
    quantize_blocks(Ws[z], As[z], Hinvs[z]).  Up to GROUP_MAX linears per call.  check=False
    leaves the status word to the caller (_lib.check_status(workspace))."""
    Ws = [_float_input(W) for W in Ws]
    count = len(Ws)
    if not 1 <= count <= GROUP_MAX:
        raise ValueError(f"quantize_blocks_group: 1..{GROUP_MAX} linears (got {count})")
    n, m = Ws[0].shape
    dev = Ws[0].device
    if any(W.shape != (n, m) or W.dtype != Ws[0].dtype for W in Ws):
        raise ValueError("quantize_blocks_group: every W must have the same shape and dtype")
    B = num_blocks(m, block_size)
    flags = (_lib.FLAG_SSR if use_ssr else 0) | aga
    Hinvs = [H.contiguous().float() for H in Hinvs]
    As = [None if A is None else A.contiguous().float() for A in As] if As is not None else [None] * count
    if outs is None:
        outs = [LayerOutput(torch.empty((n, B), dtype=torch.float32, device=dev),
                            torch.empty((n, B), dtype=torch.float32, device=dev),
                            torch.empty((n, m), dtype=t_dtype, device=dev),
                            torch.empty(m, dtype=torch.int64, device=dev),
                            torch.zeros(B, dtype=torch.int32, device=dev)) for _ in range(count)]
    nbytes = _lib.lib().pt2q_quantize_blocks_group_workspace_bytes(count, n, m, int(block_size), flags)
    ws = workspace if workspace is not None and workspace.numel() >= nbytes else _lib.workspace(nbytes, dev)
    arrs = [_lib.ptr_array(x) for x in (Ws, As, Hinvs, [o.alpha for o in outs], [o.mu for o in outs],
                                        [o.T for o in outs], [o.perm for o in outs], [o.iters for o in outs])]
    p = [a[0] for a in arrs]
    rc = _lib.lib().pt2q_quantize_blocks_group(
        count, p[0], _lib.dtype_code(Ws[0]), m, n, m, int(block_size), flags, p[1], m, p[2], m, int(max_iter),
        p[3], p[4], p[5], _lib.dtype_code(outs[0].T), p[6], p[7], _lib.ptr(ws), ws.numel(), _lib.stream_of(dev))
    _lib.check(rc, "pt2q_quantize_blocks_group")
    if check:
        _lib.check_status(ws, "pt2q_quantize_blocks_group")
    return outs


PC_GROUP_MAX = 16  # linears per pt2q_quantize_perchannel_group call (PT2Q_PC_GROUP_MAX)


def perchannel_group_supported(m: int) -> bool:
    """Per-channel linears (one block, block_size >= m) the grouped entry takes: m > 512."""
    return m > 512


def quantize_perchannel_group(Ws, s1ds=None, max_iter: int = 100, t_dtype=torch.int8,
                              workspace: Optional[torch.Tensor] = None, outs=None, check: bool = True):
    """Per-channel block loops (block_size >= m: one block of every column; main.py:158-230,
    BASELINE C5) of up to PC_GROUP_MAX linears of one width m and dtype in ONE launch sequence
    (pt2q_quantize_perchannel_group): their rows share one grid, so a 5120-row linear no longer
    ends its launch in a partial wave.  Ws[z] (n_z x m; row counts may differ), s1ds[z] = S1 then
    d of its raw Gram (s1_from_gram_batched's row, m + 1 fp32; None = no AGA).  Each result is
    bit-identical to quantize_blocks(Ws[z], G, None, block_size=m, s1d=s1ds[z])."""
    Ws = [_float_input(W) for W in Ws]
    count = len(Ws)
    if not 1 <= count <= PC_GROUP_MAX:
        raise ValueError(f"quantize_perchannel_group: 1..{PC_GROUP_MAX} linears (got {count})")
    m, dev, dt = Ws[0].shape[1], Ws[0].device, Ws[0].dtype
    if not perchannel_group_supported(m) or any(W.shape[1] != m or W.dtype != dt or W.device != dev for W in Ws):
        raise ValueError("quantize_perchannel_group: linears of one width m > 512, one dtype and device")
    if s1ds is not None:
        if len(s1ds) != count:
            raise ValueError("quantize_perchannel_group: one s1d per linear")
        for t in s1ds:
            if t is not None and (t.numel() != m + 1 or t.dtype != torch.float32 or not t.is_contiguous()
                                  or t.device != dev):
                raise ValueError("quantize_perchannel_group: s1d must be m + 1 contiguous fp32 on W's device")
    if outs is None:
        outs = [LayerOutput(torch.empty((W.shape[0], 1), dtype=torch.float32, device=dev),
                            torch.empty((W.shape[0], 1), dtype=torch.float32, device=dev),
                            torch.empty((W.shape[0], m), dtype=t_dtype, device=dev),
                            torch.empty(m, dtype=torch.int64, device=dev),
                            torch.zeros(1, dtype=torch.int32, device=dev)) for W in Ws]
    nbytes = _lib.lib().pt2q_quantize_perchannel_group_workspace_bytes(count)
    ws = workspace if workspace is not None and workspace.numel() >= nbytes else _lib.workspace(nbytes, dev)
    import ctypes
    ns = (ctypes.c_int * count)(*[W.shape[0] for W in Ws])
    arrs = [_lib.ptr_array(x) for x in (Ws, [None] * count if s1ds is None else s1ds, [o.alpha for o in outs],
                                        [o.mu for o in outs], [o.T for o in outs], [o.perm for o in outs],
                                        [o.iters for o in outs])]
    p = [a[0] for a in arrs]
    rc = _lib.lib().pt2q_quantize_perchannel_group(
        count, p[0], _lib.dtype_code(Ws[0]), m, ctypes.cast(ns, ctypes.c_void_p), m, p[1], int(max_iter),
        p[2], p[3], p[4], _lib.dtype_code(outs[0].T), p[5], p[6], _lib.ptr(ws), ws.numel(), _lib.stream_of(dev))
    _lib.check(rc, "pt2q_quantize_perchannel_group")
    if check:
        _lib.check_status(ws, "pt2q_quantize_perchannel_group")
    return outs


def hessian_inverse(G: torch.Tensor, nsamples: int, percdamp: float = 0.01):
    """main.py:129-141 on a raw Gram: damped H, then Hinv (pinv on Cholesky breakdown).
    Returns (Hinv, spd)."""
    H, _ = prepare_hessian(G, nsamples, percdamp)
    Hinv, spd = cholesky_inverse(H)
    if not spd:
        Hinv = torch.linalg.pinv(H)
    return Hinv, spd


def hessian_inverse_batched(G: torch.Tensor, nsamples: int, percdamp: float = 0.01,
                            Hinv: Optional[torch.Tensor] = None, info: Optional[torch.Tensor] = None,
                            scratch: Optional[dict] = None, chunk: int = 32):
    """main.py:129-139 for a batch of units of one width whose raw Grams are packed in G
    (batch, m, m), all over `nsamples` rows: damping and Cholesky inverse of every item, `chunk`
    items per pt2q_hessian_inverse_batched launch sequence (each step of the blocked
    factorisation serves all items of a chunk in one launch).  Stream-ordered, no host read:
    returns (Hinv (batch, m, m), info (batch,) int32 on the device -- non-zero items need the
    pinv fallback, see UnitRun.finish).  Item z is bit-identical to hessian_inverse(G[z]).
    scratch: a dict reused across calls for the per-chunk H and workspace buffers."""
    _lib.require_device(G)
    if G.dim() != 3 or G.shape[1] != G.shape[2] or G.dtype != torch.float32 or not G.is_contiguous():
        raise _lib.Pt2qError("hessian_inverse_batched: G must be a contiguous fp32 (batch, m, m) device tensor")
    batch, m, dev = G.shape[0], G.shape[1], G.device
    if Hinv is None:
        Hinv = torch.empty_like(G)
    if info is None:
        info = torch.empty(batch, dtype=torch.int32, device=dev)
    c = max(1, min(chunk, batch))
    sc = scratch if scratch is not None else {}
    key = (m, c)
    if key not in sc:
        sc[key] = (torch.empty((c, m, m), dtype=torch.float32, device=dev),
                   _lib.workspace(_lib.lib().pt2q_hessian_inverse_batched_workspace_bytes(m, c), dev))
    H, ws = sc[key]
    L, st = _lib.lib(), _lib.stream_of(dev)
    for z0 in range(0, batch, c):
        k = min(c, batch - z0)
        _lib.check(L.pt2q_hessian_inverse_batched(_lib.ptr(G[z0]), m, k, int(nsamples), float(percdamp),
                                                  _lib.ptr(H), _lib.ptr(Hinv[z0]), _lib.ptr(ws), ws.numel(),
                                                  _lib.ptr(info[z0:]), st), "pt2q_hessian_inverse_batched")
    return Hinv, info


def quantize_shared(Ws, G: torch.Tensor, nsamples: int, block_size: int = 128,
                    use_ssr: bool = True, percdamp: float = 0.01, max_iter: int = 100,
                    t_dtype=torch.int8):
    """Variant M for several linears that read the same activations (q/k/v, gate/up): one Gram
    G = XᵀX and one Cholesky inverse, then the block loop per weight.  Each result is
    bit-identical to quantize_layer(W, X) on that linear alone (same kernels, same inputs).
    Per-channel (block_size >= m): no inverse -- nothing reads it (pt2q_quantize_layer skips it
    the same way)."""
    m = G.shape[-1]
    if needs_inverse(m, block_size):
        Hinv, spd = hessian_inverse(G, nsamples, percdamp)
    else:
        Hinv, spd = None, True
    outs = []
    for W in Ws:
        out = quantize_blocks(W, G, Hinv, block_size, use_ssr, _lib.AGA_ACT, max_iter, t_dtype)
        out.spd = spd
        outs.append(out)
    return outs


class UnitWorkspace:
    """Device buffers for repeated work units of one input width m (bench / model loops): the
    Gram, damped Hessian and inverse, the Gram and Cholesky scratch, and one block-loop workspace
    per output width n.  Buffers are reused call after call (stream-ordered), nothing is freed."""

    def __init__(self, m: int, device, block_size: int = 128, flags=_lib.FLAG_SSR | _lib.AGA_ACT):
        dev = torch.device(device)
        self.m, self.device, self.block_size, self.flags = m, dev, block_size, flags
        self.G = torch.empty((m, m), dtype=torch.float32, device=dev)
        self.H = torch.empty_like(self.G)
        self.Hinv = torch.empty_like(self.G)
        self.damp = torch.empty(1, dtype=torch.float32, device=dev)
        self.gram_ws = _lib.workspace(_lib.lib().pt2q_gram_workspace_bytes(m), dev)
        self.chol_ws = _lib.workspace(_lib.lib().pt2q_cholesky_workspace_bytes(m), dev)
        self._blocks = {}

    def blocks(self, n: int) -> torch.Tensor:
        if n not in self._blocks:
            self._blocks[n] = _lib.workspace(blocks_workspace_bytes(n, self.m, self.block_size, self.flags),
                                             self.device)
        return self._blocks[n]


class UnitRun:
    """Outputs of quantize_unit whose device status has not been read yet (see finish())."""

    def __init__(self, outs, info, statuses, redo):
        self.outs, self.info, self.statuses, self._redo = outs, info, statuses, redo
        self.spd = None
        self.join = None  # set by UnitPipeline: the caller's stream must wait for its streams

    def finish(self):
        """One host read of the Cholesky status and every stall word; raises Pt2qError on a
        stall, and re-runs the unit with pinv (main.py:140-141) if the Hessian was not SPD."""
        if self.spd is not None:
            return self.outs
        if self.join is not None:
            self.join()
        vals = torch.cat([self.info.reshape(1)] + [s.reshape(1) for s in self.statuses]).cpu().tolist()
        for v in vals[1:]:
            _lib.raise_stall(int(v), "quantize_unit")
        self.spd = vals[0] == 0
        if not self.spd:
            self.outs = self._redo()
        for o in self.outs:
            o.spd = self.spd
        return self.outs


def quantize_unit(Ws, X: Optional[torch.Tensor] = None, G: Optional[torch.Tensor] = None,
                  nsamples: Optional[int] = None, block_size: int = 128, use_ssr: bool = True,
                  percdamp: float = 0.01, max_iter: int = 100, t_dtype=torch.int8,
                  workspace: Optional[UnitWorkspace] = None, defer: bool = False):
    """One work unit of the model loop (main.py:289-299 for linears that read the same input:
    q/k/v, gate/up, or a single linear): Gram of X (or a given raw Gram G over `nsamples` rows),
    damping, Cholesky inverse, then each weight's block loop, all stream-ordered with NO host
    synchronisation.  Results are bit-identical to quantize_layer(W, X) per linear.

    defer=False reads the status once at the end and returns [LayerOutput]; defer=True returns a
    UnitRun whose finish() does that read later (a model loop checks once per step)."""
    Ws = [_float_input(W) for W in Ws]
    m = Ws[0].shape[1]
    dev = Ws[0].device
    ws = workspace if workspace is not None and workspace.m == m else UnitWorkspace(m, dev, block_size)
    statuses = []
    if X is not None:
        X = _float_input(X.reshape(-1, X.shape[-1]))
        nsamples = X.shape[0]
        _lib.check(_lib.lib().pt2q_gram(_lib.ptr(X), _lib.dtype_code(X), nsamples, m, m, _lib.ptr(ws.G), m, 0,
                                        _lib.ptr(ws.gram_ws), ws.gram_ws.numel(), _lib.stream_of(dev)),
                   "pt2q_gram")
        statuses.append(_lib.status_view(ws.gram_ws).clone())
        Gm = ws.G
    else:
        if G is None or nsamples is None:
            raise ValueError("quantize_unit needs X, or G and nsamples")
        Gm = G.contiguous().float()
    run = _unit_tail(Ws, Gm, int(nsamples), ws, statuses, X, G, block_size, use_ssr, percdamp, max_iter,
                     t_dtype)
    return run if defer else run.finish()


def _unit_tail(Ws, Gm, nsamples, ws, statuses, X, G, block_size, use_ssr, percdamp, max_iter, t_dtype,
               Hinv=None, info=None):
    """Damping, Cholesky inverse and every weight's block loop of a unit whose raw Gram is Gm,
    on the current stream; returns the deferred UnitRun.  With Hinv (and its device info word)
    given -- an item of hessian_inverse_batched -- only the block loops run.  The pinv redo
    rebuilds the Gram from the caller's X (or G): Gm may be a reused buffer by the time the
    status is read."""
    m, dev = Ws[0].shape[1], Ws[0].device
    L = _lib.lib()
    st = _lib.stream_of(dev)
    if Hinv is None and not needs_inverse(m, block_size):  # per-channel: H⁻¹ is never read
        info = torch.zeros(1, dtype=torch.int32, device=dev)
    elif Hinv is None:
        _lib.check(L.pt2q_prepare_hessian(_lib.ptr(Gm), m, m, int(nsamples), float(percdamp),
                                          _lib.ptr(ws.H), m, _lib.ptr(ws.damp), st), "pt2q_prepare_hessian")
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(L.pt2q_cholesky_inverse(_lib.ptr(ws.H), m, m, _lib.ptr(ws.Hinv), m, _lib.ptr(ws.chol_ws),
                                           ws.chol_ws.numel(), _lib.ptr(info), st), "pt2q_cholesky_inverse")
        Hinv = ws.Hinv
    elif info is None:
        raise ValueError("_unit_tail: a given Hinv needs its info word")
    flags = (_lib.FLAG_SSR if use_ssr else 0) | _lib.AGA_ACT
    outs = []
    for W in Ws:
        n = W.shape[0]
        B = num_blocks(m, block_size)
        out = LayerOutput(torch.empty((n, B), dtype=torch.float32, device=dev),
                          torch.empty((n, B), dtype=torch.float32, device=dev),
                          torch.empty((n, m), dtype=t_dtype, device=dev),
                          torch.empty(m, dtype=torch.int64, device=dev),
                          torch.zeros(B, dtype=torch.int32, device=dev))
        bws = ws.blocks(n)
        rc = L.pt2q_quantize_blocks(
            _lib.ptr(W), _lib.dtype_code(W), m, n, m, int(block_size), flags, _lib.ptr(Gm), m,
            _lib.ptr(Hinv), m, int(max_iter), _lib.ptr(out.alpha), _lib.ptr(out.mu), _lib.ptr(out.T),
            _lib.dtype_code(out.T), _lib.ptr(out.perm), _lib.ptr(out.iters), _lib.ptr(bws), bws.numel(), st)
        _lib.check(rc, "pt2q_quantize_blocks")
        statuses.append(_lib.status_view(bws).clone())
        outs.append(out)

    def redo():  # main.py:140-141: pinv of the damped Hessian, then the block loops again (B > 1)
        Gr = gram(X) if X is not None else G.contiguous().float()
        Hinv = torch.linalg.pinv(prepare_hessian(Gr, nsamples, percdamp)[0])
        return [quantize_blocks(W, Gr, Hinv, block_size, use_ssr, _lib.AGA_ACT, max_iter, t_dtype)
                for W in Ws]

    return UnitRun(outs, info, statuses, redo)


class _Lane:
    """One stream of a UnitPipeline with its own raw-Gram slot and unit workspaces per width."""

    def __init__(self, dev, block_size):
        self.dev, self.bs = dev, block_size
        self.stream = torch.cuda.Stream(dev)
        self.ws = {}

    def workspace(self, m) -> UnitWorkspace:
        if m not in self.ws:
            self.ws[m] = UnitWorkspace(m, self.dev, self.bs)
        return self.ws[m]


class UnitPipeline:
    """Cross-unit overlap for a model loop of independent units (main.py:289-299 per unit).

    A unit is its Gram (MFMA-bound; every CU holds one long-lived workgroup that takes all of
    its LDS and registers) and its tail: damping, Cholesky inverse and block loops, a long chain
    of small latency-bound launches that leave most of the chip idle.  Units alternate between
    `lanes` streams, each with its own Gram slot and workspaces; the Grams are chained by events
    (one Gram at a time: a stream-K Gram needs every CU for its co-resident hand-offs).  The
    next Gram takes the chip as soon as the previous one ends, so the tail of unit i is held
    back until Gram i+1 is done and then runs beside the tail of unit i+1 -- two latency-bound
    chains filling each other's gaps.  Every kernel sees exactly the operands of the sequential
    order (per-lane buffers, stream order within a lane), so the results are bit-identical to
    quantize_unit one unit after another.

    run(Ws, X) returns a deferred UnitRun; its finish() joins the lanes into the caller's
    stream (or call join())."""

    def __init__(self, device, block_size: int = 128, use_ssr: bool = True, percdamp: float = 0.01,
                 max_iter: int = 100, lanes: int = 3):
        self.dev = torch.device(device)
        self.bs, self.use_ssr, self.percdamp, self.max_iter = block_size, use_ssr, percdamp, max_iter
        self.lanes = [_Lane(self.dev, block_size) for _ in range(lanes)]
        self.turn = 0
        self.gram_done = None  # event: the last Gram issued

    def workspace(self, m) -> UnitWorkspace:
        """Allocate every lane's buffers for width m now (outside any timed region)."""
        for ln in self.lanes:
            ln.workspace(m)
        return self.lanes[0].workspace(m)

    def run(self, Ws, X: Optional[torch.Tensor] = None, G: Optional[torch.Tensor] = None,
            nsamples: Optional[int] = None, Hinv: Optional[torch.Tensor] = None,
            info: Optional[torch.Tensor] = None):
        """Issue one unit: its Gram from X, or -- with G (a raw Gram over nsamples rows, e.g. a
        GramAccumulator's, read in place and not modified) -- its tail alone; with Hinv and info
        as well (an item of hessian_inverse_batched), only its block loops."""
        Ws = [_float_input(W) for W in Ws]
        if X is not None:
            X = _float_input(X.reshape(-1, X.shape[-1]))
            nsamples = X.shape[0]
        elif G is None or nsamples is None:
            raise ValueError("UnitPipeline.run needs X, or G and nsamples")
        m, N = Ws[0].shape[1], int(nsamples)
        ln = self.lanes[self.turn]
        self.turn = (self.turn + 1) % len(self.lanes)
        ws = ln.workspace(m)
        st = ln.stream
        st.wait_stream(torch.cuda.current_stream(self.dev))  # inputs written on the caller's stream
        with torch.cuda.stream(st):
            if G is not None:
                G = G.contiguous().float()
                run = _unit_tail(Ws, G, N, ws, [], X, G, self.bs, self.use_ssr, self.percdamp,
                                 self.max_iter, torch.int8, Hinv=Hinv, info=info)
                run.join = self.join
                return run
            if self.gram_done is not None:
                st.wait_event(self.gram_done)
            _lib.check(_lib.lib().pt2q_gram(_lib.ptr(X), _lib.dtype_code(X), N, m, m, _lib.ptr(ws.G), m, 0,
                                            _lib.ptr(ws.gram_ws), ws.gram_ws.numel(), _lib.stream_of(self.dev)),
                       "pt2q_gram")
            self.gram_done = torch.cuda.Event()
            self.gram_done.record(st)
            statuses = [_lib.status_view(ws.gram_ws).clone()]
            run = _unit_tail(Ws, ws.G, N, ws, statuses, X, None, self.bs, self.use_ssr, self.percdamp,
                             self.max_iter, torch.int8)
        run.join = self.join
        return run

    def join(self):
        """The caller's current stream waits for every unit issued so far."""
        caller = torch.cuda.current_stream(self.dev)
        for ln in self.lanes:
            caller.wait_stream(ln.stream)


class LayerWorkspace:
    """Reusable device workspace for repeated layers of one shape (bench / model loops)."""

    def __init__(self, n, m, block_size, device, flags=_lib.FLAG_SSR | _lib.AGA_ACT):
        self.nbytes = int(_lib.lib().pt2q_layer_workspace_bytes(n, m, block_size, flags))
        self.buf = _lib.workspace(self.nbytes, device)
        self.shape = (n, m, block_size)

    def gram_view(self, m):
        # pt2q_quantize_layer carves the status word first, then the raw Gram (256-byte aligned)
        o = _lib.STATUS_BYTES
        return self.buf[o: o + m * m * 4].view(torch.float32).view(m, m)

    def status(self):
        return _lib.status_view(self.buf)


def quantize_layer(W: torch.Tensor, X: torch.Tensor, block_size: int = 128, use_ssr: bool = True,
                   percdamp: float = 0.01, max_iter: int = 100, t_dtype=torch.int8,
                   workspace: Optional[LayerWorkspace] = None, check_spd: bool = True,
                   outputs: Optional[LayerOutput] = None) -> LayerOutput:
    """Variant M whole layer (main.py:102-230) as one fused launch sequence (pt2q_quantize_layer).

    check_spd=False skips the single host read of the Cholesky and stall status (benchmark
    loops; the caller must then check `outputs.info` and `workspace.status()` itself, e.g.
    `check_layer_status`)."""
    W = _float_input(W)
    X = _float_input(X.reshape(-1, X.shape[-1]))
    n, m = W.shape
    N = X.shape[0]
    dev = W.device
    B = num_blocks(m, block_size)
    flags = (_lib.FLAG_SSR if use_ssr else 0) | _lib.AGA_ACT
    if workspace is None or workspace.shape != (n, m, block_size):
        workspace = LayerWorkspace(n, m, block_size, dev, flags)
    if outputs is None:
        outputs = LayerOutput(torch.empty((n, B), dtype=torch.float32, device=dev),
                              torch.empty((n, B), dtype=torch.float32, device=dev),
                              torch.empty((n, m), dtype=t_dtype, device=dev),
                              torch.empty(m, dtype=torch.int64, device=dev),
                              torch.zeros(B, dtype=torch.int32, device=dev))
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = _lib.lib().pt2q_quantize_layer(
        _lib.ptr(W), _lib.dtype_code(W), m, n, m, _lib.ptr(X), _lib.dtype_code(X), N, m,
        int(block_size), flags, float(percdamp), int(max_iter), _lib.ptr(outputs.alpha),
        _lib.ptr(outputs.mu), _lib.ptr(outputs.T), _lib.dtype_code(outputs.T), _lib.ptr(outputs.perm),
        _lib.ptr(outputs.iters), _lib.ptr(info), _lib.ptr(workspace.buf), workspace.nbytes,
        _lib.stream_of(dev))
    _lib.check(rc, "pt2q_quantize_layer")
    outputs.info = info
    outputs.status = workspace.status()
    if check_spd and not check_layer_status(outputs, "pt2q_quantize_layer"):
        # main.py:140-141: Cholesky failed -> pinv of the damped Hessian; the raw Gram is intact.
        G = workspace.gram_view(m).clone()
        H, _ = prepare_hessian(G, N, percdamp)
        Hinv = torch.linalg.pinv(H)
        out = quantize_blocks(W, G, Hinv, block_size, use_ssr, _lib.AGA_ACT, max_iter, t_dtype)
        out.spd = False
        return out
    return outputs


def check_layer_status(out: LayerOutput, what="layer") -> bool:
    """One host read of the Cholesky status and the stall word of a quantize_layer call.
    Raises Pt2qError on a stall; returns True when the Hessian was positive definite."""
    info, status = (int(v) for v in torch.stack([out.info.reshape(-1)[0],
                                                 out.status.reshape(-1)[0]]).cpu())
    _lib.raise_stall(status, what)
    return info == 0


class LayerGraph:
    """One whole layer (pt2q_quantize_layer: ~600 kernel launches at d=4096) captured into a
    hipGraph and replayed; W and X are captured by address, so update them in place between
    replays.  The Cholesky status is read with `spd()` after a replay (one host read)."""

    def __init__(self, W: torch.Tensor, X: torch.Tensor, block_size: int = 128,
                 use_ssr: bool = True, percdamp: float = 0.01, max_iter: int = 100,
                 t_dtype=torch.int8):
        self.W = _float_input(W)
        self.X = _float_input(X.reshape(-1, X.shape[-1]))
        n, m = self.W.shape
        dev = self.W.device
        B = num_blocks(m, block_size)
        self.args = (block_size, use_ssr, percdamp, max_iter, t_dtype)
        self.ws = LayerWorkspace(n, m, block_size, dev)
        self.out = LayerOutput(torch.empty((n, B), dtype=torch.float32, device=dev),
                               torch.empty((n, B), dtype=torch.float32, device=dev),
                               torch.empty((n, m), dtype=t_dtype, device=dev),
                               torch.empty(m, dtype=torch.int64, device=dev),
                               torch.zeros(B, dtype=torch.int32, device=dev))
        self._run()  # eager warm-up: loads every kernel before capture
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._run()

    def _run(self):
        bs, ssr, pd, mi, td = self.args
        return quantize_layer(self.W, self.X, bs, ssr, pd, mi, td, workspace=self.ws,
                              check_spd=False, outputs=self.out)

    def replay(self) -> LayerOutput:
        self.graph.replay()
        return self.out

    def spd(self) -> bool:
        """Cholesky status of the last replay; raises Pt2qError if a hand-off stalled."""
        return check_layer_status(self.out, "LayerGraph")


def error_feedback(W: torch.Tensor, blk: torch.Tensor, rem: torch.Tensor, E: torch.Tensor,
                   Hinv: torch.Tensor) -> torch.Tensor:
    """main.py:187-214 for one block, in place on fp32 W (n x m):
    W[:, rem] -= E @ (Hinv[blk][:, rem] / clamp(Hinv[blk, blk], 1e-8))."""
    _lib.require_device(W)
    if W.dtype != torch.float32 or not W.is_contiguous():
        raise _lib.Pt2qError("error_feedback updates a contiguous fp32 W in place")
    n, m = W.shape
    blk = blk.to(device=W.device, dtype=torch.int64).contiguous()
    rem = rem.to(device=W.device, dtype=torch.int64).contiguous()
    E = E.to(device=W.device, dtype=torch.float32).contiguous()
    Hinv = Hinv.to(device=W.device, dtype=torch.float32).contiguous()
    bs, r = blk.numel(), rem.numel()
    if E.shape != (n, bs) or Hinv.shape != (m, m):
        raise ValueError("error_feedback: E must be n x len(blk) and Hinv m x m")
    # the kernels gather Hinv / W rows with these indices: out-of-range or overlapping sets would
    # read or write out of bounds where the reference's torch indexing raises (one host read)
    idx = torch.cat([blk, rem])
    if idx.numel():
        lo, hi = (int(v) for v in torch.stack([idx.min(), idx.max()]).cpu())
        if lo < 0 or hi >= m:
            raise IndexError(f"error_feedback: column index out of range [0, {m}) (got {lo}..{hi})")
        if torch.unique(idx).numel() != idx.numel():
            raise ValueError("error_feedback: blk and rem must be disjoint sets of distinct columns")
    ws = _lib.workspace(_lib.lib().pt2q_error_feedback_workspace_bytes(n, m, max(bs, 1)), W.device)
    _lib.check(_lib.lib().pt2q_error_feedback(_lib.ptr(W), m, n, m, _lib.ptr(blk), bs, _lib.ptr(rem), r,
                                              _lib.ptr(E), bs, _lib.ptr(Hinv), m, _lib.ptr(ws),
                                              ws.numel(), _lib.stream_of(W.device)),
               "pt2q_error_feedback")
    return W


def dequantize(alpha, mu, T, perm, block_size):
    """Correct reconstruction W_q[:, perm[k*b:(k+1)*b]] = alpha[:,k]*T + mu[:,k] (gptq.py:201-230)."""
    n, m = T.shape
    dev = T.device
    out = torch.empty((n, m), dtype=torch.float32, device=dev)
    Tc = T.contiguous()
    if Tc.dtype not in (torch.int8, torch.float32):
        Tc = Tc.float()
    _lib.check(_lib.lib().pt2q_dequantize(_lib.ptr(alpha.float().contiguous()),
                                          _lib.ptr(mu.float().contiguous()), _lib.ptr(Tc),
                                          _lib.dtype_code(Tc), _lib.ptr(perm.contiguous()), n, m,
                                          int(block_size), _lib.ptr(out), _lib.stream_of(dev)),
               "pt2q_dequantize")
    return out


def pack_ternary(T: torch.Tensor):
    """utils.py:189-219 2-bit packing ({-1,0,1} -> {0,1,2}, 4 codes per byte), on device."""
    Tc = T.contiguous().to(torch.int8)
    cnt = Tc.numel()
    out = torch.empty((cnt + 3) // 4, dtype=torch.uint8, device=Tc.device)
    _lib.check(_lib.lib().pt2q_pack_ternary(_lib.ptr(Tc), cnt, _lib.ptr(out), _lib.stream_of(Tc.device)),
               "pt2q_pack_ternary")
    return out, T.shape


def unpack_ternary(packed: torch.Tensor, orig_shape):
    """utils.py:222-248."""
    cnt = 1
    for d in orig_shape:
        cnt *= d
    out = torch.empty(cnt, dtype=torch.int8, device=packed.device)
    _lib.check(_lib.lib().pt2q_unpack_ternary(_lib.ptr(packed.contiguous()), cnt, _lib.ptr(out),
                                              _lib.stream_of(packed.device)), "pt2q_unpack_ternary")
    return out.reshape(orig_shape)


def fill_synthetic(shape, seed, std=1.0, outliers=False, device="cuda"):
    """Device twin of tests/synth.py (bit-identical values)."""
    import numpy as np
    out = torch.empty(shape, dtype=torch.float32, device=device)
    scale = np.float32(std * np.sqrt(3.0) / float(1 << 23))
    oscale = np.float32(scale * np.float32(20.0))
    cols = shape[-1]
    _lib.check(_lib.lib().pt2q_fill_synthetic(_lib.ptr(out), out.numel(), int(seed) & (2**64 - 1),
                                              float(scale), cols, 100 if outliers else 0,
                                              float(oscale), _lib.stream_of(out.device)),
               "pt2q_fill_synthetic")
    return out
