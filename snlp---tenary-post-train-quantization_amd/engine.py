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
         workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """XᵀX (main.py:128), X (N, m) or (B, L, m).

    accumulate=False: G = XᵀX.  True: G = G + XᵀX (gptq.py:75 add_batch).  "continue": every
    entry's fp32 chain resumes from G, so a Gram streamed batch by batch is bit-identical to one
    Gram of the concatenated rows (the captured-and-concatenated X of main.py:293) — for fp16 /
    bf16 activations, whose 16-bit MFMA chain advances in groups of 8 rows, when every batch
    but the last has a multiple of 8 rows."""
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
    return G


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


def quantize_blocks(W: torch.Tensor, A: Optional[torch.Tensor], Hinv: torch.Tensor,
                    block_size: int = 128, use_ssr: bool = True, aga: int = _lib.AGA_ACT,
                    max_iter: int = 100, t_dtype=torch.int8) -> LayerOutput:
    """The block loop given the AGA matrix A (raw Gram for variant M, damped H for variant G)."""
    W = _float_input(W)
    n, m = W.shape
    dev = W.device
    B = num_blocks(m, block_size)
    alpha = torch.empty((n, B), dtype=torch.float32, device=dev)
    mu = torch.empty((n, B), dtype=torch.float32, device=dev)
    T = torch.empty((n, m), dtype=t_dtype, device=dev)
    perm = torch.empty(m, dtype=torch.int64, device=dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    flags = (_lib.FLAG_SSR if use_ssr else 0) | aga
    ws = _lib.workspace(_lib.lib().pt2q_layer_workspace_bytes(n, m, block_size, flags), dev)
    Hinv = Hinv.contiguous().float()
    rc = _lib.lib().pt2q_quantize_blocks(
        _lib.ptr(W), _lib.dtype_code(W), m, n, m, int(block_size), flags,
        _lib.ptr(A), m, _lib.ptr(Hinv), m, int(max_iter), _lib.ptr(alpha), _lib.ptr(mu), _lib.ptr(T),
        _lib.dtype_code(T), _lib.ptr(perm), _lib.ptr(iters), _lib.ptr(ws), ws.numel(),
        _lib.stream_of(dev))
    _lib.check(rc, "pt2q_quantize_blocks")
    return LayerOutput(alpha, mu, T, perm, iters)


def hessian_inverse(G: torch.Tensor, nsamples: int, percdamp: float = 0.01):
    """main.py:129-141 on a raw Gram: damped H, then Hinv (pinv on Cholesky breakdown).
    Returns (Hinv, spd)."""
    H, _ = prepare_hessian(G, nsamples, percdamp)
    Hinv, spd = cholesky_inverse(H)
    if not spd:
        Hinv = torch.linalg.pinv(H)
    return Hinv, spd


def quantize_shared(Ws, G: torch.Tensor, nsamples: int, block_size: int = 128,
                    use_ssr: bool = True, percdamp: float = 0.01, max_iter: int = 100,
                    t_dtype=torch.int8):
    """Variant M for several linears that read the same activations (q/k/v, gate/up): one Gram
    G = XᵀX and one Cholesky inverse, then the block loop per weight.  Each result is
    bit-identical to quantize_layer(W, X) on that linear alone (same kernels, same inputs)."""
    Hinv, spd = hessian_inverse(G, nsamples, percdamp)
    outs = []
    for W in Ws:
        out = quantize_blocks(W, G, Hinv, block_size, use_ssr, _lib.AGA_ACT, max_iter, t_dtype)
        out.spd = spd
        outs.append(out)
    return outs


class LayerWorkspace:
    """Reusable device workspace for repeated layers of one shape (bench / model loops)."""

    def __init__(self, n, m, block_size, device, flags=_lib.FLAG_SSR | _lib.AGA_ACT):
        self.nbytes = int(_lib.lib().pt2q_layer_workspace_bytes(n, m, block_size, flags))
        self.buf = _lib.workspace(self.nbytes, device)
        self.shape = (n, m, block_size)

    def gram_view(self, m):
        # pt2q_quantize_layer carves the raw Gram first (256-byte aligned base)
        return self.buf[: m * m * 4].view(torch.float32).view(m, m)


def quantize_layer(W: torch.Tensor, X: torch.Tensor, block_size: int = 128, use_ssr: bool = True,
                   percdamp: float = 0.01, max_iter: int = 100, t_dtype=torch.int8,
                   workspace: Optional[LayerWorkspace] = None, check_spd: bool = True,
                   outputs: Optional[LayerOutput] = None) -> LayerOutput:
    """Variant M whole layer (main.py:102-230) as one fused launch sequence (pt2q_quantize_layer).

    check_spd=False skips the single host read of the Cholesky status (benchmark loops; the
    caller must then check `info` itself)."""
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
    if check_spd and int(info.item()) != 0:
        # main.py:140-141: Cholesky failed -> pinv of the damped Hessian; the raw Gram is intact.
        G = workspace.gram_view(m).clone()
        H, _ = prepare_hessian(G, N, percdamp)
        Hinv = torch.linalg.pinv(H)
        out = quantize_blocks(W, G, Hinv, block_size, use_ssr, _lib.AGA_ACT, max_iter, t_dtype)
        out.spd = False
        return out
    return outputs


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
        return int(self.out.info.item()) == 0


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
