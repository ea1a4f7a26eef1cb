"""AsymmetricTernaryQuantizer on MI355X — same surface as the reference's quantizer.py:16-306.

Every method runs one HIP kernel of libpt2q (pt2q_atq_stage, atq.hip); results are bit-identical
to the CPU oracle and match the reference's codes exactly (tests/test_gpu_parity.py).
Inputs are computed in fp32: fp16/bf16 weights are upcast (exact) and outputs cast back to the
weight dtype (the reference itself overflows fp16 in `d = 1ᵀS1`, quantizer.py:218 — SURVEY §0.2).
CPU tensors (the reference's own call shape) are computed on the current HIP device and the
results returned on the CPU; with no HIP device the call raises (_lib.compute_device).
"""
from typing import Optional, Tuple

import torch

from . import _lib


def _dev_f32(t, dev):
    t = t.to(dev)
    return t.contiguous().float() if t.dtype != torch.float32 else t.contiguous()


def _col(v, n, device):
    return v.reshape(n).float().contiguous().to(device)


class AsymmetricTernaryQuantizer:
    """quantizer.py:16-293. ITF `max_iter` defaults to 100 (quantizer.py:25)."""

    def __init__(self, max_iter: int = 100):
        self.max_iter = max_iter
        self.last_itf_iters = None

    # --------------------------------------------------------------- helpers
    def _stage(self, mode, W, alpha=None, mu=None, T=None, S1=None, d=None):
        dev = _lib.compute_device(W)
        Wf = _dev_f32(W, dev)
        n, b = Wf.shape
        a = torch.empty(n, dtype=torch.float32, device=dev) if alpha is None else _col(alpha, n, dev).clone()
        m = torch.empty(n, dtype=torch.float32, device=dev) if mu is None else _col(mu, n, dev).clone()
        Tt = (torch.empty((n, b), dtype=torch.float32, device=dev) if T is None
              else T.to(dev).float().contiguous().clone())
        iters = torch.zeros(1, dtype=torch.int32, device=dev)
        ws = _lib.workspace(256, dev)
        rc = _lib.lib().pt2q_atq_stage(
            mode, _lib.ptr(Wf), b, n, b, _lib.ptr(a), _lib.ptr(m), _lib.ptr(Tt), b,
            _lib.ptr(S1), _lib.ptr(d), int(self.max_iter), _lib.ptr(iters), _lib.ptr(ws), ws.numel(),
            _lib.stream_of(dev))
        _lib.check(rc, "pt2q_atq_stage")
        return a, m, Tt, iters

    def _out(self, W, a, m, T=None):
        """Results in W's dtype, on W's device (CPU in -> CPU out)."""
        n = a.shape[0]
        res = (a.view(n, 1).to(W.device, W.dtype), m.view(n, 1).to(W.device, W.dtype))
        if T is not None:
            res = res + (T.to(W.device, W.dtype),)
        return res

    @staticmethod
    def s1_from_activations(X: torch.Tensor, b: int):
        """S = XᵀX (quantizer.py:207), S1 = S·1 (:216), d = 1ᵀS1 (:218) on the device."""
        if X.dim() == 3:
            X = X.reshape(-1, b)
        X = X.to(_lib.compute_device(X)).contiguous()
        if X.dtype not in (torch.float32, torch.float16, torch.bfloat16):
            X = X.float()
        dev = X.device
        S = torch.empty((b, b), dtype=torch.float32, device=dev)
        st = _lib.stream_of(dev)
        _lib.check(_lib.lib().pt2q_gram(_lib.ptr(X), _lib.dtype_code(X), X.shape[0], b, b,
                                        _lib.ptr(S), b, 0, None, 0, st), "pt2q_gram")
        S1 = torch.empty(b, dtype=torch.float32, device=dev)
        d = torch.empty(1, dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().pt2q_s1_from_gram(_lib.ptr(S), b, b, _lib.ptr(S1), _lib.ptr(d), st),
                   "pt2q_s1_from_gram")
        return S1, d

    # --------------------------------------------------------------- reference surface
    def ternary_init(self, W: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """quantizer.py:32-69."""
        a, m, T, _ = self._stage(_lib.STAGE_INIT, W)
        return self._out(W, a, m, T)

    def build_optimal_grid(self, W: torch.Tensor, T: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """quantizer.py:71-108."""
        a, m, _, _ = self._stage(_lib.STAGE_GRID, W, T=T)
        return self._out(W, a, m)

    def flexible_round(self, W: torch.Tensor, alpha: torch.Tensor, mu: torch.Tensor) -> torch.Tensor:
        """quantizer.py:110-134."""
        _, _, T, _ = self._stage(_lib.STAGE_ROUND, W, alpha=alpha, mu=mu)
        return T.to(W.dtype)

    def iterative_ternary_fitting(self, W, alpha, mu, T):
        """quantizer.py:136-175 (whole-block convergence semantics).  `last_itf_iters` holds the
        iteration count (device int32)."""
        a, m, Tn, it = self._stage(_lib.STAGE_ITF, W, alpha=alpha, mu=mu, T=T)
        self.last_itf_iters = it
        return self._out(W, a, m, Tn)

    def activation_aware_grid_alignment(self, W, T, X):
        """quantizer.py:177-248."""
        b = W.shape[1]
        S1, d = self.s1_from_activations(X, b)
        a, m, _, _ = self._stage(_lib.STAGE_AGA, W, T=T, S1=S1, d=d)
        return self._out(W, a, m)

    def quantize(self, W: torch.Tensor, X: Optional[torch.Tensor] = None):
        """quantizer.py:250-277: init -> ITF -> AGA (if X) in one fused kernel."""
        S1 = d = None
        if X is not None:
            X = X.to(_lib.compute_device(W, X))
            S1, d = self.s1_from_activations(X, W.shape[1])
        a, m, T, it = self._stage(_lib.STAGE_FULL, W, S1=S1, d=d)
        self.last_itf_iters = it
        return self._out(W, a, m, T)

    def dequantize(self, alpha: torch.Tensor, mu: torch.Tensor, T: torch.Tensor) -> torch.Tensor:
        """quantizer.py:279-293."""
        return alpha * T + mu


def compute_quantization_error(W: torch.Tensor, W_c: torch.Tensor) -> float:
    """quantizer.py:296-298 (reporting metric)."""
    return ((W - W_c) ** 2).sum().item()


def compute_output_error(W: torch.Tensor, W_c: torch.Tensor, X: torch.Tensor) -> float:
    """quantizer.py:301-306 (reporting metric)."""
    if X.dim() == 3:
        X = X.reshape(-1, X.shape[-1])
    diff = (W - W_c) @ X.T
    return (diff ** 2).sum().item()
