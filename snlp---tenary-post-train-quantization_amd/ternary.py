"""Ternary inference layer on MI355X — the reference's TernaryLinear (model.py:17-127),
replace_linear_with_ternary (model.py:174-225) and save/load (utils.py:288-304).

Buffers and their state_dict names are the reference's (T int8, alpha, mu, perm, inv_perm, bias),
so checkpoints move between the two.  The forward pass is the libpt2q kernel
pt2q_ternary_linear (csrc/ternary_linear.hip): 2-bit packed codes dequantised in registers into
f16/bf16 MFMA operands.  Two semantics:

  compat=False (default)  y = x · Ŵᵀ + b with the correct reconstruction of gptq.py:201-230
                          (block k of alpha/mu belongs to columns perm[k·bs:(k+1)·bs]).
  compat=True             exactly what the reference forward computes: contiguous blocks of T
                          and a double permutation (model.py:75-110).
"""
import os
from typing import Dict, Optional

import torch
import torch.nn as nn

from . import _lib


class TernaryLinear(nn.Module):
    """model.py:17-127."""

    def __init__(self, in_features: int, out_features: int, block_size: int = 128,
                 bias: bool = True, dtype: torch.dtype = torch.float16, compat: bool = False,
                 device=None):
        super().__init__()
        if dtype not in (torch.float16, torch.bfloat16):
            raise _lib.Pt2qError("TernaryLinear runs fp16/bf16 activations on the f16/bf16 MFMA "
                                 f"(got {dtype})")
        device = torch.device(device) if device is not None else torch.device("cuda")
        self.in_features = in_features
        self.out_features = out_features
        self.block_size = block_size
        self.compat = compat
        num_blocks = (in_features + block_size - 1) // block_size
        self.register_buffer("T", torch.zeros(out_features, in_features, dtype=torch.int8, device=device))
        self.register_buffer("alpha", torch.ones(out_features, num_blocks, dtype=dtype, device=device))
        self.register_buffer("mu", torch.zeros(out_features, num_blocks, dtype=dtype, device=device))
        self.register_buffer("perm", torch.arange(in_features, dtype=torch.long, device=device))
        self.register_buffer("inv_perm", torch.arange(in_features, dtype=torch.long, device=device))
        if bias:
            self.register_buffer("bias", torch.zeros(out_features, dtype=dtype, device=device))
        else:
            self.bias = None
        self._packed = None

    @property
    def dtype(self):
        return self.alpha.dtype

    def set_quantized_params(self, alpha: torch.Tensor, mu: torch.Tensor, T: torch.Tensor,
                             perm: torch.Tensor, bias: Optional[torch.Tensor] = None):
        """model.py:59-73, then packs the codes for the kernel."""
        self.T.copy_(T.to(torch.int8))
        self.alpha.copy_(alpha)
        self.mu.copy_(mu)
        self.perm.copy_(perm)
        self.inv_perm.copy_(torch.argsort(self.perm))
        if bias is not None and self.bias is not None:
            self.bias.copy_(bias)
        self._packed = None

    def _prepare(self):
        _lib.require_device(self.T)
        n, m = self.out_features, self.in_features
        dev = self.T.device
        P = int(_lib.lib().pt2q_ternary_linear_positions(m))
        codes = torch.empty((n, P // 4), dtype=torch.uint8, device=dev)
        gather = torch.empty(P, dtype=torch.int32, device=dev)
        st = _lib.stream_of(dev)
        _lib.check(_lib.lib().pt2q_ternary_pack(_lib.ptr(self.T.contiguous()), m, n, m,
                                                _lib.ptr(self.perm.contiguous()), int(self.compat),
                                                _lib.ptr(codes), _lib.ptr(gather), st),
                   "pt2q_ternary_pack")
        # scales as the reference stores them (alpha's dtype), widened exactly to fp32
        self._packed = (codes, gather, self.alpha.float().contiguous(), self.mu.float().contiguous(),
                        None if self.bias is None else self.bias.float().contiguous())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """model.py:75-95 (compat) or x·Ŵᵀ + b (default), on the ternary MFMA kernel."""
        if self._packed is None:
            self._prepare()
        codes, gather, a32, m32, b32 = self._packed
        _lib.require_device(x)
        shape = x.shape
        xt = x.reshape(-1, self.in_features).to(self.dtype).contiguous()
        tokens = xt.shape[0]
        n, m = self.out_features, self.in_features
        y = torch.empty((tokens, n), dtype=self.dtype, device=x.device)
        if tokens == 0:
            return y.reshape(*shape[:-1], n)
        ws = _lib.workspace(_lib.lib().pt2q_ternary_linear_workspace_bytes(tokens, n, m), x.device)
        B = a32.shape[1]
        _lib.check(_lib.lib().pt2q_ternary_linear(
            _lib.ptr(xt), _lib.dtype_code(xt), tokens, m, n, m, _lib.ptr(codes), _lib.ptr(gather),
            _lib.ptr(a32), _lib.ptr(m32), B, self.block_size, _lib.ptr(b32), _lib.ptr(y),
            _lib.dtype_code(y), n, _lib.ptr(ws), ws.numel(), _lib.stream_of(x.device)),
            "pt2q_ternary_linear")
        return y.reshape(*shape[:-1], n)

    def _dequantize(self) -> torch.Tensor:
        """model.py:97-110 as written (contiguous blocks of T; meaningful when perm = identity)."""
        W = torch.zeros(self.out_features, self.in_features, device=self.T.device, dtype=self.alpha.dtype)
        for b in range(self.alpha.shape[1]):
            s, e = b * self.block_size, min((b + 1) * self.block_size, self.in_features)
            W[:, s:e] = self.alpha[:, b:b + 1] * self.T[:, s:e].to(self.alpha.dtype) + self.mu[:, b:b + 1]
        return W

    def memory_footprint(self) -> int:
        """model.py:112-127 (bytes, reference accounting: int8 T, 2-byte scales)."""
        bias_bytes = self.bias.numel() * 2 if self.bias is not None else 0
        return (self.T.numel() + self.alpha.numel() * 2 + self.mu.numel() * 2 +
                self.perm.numel() * 8 + bias_bytes)

    def packed_footprint(self) -> int:
        """Bytes the kernel actually reads per call: 2-bit codes + fp32 scales (+ bias)."""
        if self._packed is None:
            self._prepare()
        codes, gather, a32, m32, b32 = self._packed
        return (codes.numel() + gather.numel() * 4 + a32.numel() * 4 + m32.numel() * 4 +
                (b32.numel() * 4 if b32 is not None else 0))


def replace_linear_with_ternary(model: nn.Module, quantized_params: Dict[str, Dict[str, torch.Tensor]],
                                block_size: int = 128, compat: bool = False) -> nn.Module:
    """model.py:174-225: swap each quantised nn.Linear for a TernaryLinear."""
    for name, params in quantized_params.items():
        parts = name.split(".")
        parent = model
        for part in parts[:-1]:
            parent = getattr(parent, part)
        orig = getattr(parent, parts[-1])
        dt = params["alpha"].dtype if params["alpha"].dtype in (torch.float16, torch.bfloat16) \
            else torch.float16
        layer = TernaryLinear(orig.in_features, orig.out_features, block_size,
                              bias=orig.bias is not None, dtype=dt, compat=compat,
                              device=orig.weight.device)
        layer.set_quantized_params(params["alpha"], params["mu"], params["T"], params["perm"],
                                   orig.bias.data if orig.bias is not None else None)
        setattr(parent, parts[-1], layer)
        del orig
    return model


def compute_bits_per_weight(model: nn.Module, include_scales: bool = True) -> float:
    """utils.py:251-285: average bits per weight over the ternary layers of `model` -- log2(3)
    rounded to 1.58 bits per code plus 16 bits per alpha / mu entry; 16.0 when the model has no
    ternary layer (the reference finds none after its own CLI run).  Host
    arithmetic on buffer sizes only."""
    total_params = 0
    total_bits = 0.0
    for _, module in model.named_modules():
        if hasattr(module, "T"):  # TernaryLinear (the reference's duck test)
            nw = module.T.numel()
            total_params += nw
            total_bits += nw * 1.58
            if include_scales:
                total_bits += (module.alpha.numel() + module.mu.numel()) * 16
    if total_params == 0:
        return 16.0
    return total_bits / total_params


def save_quantized_model(model: nn.Module, save_path: str,
                         quantized_params: Dict[str, Dict[str, torch.Tensor]]):
    """utils.py:288-296 (same file layout)."""
    torch.save({"model_state_dict": model.state_dict(), "quantized_params": quantized_params},
               save_path)


def load_quantized_model(model: nn.Module, load_path: str):
    """utils.py:299-304, with the safe loader (tensors and dicts only)."""
    ckpt = torch.load(load_path, map_location="cpu", weights_only=True)
    model.load_state_dict(ckpt["model_state_dict"])
    for mod in model.modules():
        if isinstance(mod, TernaryLinear):
            mod._packed = None
    return model, ckpt.get("quantized_params", {})
