"""GPTQ / GPTQQuantizer on MI355X — same surface as the reference's gptq.py:21-272 (variant G).

add_batch accumulates H += XᵀX with the f32-MFMA Gram kernel; quantize() runs damping, the HIP
Cholesky inverse (pinv fallback on breakdown, gptq.py:104-106) and the fused block loop with the
AGA fed by the damped Hessian block H[blk][:, blk] (gptq.py:147-150).

Deliberate differences (documented in DESIGN.md §6):
  - H is kept in fp32 whatever the layer dtype (the reference's fp16/bf16 H crashes in pinv,
    SURVEY §0.2); outputs are cast back to the layer dtype.
  - columns <= block_size: the reference raises UnboundLocalError (gptq.py:162-170); here the
    layer is quantised per-channel (one block).
"""
from typing import Dict, Tuple

import torch
import torch.nn as nn

from . import _lib
from . import engine


class GPTQ:
    def __init__(self, layer: nn.Linear, block_size: int = 128, percdamp: float = 0.01):
        self.layer = layer
        self.block_size = block_size
        self.percdamp = percdamp
        self.device = layer.weight.device
        self.dtype = layer.weight.dtype
        W = layer.weight.data
        self.rows, self.columns = W.shape
        # the kernels' device: the layer's own, or the current HIP device for a CPU layer (the
        # reference's CPU call shape; results are returned on the layer's device)
        self._dev = _lib.compute_device(W)
        self.H = torch.zeros((self.columns, self.columns), device=self._dev, dtype=torch.float32)
        self.nsamples = 0
        self.alpha = None
        self.mu = None
        self.T = None
        self.perm = None
        self.last_output = None

    def add_batch(self, inp: torch.Tensor):
        """gptq.py:59-76: H += inpᵀ inp; nsamples += rows."""
        if inp.dim() == 3:
            inp = inp.reshape(-1, inp.shape[-1])
        engine.gram(inp.to(self._dev), self.H, accumulate=True)
        self.nsamples += inp.shape[0]

    def quantize(self, use_ssr: bool = True) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        """gptq.py:78-199. Returns (alpha (rows, B), mu, T (rows, columns) float, perm)."""
        if self.nsamples == 0:
            raise RuntimeError("GPTQ.quantize: no calibration data (call add_batch first)")
        H, _ = engine.prepare_hessian(self.H, self.nsamples, self.percdamp)
        Hinv, spd = engine.cholesky_inverse(H)
        out = engine.quantize_blocks(self.layer.weight.data.to(self._dev), H, Hinv, self.block_size,
                                     use_ssr, _lib.AGA_HESS, 100, torch.float32)
        out.spd = spd
        self.last_output = out
        self.alpha = out.alpha.to(self.device, self.dtype)
        self.mu = out.mu.to(self.device, self.dtype)
        self.T = out.T.to(self.device, self.dtype)
        self.perm = out.perm.to(self.device)
        return self.alpha, self.mu, self.T, self.perm

    def get_quantized_weight(self) -> torch.Tensor:
        """gptq.py:201-230 (correct per-block reconstruction through perm)."""
        if self.T is None:
            raise RuntimeError("Must call quantize() first")
        bs = self.block_size if self.block_size < self.columns else self.columns
        d = self._dev
        return engine.dequantize(self.alpha.to(d), self.mu.to(d), self.T.to(d), self.perm.to(d),
                                 bs).to(self.device, self.dtype)


class GPTQQuantizer:
    """gptq.py:233-272."""

    def __init__(self, model: nn.Module, block_size: int = 128, percdamp: float = 0.01,
                 use_ssr: bool = True):
        self.model = model
        self.block_size = block_size
        self.percdamp = percdamp
        self.use_ssr = use_ssr
        self.quantizers: Dict[str, GPTQ] = {}
        self.calibration_data = []

    def add_calibration_data(self, data: torch.Tensor):
        self.calibration_data.append(data)

    def prepare_quantizer(self, name: str, layer: nn.Linear):
        self.quantizers[name] = GPTQ(layer, self.block_size, self.percdamp)

    def quantize_layer(self, name: str) -> Dict[str, torch.Tensor]:
        if name not in self.quantizers:
            raise ValueError(f"Layer {name} not prepared for quantization")
        alpha, mu, T, perm = self.quantizers[name].quantize(use_ssr=self.use_ssr)
        return {"alpha": alpha, "mu": mu, "T": T, "perm": perm}
