"""PT2LLMQuantizer.quantize_layer on MI355X — the reference's CLI hot path (main.py:102-230).

Only the per-layer engine is in scope.  The model-level calibration loop, HF model
loading and the CLI (main.py:232-433, model.py, utils.py) need network access in the reference
and are out of scope for this engine; `quantize()` says so instead of silently doing nothing.
"""
from typing import Dict

import torch
import torch.nn as nn

from . import engine


class PT2LLMQuantizer:
    def __init__(self, model: nn.Module = None, tokenizer=None, model_type: str = "llama",
                 block_size: int = 128, num_calibration_samples: int = 128, seq_len: int = 2048,
                 use_ssr: bool = True, percdamp: float = 0.01, seed: int = 42,
                 device: str = "cuda"):
        self.model = model
        self.tokenizer = tokenizer
        self.model_type = model_type
        self.block_size = block_size
        self.num_calibration_samples = num_calibration_samples
        self.seq_len = seq_len
        self.use_ssr = use_ssr
        self.percdamp = percdamp
        self.seed = seed
        if not torch.cuda.is_available():
            raise RuntimeError("PT2LLMQuantizer (pt2q) needs a HIP device; there is no CPU path")
        self.device = torch.device(device if device != "cpu" else "cuda")
        self.quantized_params: Dict[str, Dict[str, torch.Tensor]] = {}
        self.last_output = None
        self._ws = None

    @torch.no_grad()
    def quantize_layer(self, layer: nn.Linear, layer_name: str,
                       calibration_activations: torch.Tensor) -> Dict[str, torch.Tensor]:
        """main.py:102-230. Returns CPU tensors {alpha, mu (n x B), T int8 (n x m), perm int64}."""
        W = layer.weight.data.to(self.device)
        X = calibration_activations
        if X.dim() == 3:
            X = X.reshape(-1, X.shape[-1])
        X = X.to(self.device)
        n, m = W.shape
        if self._ws is None or self._ws.shape != (n, m, self.block_size):
            self._ws = engine.LayerWorkspace(n, m, self.block_size, self.device)
        out = engine.quantize_layer(W, X, self.block_size, self.use_ssr, self.percdamp,
                                    workspace=self._ws)
        self.last_output = out
        dt = layer.weight.dtype
        return {
            "alpha": out.alpha.to(dt).cpu(),
            "mu": out.mu.to(dt).cpu(),
            "T": out.T.cpu(),
            "perm": out.perm.cpu(),
        }

    def quantize(self):
        raise NotImplementedError(
            "model-level calibration (main.py:232-311) needs HF models/datasets over the network and "
            "is outside this engine's scope; call quantize_layer per linear (see INTEGRATION.md)")
