"""PT2LLMQuantizer.quantize_layer on MI355X — the reference's CLI hot path (main.py:102-230).

quantize() runs the model-level loop of main.py:232-308 on caller-supplied calibration samples
(the reference downloads them; there is no network here), streaming each linear's inputs into
shared Grams (calibration.py).  HF model loading and the CLI (model.py:228-260, main.py:338)
stay out of scope.
"""
from typing import Dict

import torch
import torch.nn as nn

from . import calibration, engine


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

    def get_calibration_data(self):
        """main.py:89-99 downloads wikitext through `datasets`; there is no network here, so
        calibration token tensors must be passed to quantize() explicitly."""
        raise RuntimeError("pass calibration_samples (list of token-id tensors) to quantize(); "
                           "dataset download (utils.py:47-60) is not available offline")

    @torch.no_grad()
    def quantize(self, calibration_samples=None, writeback: str = "reference"):
        """main.py:232-308: decoder layer by decoder layer, capture the linears' inputs over the
        calibration forwards, quantise every linear, write the weights back.  The captured
        inputs go straight into per-input Grams (calibration.GramCapture), so q/k/v and gate/up
        share one Gram and one Cholesky inverse; results equal quantize_layer on the
        concatenated activations bit-for-bit.  Returns {name: {alpha, mu, T, perm}} on CPU."""
        if self.model is None:
            raise RuntimeError("PT2LLMQuantizer.quantize needs a model")
        if calibration_samples is None:
            calibration_samples = self.get_calibration_data()
        layers = calibration.get_llm_layers(self.model, self.model_type)
        self.model.eval()
        # the calibration forwards run wherever the model lives (main.py:281 moves samples to the
        # model's device); captured inputs stream to the GPU Grams either way
        model_dev = next(self.model.parameters()).device
        # the units of one decoder layer are independent: their tails run on concurrent lanes
        pipe = engine.UnitPipeline(self.device, self.block_size, self.use_ssr,
                                   self.percdamp)
        for idx, layer in enumerate(layers):
            def run(cap):
                for sample in calibration_samples:
                    self.model(sample.to(model_dev))
                    cap.next_pass()
            res = calibration.quantize_decoder_layer(layer, run, self.block_size, self.use_ssr,
                                                     self.percdamp, idx, writeback, self.device, pipe)
            for name, p in res.items():
                self.quantized_params[name] = {k: v.cpu() for k, v in p.items()}
        return self.quantized_params
