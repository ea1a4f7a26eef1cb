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
    def quantize(self, calibration_samples=None, writeback: str = "reference",
                 propagate: str = "model", schedule: str = "grams-first", timings=None):
        """main.py:232-308: decoder layer by decoder layer, capture the linears' inputs over the
        calibration forwards, quantise every linear, write the weights back.  The captured
        inputs go straight into per-input Grams (calibration.GramCapture), so q/k/v and gate/up
        share one Gram and one Cholesky inverse; results equal quantize_layer on the
        concatenated activations bit-for-bit.  Returns {name: {alpha, mu, T, perm}} on CPU.

        propagate="model" runs, per decoder layer, a full-model forward per sample as the
        reference does (main.py:280-282; O(layers²) layer forwards).  "layerwise" records layer
        0's inputs once (calibration.capture_layer_inputs) and then runs each layer on its
        recorded inputs: for capture, and -- after the write-back -- to produce the next layer's
        inputs (calibration.propagate_layer).  Those are the hidden states the full forward hands
        that layer, so the results are the same; the forward work drops from L² to 2L layer passes.
        schedule="grams-first": one layer's captured Grams go into a sharding.GramsFirst (its
        inverses batched per width, the block loops grouped by shape on the lanes); "lanes": one
        unit per lane of an engine.UnitPipeline.  Bit-identical.
        timings: a list that receives one dict per decoder layer (wall seconds of capture,
        quantise, write-back, propagate and the host copies; device-synchronised between them)."""
        import time
        from . import sharding
        if self.model is None:
            raise RuntimeError("PT2LLMQuantizer.quantize needs a model")
        if propagate not in ("model", "layerwise") or schedule not in ("grams-first", "lanes"):
            raise ValueError("propagate must be model|layerwise and schedule grams-first|lanes")
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
        gf = sharding.GramsFirst(pipe, self.device) if schedule == "grams-first" else None
        inputs = (calibration.capture_layer_inputs(self.model, layers[0], calibration_samples, model_dev)
                  if propagate == "layerwise" else None)

        def mark():
            if timings is not None:
                torch.cuda.synchronize(self.device)
            return time.perf_counter()

        for idx, layer in enumerate(layers):
            t0 = mark()
            if inputs is None:
                def run(cap):
                    for sample in calibration_samples:
                        self.model(sample.to(model_dev))
                        cap.next_pass()
            else:
                def run(cap, layer=layer):
                    for args, kwargs in inputs:
                        layer(*args, **kwargs)
                        cap.next_pass()
            tq = [0.0]

            def run_timed(cap):
                run(cap)
                tq[0] = mark()
            res = calibration.quantize_decoder_layer(layer, run_timed, self.block_size, self.use_ssr,
                                                     self.percdamp, idx, writeback, self.device,
                                                     None if gf is not None else pipe, gf)
            t2 = mark()
            if inputs is not None and idx + 1 < len(layers):
                inputs = calibration.propagate_layer(layer, inputs)
            t3 = mark()
            for name, p in res.items():
                self.quantized_params[name] = {k: v.cpu() for k, v in p.items()}
            t4 = mark()
            if timings is not None:
                timings.append({"layer": idx, "capture_s": tq[0] - t0, "quantize_writeback_s": t2 - tq[0],
                                "propagate_s": t3 - t2, "to_host_s": t4 - t3, "total_s": t4 - t0})
        return self.quantized_params
