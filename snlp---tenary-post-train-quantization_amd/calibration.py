"""Calibration capture with on-the-fly Grams — the caller of the hot path.

The reference (main.py:257-299) registers forward hooks on every nn.Linear of one decoder layer,
keeps every captured input (128 samples x 2048 tokens x d fp32 = 4 GB per linear at d=4096),
concatenates them and calls quantize_layer(linear, X) once per linear.  Only the Gram of X is
ever needed by the layer loop (H = XᵀX/N, and the AGA statistics S1 = G[blk,blk]·1 of
main.py:177 come from the raw Gram), so here each hook streams its batch straight into an
m x m fp32 Gram with the chain-continuing Gram kernel (pt2q_gram accumulate=2).  The result is
bit-identical to the Gram of the concatenated activations, memory is O(m²) instead of O(N·m),
and linears that read the same tensor (q/k/v, gate/up) share one Gram and one Cholesky
inverse.

Reference helpers mirrored: find_linear_layers (model.py:162-171), get_llm_layers
(model.py:139-159), the per-layer loop of PT2LLMQuantizer.quantize (main.py:232-308) and its
weight write-back _dequantize_weight (main.py:313-335).
"""
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import _lib
from . import engine


def find_linear_layers(module: nn.Module, prefix: str = "") -> Dict[str, nn.Linear]:
    """model.py:162-171: recursive name -> nn.Linear map (children order)."""
    out = {}
    for name, child in module.named_children():
        full = f"{prefix}.{name}" if prefix else name
        if isinstance(child, nn.Linear):
            out[full] = child
        else:
            out.update(find_linear_layers(child, full))
    return out


def get_llm_layers(model: nn.Module, model_type: str = "llama"):
    """model.py:139-159: the decoder-layer list of the supported architectures."""
    if model_type in ("llama", "llama2", "llama3", "qwen", "qwen3"):
        return model.model.layers
    if model_type in ("gemma", "gemma3"):
        if hasattr(model, "language_model") and hasattr(model.language_model, "layers"):
            return model.language_model.layers
        if hasattr(model, "model") and hasattr(model.model, "layers"):
            return model.model.layers
        raise AttributeError("Cannot find layers in Gemma model")
    if model_type == "opt":
        return model.model.decoder.layers
    if model_type == "bloom":
        return model.transformer.h
    raise ValueError(f"Unknown model type: {model_type}")


class GramAccumulator:
    """An m x m fp32 Gram fed batch by batch; bit-identical to XᵀX of the concatenated rows.

    Batches are copied into a staging buffer of `buffer_rows` rows (a multiple of 8, capped at
    ~512 MiB) and the Gram runs once per full buffer, chain-continuing (pt2q_gram accumulate=2):
    one calibration sample's 2048 rows make a Gram launch too short to fill the chip (0.55 PF/s on
    a Llama-2-7B layer's captures, against 1.2 PF/s for the long chains).  The 16-bit MFMA Gram
    advances each fp32 chain in groups of 8 rows, so a chain may only be continued from a row
    count that is a multiple of 8: every full buffer is, and only the last (flushed) launch may be
    ragged.  Stall reports of the Gram launches are OR-ed into a device word and checked once,
    when `G` is read.  buffer_rows=0: a Gram launch per batch (the remainder rows of a 16-bit batch
    held back to lead the next one)."""

    MAX_BUFFER_BYTES = 512 << 20

    def __init__(self, m: int, device, buffer_rows: int = 32768):
        self.m = m
        self.device = torch.device(device)
        self._G = torch.zeros((m, m), dtype=torch.float32, device=self.device)
        self.nsamples = 0
        self._rows_in_G = 0
        self._pend: Optional[torch.Tensor] = None
        self._ws = _lib.workspace(_lib.lib().pt2q_gram_workspace_bytes(m), self.device)
        self._stall = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._cap = max(0, int(buffer_rows)) // 8 * 8
        self._buf: Optional[torch.Tensor] = None
        self._fill = 0

    def _run(self, X: torch.Tensor):
        mode = "continue" if self._rows_in_G else False
        engine.gram(X, self._G, accumulate=mode, workspace=self._ws, check=False)
        torch.bitwise_or(self._stall, _lib.status_view(self._ws), out=self._stall)
        self._rows_in_G += X.shape[0]

    def _flush(self):
        if self._buf is not None and self._fill:
            fill, self._fill = self._fill, 0
            self._run(self._buf[:fill])
        if self._pend is not None:
            pend, self._pend = self._pend, None
            self._run(pend)

    def _buffered(self, X: torch.Tensor):
        if self._buf is None or self._buf.dtype != X.dtype:
            self._flush()
            cap = min(self._cap, max(8, self.MAX_BUFFER_BYTES // (self.m * X.element_size()) // 8 * 8))
            self._buf = torch.empty((cap, self.m), dtype=X.dtype, device=self.device)
        cap = self._buf.shape[0]
        o = 0
        while o < X.shape[0]:
            k = min(cap - self._fill, X.shape[0] - o)
            self._buf[self._fill:self._fill + k].copy_(X[o:o + k])
            self._fill += k
            o += k
            if self._fill == cap:  # a full buffer: a multiple of 8 rows, so the chain may continue
                self._fill = 0
                self._run(self._buf)

    def add(self, X: torch.Tensor):
        X = X.reshape(-1, X.shape[-1])
        if X.shape[-1] != self.m:
            raise ValueError(f"GramAccumulator: expected {self.m} features, got {X.shape[-1]}")
        X = X.to(self.device)
        if X.shape[0] == 0:
            return
        self.nsamples += X.shape[0]
        if self._cap:
            self._buffered(X)
            return
        if X.dtype not in (torch.float16, torch.bfloat16):
            self._flush()  # f32 chains advance row by row: any split is exact
            self._run(X)
            return
        if self._pend is not None:
            if self._pend.dtype != X.dtype:
                self._flush()
            else:
                need = 8 - self._pend.shape[0]
                head = torch.cat([self._pend, X[:need]])
                X = X[need:]
                self._pend = None
                if head.shape[0] < 8:
                    self._pend = head
                    return
                self._run(head)
        k = X.shape[0] // 8 * 8
        if k:
            self._run(X[:k])
        if k < X.shape[0]:
            self._pend = X[k:].clone()

    @property
    def G(self) -> torch.Tensor:
        """The finished Gram (flushes held rows; raises Pt2qError if a Gram launch stalled)."""
        self._flush()
        _lib.raise_stall(int(self._stall.item()), "GramAccumulator")
        return self._G


class GramCapture:
    """Forward hooks on a set of linears (main.py:262-275) that stream each input batch into a
    Gram.  Linears whose input is the very same tensor in a forward pass share one accumulator
    (grouping is fixed at the first pass and checked afterwards)."""

    def __init__(self, linears: Dict[str, nn.Linear], device=None, buffer_rows: int = 32768):
        self.linears = linears
        self.device = device
        self.buffer_rows = buffer_rows  # GramAccumulator staging (0: a Gram launch per batch)
        self.group_of: Dict[str, int] = {}
        self.accs: List[GramAccumulator] = []
        self.members: List[List[str]] = []
        self._last_key: Dict[int, tuple] = {}
        # the last input of each group is held until the next pass, so its storage cannot be
        # recycled for another tensor of the same shape within the pass (that would alias keys)
        self._held: Dict[int, torch.Tensor] = {}
        self._pass = 0
        self._hooks = []

    @staticmethod
    def _key(t: torch.Tensor, pass_id: int):
        return (pass_id, t.data_ptr(), tuple(t.shape), tuple(t.stride()), t._version)

    def _hook(self, name):
        def hook(module, inp, out):
            x = inp[0] if isinstance(inp, tuple) else inp
            x = x.detach()
            key = self._key(x, self._pass)
            if name not in self.group_of:
                gid = None
                for g, k in self._last_key.items():
                    if k == key and self.accs[g].m == x.shape[-1]:
                        gid = g
                        break
                if gid is None:
                    dev = self.device if self.device is not None else x.device
                    self.accs.append(GramAccumulator(x.shape[-1], dev, self.buffer_rows))
                    self.members.append([])
                    gid = len(self.accs) - 1
                self.group_of[name] = gid
                self.members[gid].append(name)
            gid = self.group_of[name]
            if self._last_key.get(gid) == key:
                return  # same tensor already added by a group partner in this pass
            if self._last_key.get(gid, (None,))[0] == self._pass:
                raise RuntimeError(f"GramCapture: linears {self.members[gid]} were grouped on a "
                                   "shared input but received different inputs")
            self._last_key[gid] = key
            self._held[gid] = x
            self.accs[gid].add(x)
        return hook

    def __enter__(self):
        for name, lin in self.linears.items():
            self._hooks.append(lin.register_forward_hook(self._hook(name)))
        return self

    def __exit__(self, *exc):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self._held.clear()
        return False

    def next_pass(self):
        """Call between forward passes (one per calibration sample)."""
        self._pass += 1
        self._held.clear()

    def groups(self):
        """[(accumulator, [linear names])] in first-seen order."""
        return list(zip(self.accs, self.members))


def dequantize_weight_reference(params, block_size: int) -> torch.Tensor:
    """main.py:313-335 exactly as the reference writes weights back between layers: blocks are
    taken as contiguous column ranges of T (which is in ORIGINAL order) and then the inverse
    permutation is applied, which mis-assigns scales when SSR reorders.  Kept for
    reference-compatible model propagation; `engine.dequantize` is the correct reconstruction."""
    T = params["T"].float()
    alpha, mu, perm = params["alpha"], params["mu"], params["perm"]
    n, m = T.shape
    W = torch.zeros(n, m, dtype=alpha.dtype, device=T.device)
    for b in range(alpha.shape[1]):
        s, e = b * block_size, min((b + 1) * block_size, m)
        W[:, s:e] = alpha[:, b:b + 1] * T[:, s:e] + mu[:, b:b + 1]
    return W[:, torch.argsort(perm)]


class _StopForward(Exception):
    pass


@torch.no_grad()
def capture_layer_inputs(model: nn.Module, layer: nn.Module, samples, model_dev=None):
    """The inputs of decoder layer `layer` (normally layer 0) for every calibration sample:
    [(args, kwargs)] as the model's forward passes them, recorded by a forward pre-hook that
    stops the forward there (only the embeddings and the layers before it run).  The forward
    is called with use_cache=False (a KV cache never changes a single forward's outputs)."""
    rec = []

    def hook(mod, args, kwargs):
        rec.append((tuple(args), dict(kwargs)))
        raise _StopForward

    h = layer.register_forward_pre_hook(hook, with_kwargs=True)
    try:
        for sample in samples:
            try:
                model(sample.to(model_dev) if model_dev is not None else sample, use_cache=False)
            except _StopForward:
                pass
    finally:
        h.remove()
    return rec


def _with_hidden(args, kwargs, x):
    if args:
        return (x,) + tuple(args[1:]), kwargs
    kw = dict(kwargs)
    kw["hidden_states"] = x
    return args, kw


@torch.no_grad()
def propagate_layer(layer: nn.Module, inputs):
    """Run the (quantised, written-back) layer on every sample's recorded inputs -> the next
    layer's inputs (the same hidden states the reference's full-model forward would hand it)."""
    out = []
    for args, kwargs in inputs:
        y = layer(*args, **kwargs)
        y = y[0] if isinstance(y, (tuple, list)) else y
        out.append(_with_hidden(args, kwargs, y))
    return out


@torch.no_grad()
def quantize_decoder_layer(layer: nn.Module, run_forward, block_size: int = 128,
                           use_ssr: bool = True, percdamp: float = 0.01, layer_idx: int = 0,
                           writeback: str = "reference", device=None,
                           pipeline: Optional["engine.UnitPipeline"] = None, grams_first=None):
    """One iteration of main.py:258-303 for decoder layer `layer`.

    run_forward(capture) must run the calibration forwards (calling capture.next_pass() between
    samples).  Returns {"layer_<i>.<name>": {alpha, mu, T int8, perm}} (device tensors) and
    writes the quantised weights back into the linears ("reference": main.py:297-299 semantics,
    "correct": gptq.py:201-230 reconstruction, "none": leave weights untouched).  With a
    UnitPipeline the input groups' tails (their Grams are already captured) run concurrently on
    its lanes -- they are independent: every input was captured before any write-back -- with
    results identical to the one-after-another order.
    With a sharding.GramsFirst (`grams_first`, built on such a pipeline) the captured Grams go into
    its packed slots instead: the layer's Hessian inverses run batched per width and the block
    loops grouped by shape on the lanes (q/k/v/o, gate/up) -- bit-identical again."""
    linears = find_linear_layers(layer)
    cap = GramCapture(linears, device)
    with cap:
        run_forward(cap)
    results = {}
    issued = []
    groups = cap.groups()
    if grams_first is not None:
        gf = grams_first
        gf.begin([(g, acc.m, acc.nsamples) for g, (acc, _) in enumerate(groups)])
        for g, (acc, _) in enumerate(groups):
            gf.set_gram(g, acc.G)
        gf.inverses()
        jobs = [(g, [linears[nm].weight.data.to(acc.device) for nm in names], acc.nsamples)
                for g, (acc, names) in enumerate(groups)]
        runs = gf.tails(jobs)
        issued = [(names, run) for (_, names), run in zip(groups, runs)]
    for acc, names in ([] if grams_first is not None else groups):
        Ws = [linears[nm].weight.data.to(acc.device) for nm in names]
        if pipeline is not None:
            issued.append((names, pipeline.run(Ws, G=acc.G, nsamples=acc.nsamples)))
        else:
            issued.append((names, engine.quantize_shared(Ws, acc.G, acc.nsamples, block_size, use_ssr,
                                                         percdamp)))
    for names, outs in issued:
        if pipeline is not None or grams_first is not None:
            outs = outs.finish()
        for nm, out in zip(names, outs):
            lin = linears[nm]
            dt = lin.weight.dtype
            params = {"alpha": out.alpha.to(dt), "mu": out.mu.to(dt), "T": out.T, "perm": out.perm}
            results[f"layer_{layer_idx}.{nm}"] = params
            if writeback == "reference":
                Wq = dequantize_weight_reference(params, block_size)
            elif writeback == "correct":
                bs = block_size if block_size < out.T.shape[1] else out.T.shape[1]
                Wq = engine.dequantize(out.alpha, out.mu, out.T, out.perm, bs)
            elif writeback == "none":
                continue
            else:
                raise ValueError(f"writeback must be reference|correct|none, got {writeback}")
            lin.weight.data = Wq.to(lin.weight.device, dt)
    return results
