"""Perplexity evaluation -- the reference's evaluate_perplexity (utils.py:128-186), SURVEY §8 f4.

The window / NLL loop is the reference's exactly: non-overlapping windows of seq_len tokens
(stride = seq_len), each window's labels = its inputs with the first len - trg_len positions set
to -100 (trg_len = end - prev_end, so with stride = seq_len nothing is masked -- kept as written),
the window's NLL = the model's mean token loss x trg_len, and ppl = exp(sum of NLLs / the last
window's end).  The forwards run wherever the model lives: a model whose linears were swapped for
TernaryLinear (ternary.replace_linear_with_ternary) runs them on the libpt2q MFMA kernels.

Data: the reference downloads wikitext-2 / C4 with `datasets.load_dataset` and tokenises the
joined text.  There is no network here, so the caller may pass `input_ids` (1 x L token ids) or
`text` (tokenised with `tokenizer`); only without both is `load_dataset` attempted, as the
reference does.
"""
from typing import Optional

import torch


def _load_text(dataset_name: str, dataset_config: str) -> str:
    """utils.py:151-160: the joined evaluation text (needs the datasets hub)."""
    try:
        from datasets import load_dataset
    except ImportError as e:  # pragma: no cover - datasets is installed in this image
        raise RuntimeError("evaluate_perplexity: `datasets` is not importable; pass input_ids or text") from e
    if dataset_name == "wikitext":
        ds = load_dataset(dataset_name, dataset_config, split="test")
        return "\n\n".join(ds["text"])
    if dataset_name == "c4":
        ds = load_dataset("allenai/c4", "en", split="validation", streaming=True)
        return "\n\n".join(item["text"] for item in list(ds.take(1000)))
    raise ValueError(f"Unknown dataset: {dataset_name}")


@torch.no_grad()
def evaluate_perplexity(model: torch.nn.Module, tokenizer=None, dataset_name: str = "wikitext",
                        dataset_config: str = "wikitext-2-raw-v1", seq_len: int = 2048,
                        device: Optional[torch.device] = None, *, text: Optional[str] = None,
                        input_ids: Optional[torch.Tensor] = None) -> float:
    """Perplexity of `model` (a causal LM returning `.loss` for `labels`) over a token stream,
    utils.py:128-186.  Returns a Python float, like the reference."""
    if device is None:
        t = next(model.parameters(), None)
        device = (t if t is not None else next(model.buffers())).device
    if input_ids is None:
        if text is None:
            text = _load_text(dataset_name, dataset_config)
        if tokenizer is None:
            raise ValueError("evaluate_perplexity: a tokenizer is needed to encode text")
        input_ids = tokenizer(text, return_tensors="pt")["input_ids"]
    input_ids = input_ids.to(device)
    if input_ids.dim() == 1:
        input_ids = input_ids[None, :]
    L = input_ids.size(1)
    seq_len = min(seq_len, L)
    nlls = []
    prev_end_loc = 0
    for begin_loc in range(0, L, seq_len):
        end_loc = min(begin_loc + seq_len, L)
        trg_len = end_loc - prev_end_loc
        input_chunk = input_ids[:, begin_loc:end_loc]
        target_ids = input_chunk.clone()
        target_ids[:, :-trg_len] = -100
        outputs = model(input_chunk, labels=target_ids)
        nlls.append(outputs.loss * trg_len)
        prev_end_loc = end_loc
        if end_loc >= L:
            break
    return torch.exp(torch.stack(nlls).sum() / prev_end_loc).item()
