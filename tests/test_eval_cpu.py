"""evaluate_perplexity (utils.py:128-186) vs the reference's own function run on
the same model and token stream (tests/golden/ppl_llama2l.npz, gen_golden.gen_ppl: the
reference's load_dataset / tokenizer replaced by fixed token ids -- no network).  The window /
NLL loop is host logic, so on the CPU model the result must be the reference's bit for bit."""
import numpy as np
import pytest
import torch

from conftest import load_golden


def _model():
    pytest.importorskip("transformers")
    from test_gpu_model import tiny_llama_and_samples
    return tiny_llama_and_samples()[0]


@pytest.fixture(scope="module")
def evaluate_perplexity():
    import pt2q_loader
    return pt2q_loader.load().evaluate_perplexity


def test_perplexity_window_loop_equals_reference(evaluate_perplexity):
    g = load_golden("ppl_llama2l")
    model = _model()
    ids = torch.from_numpy(g["ids"])
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        for s, want in zip(g["seq_lens"], g["ppl"]):
            got = evaluate_perplexity(model, seq_len=int(s), input_ids=ids)
            assert got == float(want), (int(s), got, float(want))  # 300 tokens: 128,128,44 / one window

        class Tok:  # the text path: tokenizer(text, return_tensors="pt")["input_ids"]
            def __call__(self, text, return_tensors="pt"):
                assert text == "the joined text" and return_tensors == "pt"
                return {"input_ids": ids}
        assert evaluate_perplexity(model, Tok(), seq_len=128, text="the joined text") == float(g["ppl"][0])
    finally:
        torch.set_num_threads(threads)
