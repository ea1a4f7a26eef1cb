"""Host-side reporting helpers on CPU: the error metrics (quantizer.py:296-306) and
bits per weight (utils.py:251-285, §8 f4), checked against the reference's own numbers."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import oracle as orc


def test_error_metrics_match_reference_examples(pt2q):
    """examples.py:15-45 example 1: E_w after init / ITF and E_x after AGA, as the reference
    printed them (examples_atq fixture), from the same metrics on the oracle's fitted grids."""
    g = load_golden("examples_atq")
    W, X = torch.from_numpy(g["W"]), torch.from_numpy(g["X"])
    a0, m0, T0 = orc.ternary_init(g["W"])
    e0 = pt2q.compute_quantization_error(W, torch.from_numpy(a0 * T0 + m0))
    assert e0 == pytest.approx(float(g["err_init"]), rel=1e-5)
    a1, m1, T1, _ = orc.iterative_ternary_fitting(g["W"], a0, m0, T0)
    e1 = pt2q.compute_quantization_error(W, torch.from_numpy(a1 * T1 + m1))
    assert e1 == pytest.approx(float(g["err_itf"]), rel=1e-5)
    ox = pt2q.compute_output_error(W, torch.from_numpy(a1 * T1 + m1), X)
    assert ox == pytest.approx(float(g["out_err_itf"]), rel=1e-5)
    a2, m2 = orc.activation_aware_grid_alignment(g["W"], T1, g["X"])
    ox2 = pt2q.compute_output_error(W, torch.from_numpy(a2 * T1 + m2), X.reshape(2, 16, -1))
    assert ox2 == pytest.approx(float(g["out_err_aga"]), rel=1e-5)


def test_bits_per_weight(pt2q):
    """utils.py:251-285: 1.58 bits per code + 16 bits per alpha / mu entry; 16.0 without ternary
    layers."""
    m1, n1, m2, n2, bs = 512, 256, 1000, 64, 128
    model = torch.nn.Sequential(
        pt2q.TernaryLinear(m1, n1, bs, device="cpu"),
        torch.nn.ReLU(),
        pt2q.TernaryLinear(m2, n2, bs, device="cpu"),
        torch.nn.Linear(8, 8))
    nw = n1 * m1 + n2 * m2
    ns = 2 * (n1 * -(-m1 // bs) + n2 * -(-m2 // bs))
    assert pt2q.compute_bits_per_weight(model) == pytest.approx((1.58 * nw + 16 * ns) / nw)
    assert pt2q.compute_bits_per_weight(model, include_scales=False) == pytest.approx(1.58)
    assert pt2q.compute_bits_per_weight(torch.nn.Linear(4, 4)) == 16.0
    # Llama-2-7B q_proj shape at block 128: 1.58 + 32/128 = 1.83 bits
    big = torch.nn.Sequential(pt2q.TernaryLinear(4096, 4096, 128, device="meta"))
    assert pt2q.compute_bits_per_weight(big) == pytest.approx(1.58 + 32 / 128)
