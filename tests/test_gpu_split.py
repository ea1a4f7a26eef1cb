"""Intra-layer split: the Gram of one layer data-parallel over the calibration
rows, partial Grams folded in rank order (pt2q_sum_partials), the rest of the layer on the
folded G -- HIP path vs oracle.quantize_layer_split, bit-exact.  The ranks' Grams run in one
process here (the box has one GPU); tests/test_sharding_gloo.py covers the multi-process
exchange on gloo.  Reference: main.py:128-230."""
import importlib

import numpy as np
import pytest
import torch

import pt2q_loader
import synth
from oracle import oracle as orc
from test_gpu_parity import bits_equal, host

pytestmark = pytest.mark.gpu

pt2q = pt2q_loader.load()
sharding = importlib.import_module("pt2q.sharding")


@pytest.mark.parametrize("parts", [1, 2, 3, 8, 9, 17])
def test_sum_partials_rank_order(parts):
    m = 260  # 67600 floats: a multiple of 4, not of the launch width
    rng = np.random.default_rng(parts)
    P = (rng.standard_normal((parts, m, m)) * 10.0 ** rng.integers(-6, 6, (parts, m, m))).astype(np.float32)
    Pd = torch.from_numpy(P).cuda()
    got = pt2q.sum_partials(Pd)
    ref = orc.sum_partials(list(P))
    assert bits_equal(host(got), ref)
    pt2q.sum_partials(Pd, out=Pd[0])  # in place over part 0
    assert bits_equal(host(Pd[0]), ref)


@pytest.mark.parametrize("world,dtype", [(2, "fp16"), (3, "fp16"), (4, "fp32"), (8, "bf16")])
def test_layer_split_vs_oracle(world, dtype):
    n, m, N = 320, 384, 1203  # ragged row slices
    W = synth.weights(9001, n, m)
    X = synth.activations(9002, N, m)
    Xd = torch.from_numpy(X).cuda()
    if dtype == "fp16":
        Xd = Xd.half()
        Xo = X.astype(np.float16)
    elif dtype == "bf16":
        Xd = Xd.bfloat16()
        Xo = Xd.cpu()
    else:
        Xo = X
    Wd = torch.from_numpy(W).cuda()
    parts = torch.empty((world, m, m), dtype=torch.float32, device="cuda")
    for r in range(world):
        lo, hi = sharding.row_slice(N, r, world)
        pt2q.gram(Xd[lo:hi], G=parts[r])
    G = pt2q.sum_partials(parts)
    out = pt2q.quantize_shared([Wd], G, N)[0]
    ref = orc.quantize_layer_split(W, Xo, world)
    assert bits_equal(host(G), ref["G"])
    assert np.array_equal(host(out.perm), ref["perm"])
    assert np.array_equal(host(out.T), ref["T"])
    assert bits_equal(host(out.alpha), ref["alpha"])
    assert bits_equal(host(out.mu), ref["mu"])


def test_layer_split_single_rank_is_the_layer():
    """Without a process group the split is the plain layer: quantize_layer_split == oracle
    quantize_layer_m (one partial, nothing to fold)."""
    n, m, N = 256, 256, 512
    W = synth.weights(9101, n, m)
    X = synth.activations(9102, N, m).astype(np.float16)
    out = sharding.quantize_layer_split([torch.from_numpy(W).cuda()], torch.from_numpy(X).cuda())[0]
    ref = orc.quantize_layer_m(W, X)
    assert np.array_equal(host(out.perm), ref["perm"])
    assert np.array_equal(host(out.T), ref["T"])
    assert bits_equal(host(out.alpha), ref["alpha"])
    assert bits_equal(host(out.mu), ref["mu"])
