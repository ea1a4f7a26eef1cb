"""Ternary inference (reference model.py:17-127 TernaryLinear).

The HIP kernel (2-bit codes dequantised into f16/bf16 MFMA operands, fp32 accumulation) is a
floating-point kernel: it is compared with the oracle's float64 restatement of the same
dtype-rounded operands (oracle.ternary_linear), and with the reference's own fp16 outputs
(tests/golden/ternary_linear_*.npz).  Tolerance: fp16 output rounding (rtol 2e-3) plus
accumulation-order noise (atol 2e-3 at these magnitudes)."""
import numpy as np
import pytest
import torch

import synth
from conftest import load_golden
from oracle import oracle as orc
from test_gpu_parity import cuda, host

pytestmark = pytest.mark.gpu

RTOL, ATOL = 2e-3, 2e-3


def _layer(pt2q, g, compat, dtype=torch.float16):
    n, m = int(g["n"]), int(g["m"])
    lay = pt2q.TernaryLinear(m, n, int(g["block_size"]), bias=True, dtype=dtype, compat=compat)
    lay.set_quantized_params(cuda(g["alpha"]), cuda(g["mu"]), cuda(g["T"]), cuda(g["perm"]),
                             cuda(g["bias"].astype(np.float32)))
    return lay


@pytest.mark.parametrize("name", ["ternary_linear_384x512", "ternary_linear_200x1000_pc"])
def test_compat_forward_matches_reference(pt2q, name):
    g = load_golden(name)
    lay = _layer(pt2q, g, compat=True)
    y = host(lay(cuda(g["x"])).float())
    np.testing.assert_allclose(y, g["out"].astype(np.float32), rtol=RTOL, atol=ATOL)
    yo = orc.ternary_linear(g["x"], g["alpha"], g["mu"], g["T"], g["perm"], g["bias"],
                            int(g["block_size"]), compat=True).astype(np.float32)
    np.testing.assert_allclose(y, yo, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("name", ["ternary_linear_384x512", "ternary_linear_200x1000_pc"])
def test_correct_forward_matches_reconstruction(pt2q, name):
    """Default semantics: y = x·Ŵᵀ + b with Ŵ = pt2q.dequantize (gptq.py:201-230)."""
    g = load_golden(name)
    lay = _layer(pt2q, g, compat=False)
    x = cuda(g["x"])
    y = host(lay(x).float())
    yo = orc.ternary_linear(g["x"], g["alpha"], g["mu"], g["T"], g["perm"], g["bias"],
                            int(g["block_size"]), compat=False).astype(np.float32)
    np.testing.assert_allclose(y, yo, rtol=RTOL, atol=ATOL)
    # the same weight via the device dequantisation kernel (fp16-rounded scales)
    bs = min(int(g["block_size"]), int(g["m"]))
    What = pt2q.dequantize(cuda(g["alpha"]).half().float(), cuda(g["mu"]).half().float(),
                           cuda(g["T"]), cuda(g["perm"]), bs).half().float()
    yt = host((x.float() @ What.T + cuda(g["bias"].astype(np.float32))).half().float())
    np.testing.assert_allclose(y, yt, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("n,m,bs,tokens,dt", [(4096, 4096, 128, 1, torch.float16),
                                              (4096, 4096, 128, 7, torch.bfloat16),
                                              (1000, 1100, 128, 300, torch.float16),
                                              (640, 520, 520, 33, torch.bfloat16),
                                              (4096, 11008, 128, 64, torch.float16),
                                              # prefill kernel (>= 256 tokens): ragged features
                                              # and tokens, per-channel bf16, 384-wide blocks
                                              (1000, 1100, 128, 700, torch.float16),
                                              (600, 640, 640, 513, torch.bfloat16),
                                              (512, 1536, 384, 256, torch.float16),
                                              (2048, 4096, 128, 2048, torch.float16)])
def test_shapes_vs_oracle(pt2q, n, m, bs, tokens, dt):
    """Decode (1 token, K split), prefill, ragged m (padded positions), per-channel, bf16."""
    rng = np.random.default_rng(n + m + tokens)
    T = rng.integers(-1, 2, size=(n, m)).astype(np.int8)
    B = -(-m // bs)
    alpha = (rng.random((n, B)) * 0.05 + 0.005).astype(np.float32)
    mu = (rng.standard_normal((n, B)) * 0.002).astype(np.float32)
    perm = rng.permutation(m).astype(np.int64)
    bias = (rng.standard_normal(n) * 0.1).astype(np.float32)
    x = synth.activations(7 + tokens, tokens, m)
    npdt = np.float16 if dt == torch.float16 else None
    lay = pt2q.TernaryLinear(m, n, bs, bias=True, dtype=dt)
    lay.set_quantized_params(cuda(alpha), cuda(mu), cuda(T), cuda(perm), cuda(bias))
    y = host(lay(cuda(x).to(dt)).float())
    if npdt is None:  # bf16: round operands through torch on the host
        a16 = torch.from_numpy(alpha).bfloat16().float().numpy()
        m16 = torch.from_numpy(mu).bfloat16().float().numpy()
        W = np.zeros((n, m), np.float32)
        for k in range(B):
            cols = perm[k * bs:(k + 1) * bs]
            W[:, cols] = torch.from_numpy(a16[:, k:k + 1] * T[:, cols].astype(np.float32)
                                          + m16[:, k:k + 1]).bfloat16().float().numpy()
        xb = torch.from_numpy(x).bfloat16().double().numpy()
        bb = torch.from_numpy(bias).bfloat16().double().numpy()
        yo = torch.from_numpy((xb @ W.astype(np.float64).T + bb).astype(np.float32)).bfloat16().float().numpy()
        rtol, atol = 1.6e-2, 1e-2
    else:
        yo = orc.ternary_linear(x, alpha, mu, T, perm, bias, bs, compat=False).astype(np.float32)
        rtol, atol = RTOL, ATOL * max(1.0, np.sqrt(m / 512))
    np.testing.assert_allclose(y, yo, rtol=rtol, atol=atol)


def test_replace_save_load_roundtrip(pt2q, tmp_path):
    """model.py:174-225 replace_linear_with_ternary + utils.py:288-304 save/load."""
    g = load_golden("ternary_linear_384x512")
    n, m = int(g["n"]), int(g["m"])
    model = torch.nn.Sequential(torch.nn.Linear(m, n, bias=True)).cuda().half()
    model[0].bias.data = cuda(g["bias"]).half()
    params = {"0": {"alpha": cuda(g["alpha"]).half(), "mu": cuda(g["mu"]).half(),
                    "T": cuda(g["T"]), "perm": cuda(g["perm"])}}
    pt2q.replace_linear_with_ternary(model, params, block_size=128, compat=True)
    assert isinstance(model[0], pt2q.TernaryLinear)
    y1 = model(cuda(g["x"]))
    np.testing.assert_allclose(host(y1.float()), g["out"].astype(np.float32), rtol=RTOL, atol=ATOL)
    path = str(tmp_path / "q.pt")
    pt2q.save_quantized_model(model, path, {"0": {k: v.cpu() for k, v in params["0"].items()}})
    fresh = torch.nn.Sequential(pt2q.TernaryLinear(m, n, 128, bias=True, compat=True))
    fresh, qp = pt2q.load_quantized_model(fresh, path)
    assert set(qp) == {"0"}
    assert torch.equal(host_t(fresh[0].T), host_t(model[0].T))
    assert torch.equal(fresh(cuda(g["x"])), y1)
    assert model[0].packed_footprint() < model[0].memory_footprint()


def host_t(t):
    return t.detach().cpu()


def test_perplexity_ternary_model_vs_reference(pt2q):
    """f4 on the ternary path: the tiny Llama with every decoder linear swapped for the libpt2q
    TernaryLinear (per-block ATQ params of the fixture, fp16 MFMA kernel) evaluated on the GPU
    by evaluate_perplexity, vs the reference's evaluate_perplexity of the same model built with
    its own fp32 TernaryLinear on the CPU (gen_golden.gen_ppl): the perplexities agree to the
    fp16 activation rounding of the kernel (relative 5e-3)."""
    from conftest import load_golden, unpack2
    from test_gpu_model import tiny_llama_and_samples
    g = load_golden("ppl_llama2l")
    model = tiny_llama_and_samples()[0].cuda()
    params = {}
    for i in range(int(g["nlin"])):
        a = torch.from_numpy(g[f"talpha{i}"])
        params[str(g[f"tname{i}"])] = {"alpha": a, "mu": torch.from_numpy(g[f"tmu{i}"]),
                                       "T": torch.from_numpy(unpack2(g[f"tT2_{i}"], a.shape[1] * 128)),
                                       "perm": torch.arange(a.shape[1] * 128)}
    pt2q.replace_linear_with_ternary(model, params, block_size=128, compat=True)
    assert sum(isinstance(m, pt2q.TernaryLinear) for m in model.modules()) == int(g["nlin"])
    got = pt2q.evaluate_perplexity(model, seq_len=128, input_ids=torch.from_numpy(g["ids"]))
    want = float(g["ppl_ternary_128"])
    assert np.isfinite(got) and abs(got - want) <= 5e-3 * want, (got, want)
