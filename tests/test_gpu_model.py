"""Model-level loop vs the reference's own PT2LLMQuantizer.quantize.

tests/golden/model_llama2l.npz holds the reference's output (main.py:232-311 run on CPU with one
thread, get_calibration_data overridden on the instance) for a 2-layer Llama built from config
with a fixed seed.  Here the same model (state-dict checksum checked) and samples go through
pt2q's PT2LLMQuantizer.quantize with the reference-compatible write-back (main.py:313-335).
The model stays on the CPU and its forwards run single-threaded like the reference's, so the
captured activations are the reference's own bits; they stream into Grams on the GPU, where
everything else runs.  Block 0 of every linear does not depend on H⁻¹ and must match exactly
(codes; scales within the 1e-5 contract).  Later blocks inherit the H⁻¹ rounding (MKL's
sgemm/spotri order vs the engine's canonical chains, rel. ~1e-4), which flips a few
near-threshold codes (measured: 15 of 98304 in layer_0.mlp.down_proj), so the rest is held to
per-block set equality and >= 99.9 % code agreement; decoder layer 0's permutations are exact.
Layer 1's AGA statistics come from activations that went through layer 0's write-back (scales
~1e-7 apart), which AGA's per-row 2x2 solve amplifies on ill-conditioned rows, so its block-0
scales are held in aggregate (median relative difference <= 1e-3, >= 75 % of rows within 1e-3)
instead of the 1e-5 contract for identical inputs; its later blocks to >= 90 % block-set overlap
(near-tie SSR picks move between neighbouring blocks when the inputs differ) and >= 95 % code
agreement (measured in layer_1.mlp.down_proj: 97.9 % overlap, 97.9 % codes).  These bounds are
the free-running check only: test_model_layer1_teacher_forced_vs_reference holds layer 1 to the
contract (bit-exact) on the reference's own captured layer-1 inputs."""
import numpy as np
import pytest
import torch

from conftest import load_golden, unpack2
from test_oracle_golden import check_scales

pytestmark = pytest.mark.gpu

TINY_LLAMA = dict(vocab_size=512, hidden_size=256, intermediate_size=384, num_hidden_layers=2,
                  num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=256)


def tiny_llama_and_samples():
    transformers = pytest.importorskip("transformers")
    cfg = transformers.LlamaConfig(**TINY_LLAMA)
    torch.manual_seed(0)
    model = transformers.LlamaForCausalLM(cfg).eval()
    torch.manual_seed(1)
    samples = [torch.randint(0, TINY_LLAMA["vocab_size"], (1, 64)) for _ in range(3)]
    return model, samples


def test_model_loop_vs_reference(pt2q):
    g = load_golden("model_llama2l")
    model, samples = tiny_llama_and_samples()
    csum = np.array([float(p.detach().double().sum()) for p in model.state_dict().values()])
    np.testing.assert_array_equal(csum, g["checksum"])  # the very same weights as the reference's
    q = pt2q.PT2LLMQuantizer(model, None, "llama", block_size=128, use_ssr=True)
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        got = q.quantize(samples, writeback="reference")
    finally:
        torch.set_num_threads(threads)
    names = [str(n) for n in g["names"]]
    assert sorted(got) == names and len(names) == 14
    for i, name in enumerate(names):
        r = got[name]
        m = int(g[f"m{i}"])
        T_ref = unpack2(g[f"T2_{i}"], m)
        perm_ref, a_ref = g[f"perm{i}"], g[f"alpha{i}"]
        T, perm, a = r["T"].numpy(), r["perm"].numpy(), r["alpha"].float().numpy()
        b0 = perm_ref[:128]
        np.testing.assert_array_equal(perm[:128], b0, err_msg=name)
        np.testing.assert_array_equal(T[:, b0], T_ref[:, b0], err_msg=name)
        if name.startswith("layer_0."):
            # the reference's own inputs: the 1e-5 scale contract
            check_scales(a[:, 0], a_ref[:, 0], name)
            check_scales(r["mu"].float().numpy()[:, 0], g[f"mu{i}"][:, 0], name)
            np.testing.assert_array_equal(perm, perm_ref, err_msg=name)
        else:
            # inputs that went through layer 0's write-back: AGA's per-row 2x2 solve amplifies the
            # ~1e-7 input differences on ill-conditioned rows, so block 0's scales are held in
            # aggregate (measured in layer_1.mlp.gate_proj: 12 % of rows beyond 1e-3, max 7 %)
            a0, r0 = a[:, 0], a_ref[:, 0]
            rel = np.abs(a0 - r0) / np.maximum(np.abs(r0), 1e-6)
            assert np.median(rel) <= 1e-3 and np.mean(rel <= 1e-3) >= 0.75, (name, np.median(rel))
        agree = (T == T_ref).mean()
        if name.startswith("layer_0."):
            for s in range(0, m, 128):
                assert set(perm[s:s + 128]) == set(perm_ref[s:s + 128]), (name, s)
            assert agree >= 0.999, (name, agree)
        else:
            # different inputs: near-tie SSR picks may swap columns between neighbouring blocks
            overlap = np.mean([len(set(perm[s:s + 128]) & set(perm_ref[s:s + 128])) / len(perm_ref[s:s + 128])
                               for s in range(0, m, 128)])
            assert overlap >= 0.9 and agree >= 0.95, (name, overlap, agree)


def test_model_layer1_teacher_forced_vs_reference(pt2q):
    """decoder layer 1 fed the reference's OWN captured inputs (teacher forcing,
    tests/golden/model_llama2l_tf.npz) is held to the contract, not to aggregate bounds: the HIP
    engine reproduces the reference's loop (engine H^-1, the library-defined sums and tie order
    fixed to the contract's, see gen_golden.canonical_matvecs) bit for bit -- permutation,
    codes, alpha, mu -- on all seven linears.  Against the reference's unmodified quantize_layer
    on the same inputs (the fixture's ref_*), block-0 permutation and codes are exact, >= 97.9 %
    of all codes agree and block-0 scales meet the 1e-5 contract on the well-conditioned rows
    (test_oracle_golden.check_vs_unmodified_reference: the rest differ only through MKL's
    summation order, which this fixture records)."""
    from conftest import unpack2
    from test_oracle_golden import check_vs_unmodified_reference, layer1_inputs_tf
    g, names, data = layer1_inputs_tf()
    for i, (name, (W, X)) in enumerate(zip(names, data)):
        out = pt2q.quantize_layer(torch.from_numpy(W).cuda(), torch.from_numpy(X).cuda())
        m = int(g[f"m{i}"])
        np.testing.assert_array_equal(out.perm.cpu().numpy(), g[f"perm{i}"], err_msg=name)
        np.testing.assert_array_equal(out.T.cpu().numpy(), unpack2(g[f"T2_{i}"], m), err_msg=name)
        assert np.array_equal(out.alpha.cpu().numpy(), g[f"alpha{i}"]), name
        assert np.array_equal(out.mu.cpu().numpy(), g[f"mu{i}"]), name
        check_vs_unmodified_reference(g, i, name, out.perm.cpu().numpy(), out.T.cpu().numpy(),
                                      out.alpha.cpu().numpy(), out.mu.cpu().numpy())


def test_model_loop_layerwise_and_schedules_identical(pt2q):
    """PT2LLMQuantizer.quantize(propagate="layerwise") -- layer 0's inputs recorded once, every
    later layer fed by the previous layer's forward on its written-back weights -- quantises the
    same activations as the reference's full-model forward per layer (main.py:280-282), and the
    grams-first schedule (batched inverses, grouped loops) equals one unit per lane: every
    result of the three runs is bit-identical (model on the CPU, one thread, as above)."""
    runs = {}
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        for key, kw in {"model/gf": dict(propagate="model"), "layerwise/gf": dict(propagate="layerwise"),
                        "model/lanes": dict(propagate="model", schedule="lanes")}.items():
            model, samples = tiny_llama_and_samples()
            q = pt2q.PT2LLMQuantizer(model, None, "llama", block_size=128, use_ssr=True)
            timings = []
            runs[key] = q.quantize(samples, writeback="reference", timings=timings, **kw)
            assert len(timings) == 2 and all(t["total_s"] > 0 for t in timings)
    finally:
        torch.set_num_threads(threads)
    base = runs["model/gf"]
    assert len(base) == 14
    for key, got in runs.items():
        assert sorted(got) == sorted(base), key
        for name in base:
            for k in ("alpha", "mu", "T", "perm"):
                assert torch.equal(got[name][k], base[name][k]), (key, name, k)
