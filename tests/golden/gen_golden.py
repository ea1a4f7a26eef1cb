"""Generate the golden parity fixtures from the REFERENCE implementation.

Run here (the reference is importable only in the build container):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

It imports /root/reference (quantizer.py, reorder.py, gptq.py, main.py), runs them on CPU with
torch.set_num_threads(1) (the pinned oracle configuration) on counter-generated
inputs (tests/synth.py), and stores ONLY data: the seeds/shapes needed to regenerate the inputs
and the reference's outputs.  No reference source is copied.  The test-suite checks the CPU
oracle (oracle/) against these, and the HIP path against the oracle.

The per-block "trace" fixtures drive the reference's own components in the order of
main.py:158-215 and assert that the traced loop reproduces PT2LLMQuantizer.quantize_layer
bit-for-bit before anything is saved.
"""
import contextlib
import io
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (synth)
REF = "/root/reference"
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402

torch.set_num_threads(1)
import quantizer as rq  # noqa: E402
import reorder as rr  # noqa: E402
import gptq as rg  # noqa: E402
import main as rm  # noqa: E402

OUT = HERE


def save(name, **kw):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **kw)
    print(f"  {name}.npz {os.path.getsize(path) / 1024:.1f} KiB")


def linear(W):
    lin = torch.nn.Linear(W.shape[1], W.shape[0], bias=False)
    lin.weight.data = torch.from_numpy(W.copy())
    return lin


def ref_layer_m(W, X, use_ssr, bs=128, percdamp=0.01):
    q = rm.PT2LLMQuantizer(model=None, tokenizer=None, device="cpu", block_size=bs,
                           use_ssr=use_ssr, percdamp=percdamp)
    with contextlib.redirect_stdout(io.StringIO()):
        return q.quantize_layer(linear(W), "layer", torch.from_numpy(X.copy()))


def ref_layer_g(W, X, use_ssr, bs=128, nbatch=2):
    g = rg.GPTQ(linear(W), bs, 0.01)
    for c in np.array_split(X, nbatch):
        g.add_batch(torch.from_numpy(c.copy()))
    a, mu, T, perm = g.quantize(use_ssr=use_ssr)
    return dict(alpha=a, mu=mu, T=T, perm=perm)


def gen_layers():
    print("full-layer fixtures (variant M, main.py:102-230)")
    cases = [
        ("layer_m_c1_ssr", 512, 512, 128, True, 128, True),
        ("layer_m_c1_nossr", 512, 512, 128, False, 128, True),
        ("layer_m_1024x768_n2048", 1024, 768, 2048, True, 128, True),
        ("layer_m_384x300_n200", 384, 300, 200, True, 128, True),
        ("layer_m_perchannel_256x256", 256, 256, 512, True, 512, True),
        ("layer_m_512x512_n2048_noout", 512, 512, 2048, True, 128, False),
    ]
    for name, n, m, N, ssr, bs, outl in cases:
        ws, xs = 1 + n, 2 + m
        W = synth.weights(ws, n, m)
        X = synth.activations(xs, N, m, outliers=outl)
        r = ref_layer_m(W, X, ssr, bs)
        save(name, variant="M", n=n, m=m, N=N, wseed=ws, xseed=xs, outliers=outl, use_ssr=ssr,
             block_size=bs, alpha=r["alpha"].numpy(), mu=r["mu"].numpy(),
             T=r["T"].numpy().astype(np.int8), perm=r["perm"].numpy())
    print("full-layer fixtures (variant G, gptq.py:59-199; no outlier channels: with x20 outliers the"
          " H_bb² AGA is catastrophically ill-conditioned in the reference itself)")
    gcases = [
        ("layer_g_768x640_n1024_ssr", 768, 640, 1024, True),
        ("layer_g_384x300_n200_ssr", 384, 300, 200, True),
        ("layer_g_512x512_n1024_nossr", 512, 512, 1024, False),
    ]
    for name, n, m, N, ssr in gcases:
        ws, xs = 3 + n, 4 + m
        W = synth.weights(ws, n, m)
        X = synth.activations(xs, N, m, outliers=False)
        r = ref_layer_g(W, X, ssr)
        save(name, variant="G", n=n, m=m, N=N, wseed=ws, xseed=xs, outliers=False, use_ssr=ssr,
             block_size=128, nbatch=2, alpha=r["alpha"].numpy(), mu=r["mu"].numpy(),
             T=r["T"].numpy().astype(np.int8), perm=r["perm"].numpy())
    # not positive definite: zero input column + percdamp 0 -> cholesky fails -> pinv (main.py:140)
    n, m, N = 128, 256, 64
    W = synth.weights(77, n, m)
    X = synth.activations(78, N, m)
    X[:, 5] = 0.0
    H = torch.from_numpy(X).T @ torch.from_numpy(X) / N
    try:
        torch.linalg.cholesky(H)
        spd = True
    except RuntimeError:
        spd = False
    assert not spd
    r = ref_layer_m(W, X, True, 128, percdamp=0.0)
    save("layer_m_notspd", variant="M", n=n, m=m, N=N, wseed=77, xseed=78, zero_col=5,
         percdamp=0.0, use_ssr=True, block_size=128, alpha=r["alpha"].numpy(),
         mu=r["mu"].numpy(), T=r["T"].numpy().astype(np.int8), perm=r["perm"].numpy())


def gen_atq():
    print("ATQ known answers (quantizer.py:32-293)")
    atq = rq.AsymmetricTernaryQuantizer()
    for seed in (0, 1):
        W = torch.from_numpy(synth.weights(100 + seed, 4096, 128))
        X = torch.from_numpy(synth.activations(200 + seed, 512, 128))
        a0, m0, T0 = atq.ternary_init(W)
        a1, m1, T1 = atq.iterative_ternary_fitting(W, a0, m0, T0)
        a2, m2 = atq.activation_aware_grid_alignment(W, T1, X)
        af, mf, Tf = atq.quantize(W, X)
        an, mn, Tn = atq.quantize(W)
        assert torch.equal(Tf, T1) and torch.equal(Tn, T1)
        assert torch.equal(af, a2) and torch.equal(an, a1)
        save(f"atq_4096x128_s{seed}", wseed=100 + seed, xseed=200 + seed, n=4096, b=128, N=512,
             a_init=a0.numpy().ravel(), m_init=m0.numpy().ravel(), T_init=T0.numpy().astype(np.int8),
             a_itf=a1.numpy().ravel(), m_itf=m1.numpy().ravel(), T_itf=T1.numpy().astype(np.int8),
             a_aga=a2.numpy().ravel(), m_aga=m2.numpy().ravel())
    # general block width (per-channel path): b = 1000 (not a multiple of 16)
    W = torch.from_numpy(synth.weights(110, 256, 1000))
    X = torch.from_numpy(synth.activations(210, 300, 1000))
    af, mf, Tf = atq.quantize(W, X)
    save("atq_256x1000", wseed=110, xseed=210, n=256, b=1000, N=300, alpha=af.numpy().ravel(),
         mu=mf.numpy().ravel(), T=Tf.numpy().astype(np.int8))
    # edge cases: zero block, constant rows, explicit negative alpha in flexible_round,
    # build_optimal_grid on a given T
    Z = torch.zeros(64, 128)
    az, mz, Tz = atq.quantize(Z)
    azx, mzx, Tzx = atq.quantize(Z, torch.from_numpy(synth.activations(220, 64, 128)))
    Wc = torch.from_numpy(synth.weights(120, 64, 128))
    Wc[::4] = Wc[::4, :1]                       # every 4th row constant
    Wc[1] = 0.0                                 # one all-zero row
    ac, mc, Tc = atq.quantize(Wc)
    acx, mcx, Tcx = atq.quantize(Wc, torch.from_numpy(synth.activations(221, 64, 128)))
    Wr = torch.from_numpy(synth.weights(130, 32, 128))
    alpha_neg = torch.from_numpy(np.linspace(-0.02, 0.02, 32, dtype=np.float32))[:, None]
    mu_r = torch.from_numpy(synth.weights(131, 32, 1))
    Tr = atq.flexible_round(Wr, alpha_neg, mu_r)
    Tg = torch.from_numpy((synth.centered24(132, 32 * 128).reshape(32, 128) % 3 - 1).astype(np.float32))
    ag, mg = atq.build_optimal_grid(Wr, Tg)
    save("atq_edges", zero_alpha=az.numpy().ravel(), zero_mu=mz.numpy().ravel(),
         zero_T=Tz.numpy().astype(np.int8), zerox_alpha=azx.numpy().ravel(),
         zerox_mu=mzx.numpy().ravel(), zerox_T=Tzx.numpy().astype(np.int8),
         const_W=Wc.numpy(), const_alpha=ac.numpy().ravel(), const_mu=mc.numpy().ravel(),
         const_T=Tc.numpy().astype(np.int8), constx_alpha=acx.numpy().ravel(),
         constx_mu=mcx.numpy().ravel(), constx_T=Tcx.numpy().astype(np.int8),
         round_alpha=alpha_neg.numpy().ravel(), round_mu=mu_r.numpy().ravel(),
         round_T=Tr.numpy().astype(np.int8), grid_T=Tg.numpy().astype(np.int8),
         grid_alpha=ag.numpy().ravel(), grid_mu=mg.numpy().ravel())


def gen_ssr():
    print("SSR known answers (reorder.py:36-61,107-143)")
    W = torch.from_numpy(synth.weights(11, 4096, 4096))
    rem = torch.arange(4096)
    sim = rr.compute_column_similarity_to_mean(W, rem)
    blk, newrem = rr.select_next_block_ssr(W, rem, 128)
    save("ssr_4096x4096", wseed=11, n=4096, m=4096, sim=sim.numpy(), blk=blk.numpy(),
         newrem=newrem.numpy())
    W = torch.from_numpy(synth.weights(12, 1024, 1000))
    keep = np.sort(np.argsort(synth.centered24(13, 1000))[:700]).astype(np.int64)
    rem = torch.from_numpy(keep)
    sim = rr.compute_column_similarity_to_mean(W, rem)
    blk, newrem = rr.select_next_block_ssr(W, rem, 128)
    save("ssr_1024x1000_subset", wseed=12, n=1024, m=1000, rem=keep, sim=sim.numpy(),
         blk=blk.numpy(), newrem=newrem.numpy())


def gen_hessian():
    print("Hessian / inverse (main.py:127-141)")
    for N in (512, 128):
        m = 256
        X = torch.from_numpy(synth.activations(300 + N, N, m))
        H = X.T @ X
        H = H / X.shape[0]
        damp = 0.01 * torch.diag(H).mean()
        H.diagonal().add_(damp)
        Hinv = torch.cholesky_inverse(torch.linalg.cholesky(H.float()))
        save(f"hess_256_n{N}", xseed=300 + N, N=N, m=m, H=H.numpy(), Hinv=Hinv.numpy(),
             damp=np.float32(damp.item()))


def gen_trace():
    """Teacher-forced per-block trace of main.py:158-215 using the reference's own components."""
    print("per-block trace (variant M, SSR on)")
    n, m, N, bs = 512, 384, 1024, 128
    W0 = synth.weights(401, n, m)
    X0 = synth.activations(402, N, m)
    W = torch.from_numpy(W0.copy())
    X = torch.from_numpy(X0.copy())
    H = X.T @ X
    H = H / X.shape[0]
    H.diagonal().add_(0.01 * torch.diag(H).mean())
    H_inv = torch.cholesky_inverse(torch.linalg.cholesky(H.float()))
    atq = rq.AsymmetricTernaryQuantizer()
    rem = torch.arange(m)
    rec = {}
    k = 0
    T_full = torch.zeros(n, m, dtype=torch.int8)
    alphas, mus, perm = [], [], []
    while len(rem) > 0:
        if len(rem) > bs:
            rec[f"sim{k}"] = rr.compute_column_similarity_to_mean(W, rem).numpy()
        blk, rem = rr.select_next_block_ssr(W, rem, bs)
        Wb = W[:, blk]
        a, mu, Tb = atq.quantize(Wb, X[:, blk])
        rec[f"blk{k}"] = blk.numpy()
        rec[f"alpha{k}"] = a.numpy().ravel()
        rec[f"mu{k}"] = mu.numpy().ravel()
        rec[f"T{k}"] = Tb.numpy().astype(np.int8)
        T_full[:, blk] = Tb.to(torch.int8)
        alphas.append(a); mus.append(mu); perm += blk.tolist()
        E = Wb - (a * Tb + mu)
        if len(rem) > 0:
            C = H_inv[blk][:, rem] / H_inv[blk, blk].unsqueeze(1).clamp(min=1e-8)
            W[:, rem] -= E @ C
        k += 1
    ref = ref_layer_m(W0, X0, True, bs)
    assert torch.equal(ref["T"], T_full) and ref["perm"].tolist() == perm
    assert torch.equal(ref["alpha"], torch.cat(alphas, 1)) and torch.equal(ref["mu"], torch.cat(mus, 1))
    save("trace_m_512x384_n1024", wseed=401, xseed=402, n=n, m=m, N=N, block_size=bs, nblocks=k,
         Hinv=H_inv.numpy(), **rec)


def gen_examples():
    print("examples.py smoke values (examples.py:15-77)")
    torch.manual_seed(42)
    W = torch.randn(256, 512)
    X = torch.randn(32, 512)
    atq = rq.AsymmetricTernaryQuantizer(max_iter=100)
    a0, m0, T0 = atq.ternary_init(W)
    e0 = rq.compute_quantization_error(W, atq.dequantize(a0, m0, T0))
    a1, m1, T1 = atq.iterative_ternary_fitting(W, a0, m0, T0)
    e1 = rq.compute_quantization_error(W, atq.dequantize(a1, m1, T1))
    a2, m2 = atq.activation_aware_grid_alignment(W, T1, X)
    ox0 = rq.compute_output_error(W, atq.dequantize(a1, m1, T1), X)
    ox1 = rq.compute_output_error(W, atq.dequantize(a2, m2, T1), X)
    save("examples_atq", W=W.numpy(), X=X.numpy(), err_init=e0, err_itf=e1, out_err_itf=ox0,
         out_err_aga=ox1, T_itf=T1.numpy().astype(np.int8))


def gen_wide():
    print("wide-block fixtures (b > 512: per-channel, BASELINE config 5 shape class)")
    cases = [
        ("layer_m_perchannel_640x1024_n2048", 640, 1024, 2048, True, 1024, True),
        ("layer_m_wide_320x1600_b640_n1024", 320, 1600, 1024, True, 640, True),
    ]
    for name, n, m, N, ssr, bs, outl in cases:
        ws, xs = 1 + n, 2 + m
        W = synth.weights(ws, n, m)
        X = synth.activations(xs, N, m, outliers=outl)
        r = ref_layer_m(W, X, ssr, bs)
        save(name, variant="M", n=n, m=m, N=N, wseed=ws, xseed=xs, outliers=outl, use_ssr=ssr,
             block_size=bs, alpha=r["alpha"].numpy(), mu=r["mu"].numpy(),
             T=r["T"].numpy().astype(np.int8), perm=r["perm"].numpy())


def gen_ternary():
    print("TernaryLinear forward fixtures (model.py:17-127, fp16 on CPU, reference semantics)")
    import model as rmod
    for name, n, m, N, bs, tokens in (("ternary_linear_384x512", 384, 512, 256, 128, 15),
                                      ("ternary_linear_200x1000_pc", 200, 1000, 512, 1000, 4)):
        ws, xs = 11 + n, 12 + m
        W = synth.weights(ws, n, m)
        X = synth.activations(xs, N, m)
        r = ref_layer_m(W, X, True, bs)
        torch.manual_seed(n)
        bias = (torch.randn(n) * 0.1).half()
        lay = rmod.TernaryLinear(m, n, block_size=bs, bias=True, dtype=torch.float16)
        lay.set_quantized_params(r["alpha"].half(), r["mu"].half(), r["T"], r["perm"], bias)
        x = (torch.from_numpy(synth.activations(13 + m, tokens, m)) * 0.5).half()
        with torch.no_grad():
            out = lay(x)
        save(name, n=n, m=m, N=N, wseed=ws, xseed=xs, block_size=bs, alpha=r["alpha"].numpy(),
             mu=r["mu"].numpy(), T=r["T"].numpy().astype(np.int8), perm=r["perm"].numpy(),
             bias=bias.numpy(), x=x.numpy(), out=out.numpy())


def round16(a, dtype):
    """fp16 / bf16 rounding of an fp32 array, back in fp32 (exact: 16-bit values are fp32)."""
    if dtype == "fp16":
        return a.astype(np.float16).astype(np.float32)
    return torch.from_numpy(a).bfloat16().float().numpy()


def gen_fp16():
    """16-bit layers (configs C3/C4 fp16, C5 bf16).  The reference cannot run fp16/bf16 through
    its error feedback (main.py:214 dtype mismatch), so its output for a 16-bit layer
    is the fp32-upcast layer: W and X rounded to 16 bits, then run in fp32 (every 16-bit value is
    exact in fp32).  The HIP path takes the 16-bit tensors themselves (16-bit MFMA Gram)."""
    print("16-bit-input layer fixtures (variant M, fp32-upcast reference)")
    cases = [
        ("layer_m16_512x512_n2048", "fp16", 512, 512, 2048, 128),
        ("layer_m16_1024x768_n2048", "fp16", 1024, 768, 2048, 128),
        # (768 x 3072 and 1024 x 2048: see gen_loop16 -- whole-layer results there depend on
        # H⁻¹ rounding, so the loop is pinned with the engine's H⁻¹)
        ("layer_m16_bf16_640x1024_pc", "bf16", 640, 1024, 1024, 1024),
    ]
    for name, dt, n, m, N, bs in cases:
        ws, xs = 5 + n, 6 + m
        W = round16(synth.weights(ws, n, m), dt)
        X = round16(synth.activations(xs, N, m), dt)
        r = ref_layer_m(W, X, True, bs)
        save(name, variant="M", dtype=dt, n=n, m=m, N=N, wseed=ws, xseed=xs, outliers=True,
             use_ssr=True, block_size=bs, alpha=r["alpha"].numpy(), mu=r["mu"].numpy(),
             T=r["T"].numpy().astype(np.int8), perm=r["perm"].numpy())


def pack2(T):
    """int8 codes {-1,0,1} (n x m) -> 2 bits each, row-wise, MSB first (conftest.unpack2)."""
    c = (T.astype(np.int16) + 1).astype(np.uint8)
    bits = (c[..., None] >> np.array([1, 0], np.uint8)) & 1
    return np.packbits(bits.reshape(T.shape[0], -1), axis=1)


def ref_loop_with_hinv(W, X, Hinv, bs=128):
    """main.py:158-230 driven by the reference's own components (reorder.select_next_block_ssr,
    quantizer.AsymmetricTernaryQuantizer.quantize, the error feedback of main.py:199-214) with a
    GIVEN H⁻¹ in place of main.py:136-141.  gen_trace checks this restatement against
    quantize_layer bit-for-bit when H⁻¹ is the reference's own."""
    W = torch.from_numpy(W.copy())
    X = torch.from_numpy(X.copy())
    H_inv = torch.from_numpy(Hinv)
    n, m = W.shape
    atq = rq.AsymmetricTernaryQuantizer()
    rem = torch.arange(m)
    T_full = torch.zeros(n, m, dtype=torch.int8)
    alphas, mus, perm = [], [], []
    while len(rem) > 0:
        blk, rem = rr.select_next_block_ssr(W, rem, bs)
        Wb = W[:, blk]
        a, mu, Tb = atq.quantize(Wb, X[:, blk])
        T_full[:, blk] = Tb.to(torch.int8)
        alphas.append(a); mus.append(mu); perm += blk.tolist()
        E = Wb - (a * Tb + mu)
        if len(rem) > 0:
            C = H_inv[blk][:, rem] / H_inv[blk, blk].unsqueeze(1).clamp(min=1e-8)
            W[:, rem] -= E @ C
    return dict(alpha=torch.cat(alphas, 1).numpy(), mu=torch.cat(mus, 1).numpy(), T=T_full.numpy(),
                perm=np.array(perm, np.int64))


def gen_loop16():
    """Full-size block-loop pins for 16-bit layers whose whole-layer result depends on H⁻¹
    rounding (d >= 3k: a different but equally valid fp32 inverse -- MKL's vs the engine's
    canonical chains, rel. diff ~1e-4 -- moves SSR picks from block ~4 on).  The reference's
    own loop components run on the fp32 upcast of the 16-bit tensors with the ENGINE's H⁻¹ (the
    CPU oracle's orc.gram16 -> prepare_hessian -> cholesky_inverse, which the HIP path matches
    bit-for-bit); H⁻¹ itself is pinned to the reference separately (hess_* fixtures)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import oracle as orc
    orc.set_threads(8)
    print("16-bit block-loop fixtures (reference loop, engine H^-1)")
    for name, dt, n, m, N in (("loop16_768x3072_n2048", "fp16", 768, 3072, 2048),
                              ("loop16_1024x2048_n2048", "fp16", 1024, 2048, 2048)):
        ws, xs = 7 + n, 8 + m
        W = round16(synth.weights(ws, n, m), dt)
        X = round16(synth.activations(xs, N, m), dt)
        G = orc.gram16(X.astype(np.float16))
        H, _ = orc.prepare_hessian(G, N)
        Hinv, spd = orc.cholesky_inverse(H)
        assert spd
        r = ref_loop_with_hinv(W, X, Hinv)
        save(name, variant="M", dtype=dt, n=n, m=m, N=N, wseed=ws, xseed=xs, outliers=True,
             use_ssr=True, block_size=128, alpha=r["alpha"], mu=r["mu"],
             T2=pack2(r["T"]),
             perm=r["perm"])


TINY_LLAMA = dict(vocab_size=512, hidden_size=256, intermediate_size=384, num_hidden_layers=2,
                  num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=256)


def tiny_llama_and_samples():
    """A 2-layer Llama built from config (no download) with torch.manual_seed(0), fp32, and three
    64-token calibration samples (torch.manual_seed(1)).  tests/test_gpu_model.py rebuilds the
    same model and samples and checks the state-dict checksum stored with the fixture."""
    import transformers
    cfg = transformers.LlamaConfig(**TINY_LLAMA)
    torch.manual_seed(0)
    model = transformers.LlamaForCausalLM(cfg).eval()
    torch.manual_seed(1)
    samples = [torch.randint(0, TINY_LLAMA["vocab_size"], (1, 64)) for _ in range(3)]
    return model, samples


def state_checksum(model):
    return np.array([float(p.detach().double().sum()) for p in model.state_dict().values()])


def gen_model():
    """The reference's model-level loop PT2LLMQuantizer.quantize (main.py:232-311): hooks,
    calibration forwards, quantize_layer per linear and the _dequantize_weight write-back
    (main.py:313-335, wrong under SSR -- SURVEY §0.5), with get_calibration_data overridden on
    the instance (the reference downloads wikitext; there is no network)."""
    print("model-loop fixture (2-layer Llama, main.py:232-311)")
    model, samples = tiny_llama_and_samples()
    csum = state_checksum(model)
    q = rm.PT2LLMQuantizer(model, None, model_type="llama", block_size=128, use_ssr=True,
                           device="cpu")
    q.get_calibration_data = lambda: samples
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        params = q.quantize()
    kw = {"checksum": csum, "names": np.array(sorted(params))}
    for i, name in enumerate(sorted(params)):
        p = params[name]
        kw[f"alpha{i}"] = p["alpha"].numpy()
        kw[f"mu{i}"] = p["mu"].numpy()
        kw[f"T2_{i}"] = pack2(p["T"].numpy())
        kw[f"perm{i}"] = p["perm"].numpy()
        kw[f"m{i}"] = p["T"].shape[1]
    save("model_llama2l", **kw)


GENERATORS = {"layers": gen_layers, "atq": gen_atq, "ssr": gen_ssr, "hessian": gen_hessian,
              "trace": gen_trace, "examples": gen_examples, "wide": gen_wide,
              "ternary": gen_ternary, "fp16": gen_fp16, "loop16": gen_loop16,
              "model": gen_model}

if __name__ == "__main__":
    # `python gen_golden.py [group ...]` regenerates only the named groups (default: all)
    for g in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[g]()
