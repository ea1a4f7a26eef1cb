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


def gen_hessian512():
    """m = 512 beside the m = 256 pair: the element-wise H^-1 pin (test_hessian_inverse_elementwise)."""
    print("Hessian / inverse, m = 512 (main.py:127-141)")
    m, N = 512, 1024
    X = torch.from_numpy(synth.activations(300 + N + m, N, m))
    H = X.T @ X
    H = H / X.shape[0]
    damp = 0.01 * torch.diag(H).mean()
    H.diagonal().add_(damp)
    Hinv = torch.cholesky_inverse(torch.linalg.cholesky(H.float()))
    save(f"hess_{m}_n{N}", xseed=300 + N + m, N=N, m=m, Hinv=Hinv.numpy(),
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


@contextlib.contextmanager
def canonical_matvecs():
    """Inside the block, while the reference's AGA method runs (quantizer.py:177-248), every
    matrix-VECTOR product it issues through Tensor.__matmul__ (S·1, 1ᵀS1, T·S1, W·S1, (W∘T)·S1,
    T²·S1 -- MKL sgemv, whose summation order is internal to MKL and differs by CPU code path)
    runs in the PT2Q contract order instead (oracle.rowsum_seq / sequential / oracle.matvec16).
    Also torch.topk (reorder.py:133), whose order among EXACTLY tied similarities is
    std::nth_element's, takes ties by position (the contract's total order).  Every other
    operation of the reference, the SSR similarity's product included, is untouched.  On ill-conditioned AGA rows (the random-init
    model's layer-1 activations) the 2x2 solve amplifies the ulp-level order differences of
    those sums far beyond the 1e-5 scale contract, so a bit-level pin needs one fixed order."""
    from oracle import oracle as orc
    mm = torch.Tensor.__matmul__

    def canon(a, b):
        if a.dim() == 2 and b.dim() == 2 and b.shape[1] == 1 and a.shape[1] == b.shape[0] \
                and a.dtype == torch.float32 and b.dtype == torch.float32:
            A, x = a.detach().contiguous().numpy(), b.detach().contiguous().numpy()[:, 0]
            if a.shape[0] == 1 and bool(np.all(A == 1.0)):  # d = 1ᵀS1: j-ascending sum
                y = orc.rowsum_seq(x[None, :])
            elif bool(np.all(x == 1.0)):                     # S1 = S·1: l-ascending sums
                y = orc.rowsum_seq(A)
            else:                                            # row products: DOT16
                y = orc.matvec16(A, x)
            return torch.from_numpy(np.asarray(y, np.float32).reshape(-1, 1))
        return mm(a, b)
    cls = rq.AsymmetricTernaryQuantizer
    aga = cls.activation_aware_grid_alignment

    def aga_canon(self, *args, **kw):
        torch.Tensor.__matmul__ = canon
        try:
            return aga(self, *args, **kw)
        finally:
            torch.Tensor.__matmul__ = mm
    cls.activation_aware_grid_alignment = aga_canon
    # torch.topk (reorder.py:133) breaks exact ties in std::nth_element's order; the contract
    # (and the oracle) order ties by position: value descending, then position ascending
    topk = torch.topk

    def stable_topk(x, k, *args, **kw):
        if args or kw:
            return topk(x, k, *args, **kw)
        idx = torch.sort(x, descending=True, stable=True).indices[:k]
        return torch.return_types.topk((x[idx], idx))
    torch.topk = stable_topk
    try:
        yield
    finally:
        cls.activation_aware_grid_alignment = aga
        torch.topk = topk


def gen_model_tf():
    """Teacher-forced pin of decoder layer 1 of the model loop: the reference's
    PT2LLMQuantizer.quantize on the 2-layer Llama of gen_model, with its quantize_layer wrapped to
    record the activations each layer-1 linear receives (captured after layer 0's write-back,
    main.py:262-299) -- one array per distinct input (q/k/v share one, gate/up share one).
    For each layer-1 linear the fixture also holds the reference's own loop components run on
    exactly those inputs and the layer's ORIGINAL weight with the engine's canonical H^-1
    (ref_loop_with_hinv, as gen_loop16) and the AGA's matrix-vector sums in the contract order
    (canonical_matvecs), so the GPU engine fed the same inputs must reproduce codes and
    permutation exactly and scales within the contract.  The reference's own quantize_layer
    output on the same inputs (MKL H^-1 and sums) is stored beside it (ref_*)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import oracle as orc
    orc.set_threads(8)
    print("teacher-forced model-loop fixture (layer 1 inputs, main.py:262-299)")
    model, samples = tiny_llama_and_samples()
    q = rm.PT2LLMQuantizer(model, None, model_type="llama", block_size=128, use_ssr=True,
                           device="cpu")
    q.get_calibration_data = lambda: samples
    seen = {}
    orig = q.quantize_layer

    def rec(layer, name, acts):
        if name.startswith("layer_1."):
            seen[name] = (layer.weight.data.clone().numpy(), acts.detach().clone().numpy())
        return orig(layer, name, acts)
    q.quantize_layer = rec
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        params = q.quantize()
    names = sorted(seen)
    inputs, kw = {}, {"names": np.array(names)}
    for i, name in enumerate(names):
        W, A = seen[name]
        X = np.ascontiguousarray(A.reshape(-1, A.shape[-1]).astype(np.float32))
        key = next((k for k, v in inputs.items() if v.shape == X.shape and np.array_equal(v, X)), None)
        if key is None:
            key = f"X{len(inputs)}"
            inputs[key] = X
        kw[f"xkey{i}"] = key
        G = orc.gram(X)
        H, _ = orc.prepare_hessian(G, X.shape[0])
        Hinv, spd = orc.cholesky_inverse(H)
        assert spd
        with canonical_matvecs():
            r = ref_loop_with_hinv(W, X, Hinv)
        kw[f"alpha{i}"], kw[f"mu{i}"], kw[f"perm{i}"] = r["alpha"], r["mu"], r["perm"]
        kw[f"T2_{i}"] = pack2(r["T"])
        kw[f"m{i}"] = W.shape[1]
        # the reference's own quantize_layer on the same inputs (its MKL H^-1)
        p = params[name]
        kw[f"ref_perm{i}"] = p["perm"].numpy()
        kw[f"ref_T2_{i}"] = pack2(p["T"].numpy())
        kw[f"ref_alpha{i}"], kw[f"ref_mu{i}"] = p["alpha"].numpy(), p["mu"].numpy()
        o = orc.quantize_layer_m(W, X)
        print(f"    {name}: oracle vs common-H^-1 reference loop: perm "
              f"{'==' if np.array_equal(o['perm'], r['perm']) else '!='}, codes "
              f"{(o['T'] == r['T']).mean():.6f}, alpha max|d| {np.abs(o['alpha'] - r['alpha']).max():.2e}")
    kw.update(inputs)
    save("model_llama2l_tf", **kw)


def gen_ppl():
    """The reference's evaluate_perplexity (utils.py:128-186) with its data source replaced
    (load_dataset -> fixed text, the tokenizer -> a stub returning fixed token ids; there is no
    network), on the tiny Llama of gen_model: (a) the fp32 model as built, for two window lengths
    (a ragged last window; seq_len > L); (b) the model after the reference's own
    replace_linear_with_ternary (model.py:174-225) with per-block ATQ params of every decoder
    linear (stored, 2-bit packed)."""
    import utils as ru
    import model as rmod
    print("perplexity fixture (utils.py:128-186)")
    torch.manual_seed(2)
    ids = torch.randint(0, TINY_LLAMA["vocab_size"], (1, 300))

    class StubTok:
        def __call__(self, text, return_tensors="pt"):
            return {"input_ids": ids.clone()}
    orig = ru.load_dataset
    ru.load_dataset = lambda *a, **k: {"text": ["offline", "stub"]}
    try:
        model, samples = tiny_llama_and_samples()
        ppl = {s_: ru.evaluate_perplexity(model, StubTok(), seq_len=s_, device=torch.device("cpu"))
               for s_ in (128, 512)}
        # ternary params: the reference's ATQ per 128-column block without activations
        # (quantizer.py:250-277, X = None: no AGA -- the AGA of this random-init model yields
        # alphas up to ~1e28 and a NaN perplexity), columns in order (perm = arange)
        atq = rq.AsymmetricTernaryQuantizer()
        params, kw = {}, {}
        for name, mod in sorted(model.named_modules()):
            if isinstance(mod, torch.nn.Linear) and ".layers." in f".{name}":
                W = mod.weight.data.clone()
                a_, m_, T_ = [], [], []
                for c0 in range(0, W.shape[1], 128):
                    a, mu, T = atq.quantize(W[:, c0:c0 + 128])
                    a_.append(a); m_.append(mu); T_.append(T)
                params[name] = {"alpha": torch.cat(a_, 1), "mu": torch.cat(m_, 1),
                                "T": torch.cat(T_, 1).to(torch.int8), "perm": torch.arange(W.shape[1])}
        for i, name in enumerate(sorted(params)):
            kw[f"tname{i}"] = name
            kw[f"talpha{i}"] = params[name]["alpha"].numpy()
            kw[f"tmu{i}"] = params[name]["mu"].numpy()
            kw[f"tT2_{i}"] = pack2(params[name]["T"].numpy())
        rmod.replace_linear_with_ternary(model, params, block_size=128)
        ppl_t = ru.evaluate_perplexity(model, StubTok(), seq_len=128, device=torch.device("cpu"))
    finally:
        ru.load_dataset = orig
    print(f"    ppl fp32 {ppl}, ternary (reference TernaryLinear, {len(params)} linears) {ppl_t}")
    save("ppl_llama2l", ids=ids.numpy(), seq_lens=np.array([128, 512]),
         ppl=np.array([ppl[128], ppl[512]], np.float64), ppl_ternary_128=np.float64(ppl_t),
         nlin=len(params), **kw)


GENERATORS = {"layers": gen_layers, "atq": gen_atq, "ssr": gen_ssr, "hessian": gen_hessian, "hessian512": gen_hessian512,
              "trace": gen_trace, "examples": gen_examples, "wide": gen_wide,
              "ternary": gen_ternary, "fp16": gen_fp16, "loop16": gen_loop16,
              "model": gen_model, "model_tf": gen_model_tf, "ppl": gen_ppl}

if __name__ == "__main__":
    # `python gen_golden.py [group ...]` regenerates only the named groups (default: all)
    for g in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[g]()
