"""HIP path (libpt2q via the pt2q package) vs the CPU oracle (bit-exact) and vs the reference's
golden fixtures (codes/perm exact, scales within 1e-5).  Runs on an MI355X: `pytest -m gpu`."""
import numpy as np
import pytest
import torch

import synth
from conftest import golden_names, layer_inputs, load_golden
from oracle import oracle as orc
from test_oracle_golden import NEAR_TIE_LAYERS, _check_layer_sets, check_scales

pytestmark = pytest.mark.gpu

DEV = "cuda"


def cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    return t.detach().cpu().numpy()


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.uint32)
    b = np.ascontiguousarray(b, np.float32).view(np.uint32)
    # +0 and -0 compare equal (torch.equal semantics); everything else bitwise
    z = (a & 0x7FFFFFFF) == 0
    return np.array_equal(np.where(z, 0, a), np.where(z, 0, b))


# ------------------------------------------------------------------ building blocks

def oracle_gram(Xd):
    """The oracle Gram for device activations Xd: the 16-bit MFMA arithmetic for fp16/bf16
    (orc.gram16), the f32 fmaf chain for f32."""
    if Xd.dtype == torch.float16:
        return orc.gram16(host(Xd))
    if Xd.dtype == torch.bfloat16:
        return orc.gram16(Xd.cpu())
    return orc.gram(host(Xd))


def oracle_x(Xd):
    """Device activations as the oracle takes them (fp16 numpy / bf16 torch / f32 numpy)."""
    return Xd.cpu() if Xd.dtype == torch.bfloat16 else host(Xd)


@pytest.mark.parametrize("N,m,dt", [(300, 200, torch.float32), (1024, 384, torch.float32),
                                    (2048, 256, torch.float16), (512, 130, torch.bfloat16),
                                    (77, 40, torch.float16), (0, 64, torch.float16),
                                    (1000, 520, torch.bfloat16)])
def test_gram_bitexact(pt2q, N, m, dt):
    """Small / ragged shapes (m % 8 != 0 takes the register-staged 16-bit path; N = 0)."""
    X = synth.activations(7 + m, N, m)
    Xd = cuda(X).to(dt)
    G = pt2q.gram(Xd)
    ref = oracle_gram(Xd)
    assert bits_equal(host(G), ref)
    # accumulate (gptq.py add_batch): H = H + XᵀX (product rounded, then one add)
    G2 = pt2q.gram(Xd[: N // 2], G.clone(), accumulate=True)
    ref2 = ref + oracle_gram(Xd[: N // 2])
    assert bits_equal(host(G2), ref2)


@pytest.mark.parametrize("N,m,dt", [(2048, 4096, torch.float16), (1000, 4104, torch.bfloat16),
                                     (777, 4100, torch.float16), (17000, 2048, torch.float32),
                                     (1500, 4352, torch.bfloat16), (333, 8192, torch.float16),
                                     (64, 11008, torch.bfloat16)])
def test_gram_streamk_bitexact(pt2q, N, m, dt):
    """The balanced persistent Gram (static split of the tile line over one workgroup per CU,
    chains continued through fp32 partials: 16-bit X splits from m >= 4096; even tile rows: tile
    pairs worked by teams of two) must equal the oracle bit-for-bit, including ragged m / N
    (m % 8 != 0: register-staged operands)."""
    orc.set_threads(16)
    X = synth.activations(13 + m, N, m)
    Xd = cuda(X).to(dt)
    G = pt2q.gram(Xd)
    assert bits_equal(host(G), oracle_gram(Xd))


@pytest.mark.parametrize("N,m,dt,cut", [(1500, 8192, torch.float16, 1024), (2000, 11008, torch.bfloat16, 640),
                                        (4133, 13824, torch.float16, 4096)])
def test_gram_wide_tiles_continue(pt2q, N, m, dt, cut):
    """256 x 256 tiles (m % 256 == 0, >= 2 tile waves): data-parallel waves + stream-K pieces,
    a ragged last stage (N % 32 != 0), and a second launch continuing the chains
    (accumulate="continue") at a row cut: bit-identical to the one-launch Gram and, on sampled
    column blocks, to the oracle's 16-bit arithmetic."""
    from test_gpu_configs import sample_cols
    X = synth.activations(17 + m, N, m)
    Xd = cuda(X).to(dt)
    G = pt2q.gram(Xd)
    G2 = pt2q.gram(Xd[:cut], torch.empty_like(G))
    G2 = pt2q.gram(Xd[cut:], G2, accumulate="continue")
    Gh = host(G)
    assert bits_equal(host(G2), Gh)
    assert np.array_equal(Gh, Gh.T)
    orc.set_threads(16)
    S = sample_cols(m)
    Xs = Xd[:, torch.from_numpy(S).to(Xd.device)].contiguous()
    assert bits_equal(Gh[np.ix_(S, S)], orc.gram16(oracle_x(Xs)))


@pytest.mark.parametrize("m,N", [(64, 256), (100, 80), (256, 512), (384, 200), (700, 1500), (2200, 2400),
                                 (6400, 6500)])
def test_hessian_cholesky_inverse_bitexact(pt2q, m, N):
    """m = 2200: 512-row panels on one stream; m = 6400: the look-ahead (trailing terms of each
    panel on the side stream, joined before the next panel's terms)."""
    orc.set_threads(16)
    X = synth.activations(11 + m, N, m)
    G = orc.gram(X)
    H, damp = pt2q.prepare_hessian(cuda(G), N, 0.01)
    Hr, dr = orc.prepare_hessian(G, N, 0.01)
    assert bits_equal(host(H), Hr) and np.float32(host(damp)[0]) == np.float32(dr)
    Hinv, spd = pt2q.cholesky_inverse(H)
    Hinv_r, spd_r = orc.cholesky_inverse(Hr)
    assert spd and spd_r
    assert bits_equal(host(Hinv), Hinv_r)


@pytest.mark.parametrize("m,batch,chunk", [(100, 3, 32), (384, 4, 3), (2200, 2, 32), (4096, 3, 32),
                                            (6400, 2, 32), (11008, 2, 32)])
def test_hessian_inverse_batched_equals_per_item(pt2q, m, batch, chunk):
    """engine.hessian_inverse_batched (one launch per factorisation step for all items of a
    chunk) == prepare_hessian + cholesky_inverse per item, bit for bit; an item whose Hessian is
    not positive definite reports its own pivot and leaves the others intact (m = 6400: the
    per-item call uses the look-ahead, the batch does not -- same bits)."""
    Gs = []
    for z in range(batch):
        N = m + 37 * z
        Gs.append(pt2q.gram(pt2q.fill_synthetic((N, m), 50 + m + z, outliers=True, device="cuda")))
    Gs[1] = -Gs[1]  # damping a negative definite Gram: breakdown at the first pivot
    G = torch.stack(Gs).contiguous()
    Hinv, info = pt2q.engine.hessian_inverse_batched(G, 4096, 0.01, chunk=chunk)
    info = host(info)
    for z in range(batch):
        H, _ = pt2q.prepare_hessian(G[z], 4096, 0.01)
        want, spd = pt2q.cholesky_inverse(H)
        assert (info[z] == 0) == spd == (z != 1), (z, info[z])
        if spd:
            assert bits_equal(host(Hinv[z]), host(want)), z


def test_cholesky_breakdown_reports_and_falls_back(pt2q):
    H = np.eye(80, dtype=np.float32)
    H[37, 37] = -1.0
    Hinv, spd = pt2q.cholesky_inverse(cuda(H))
    assert not spd
    np.testing.assert_allclose(host(Hinv), np.linalg.pinv(H), atol=1e-6)


@pytest.mark.parametrize("seed", [0, 1])
def test_atq_stages_vs_oracle_and_reference(pt2q, seed):
    g = load_golden(f"atq_4096x128_s{seed}")
    W = synth.weights(int(g["wseed"]), 4096, 128)
    X = synth.activations(int(g["xseed"]), 512, 128)
    q = pt2q.AsymmetricTernaryQuantizer()
    Wd = cuda(W)
    a0, m0, T0 = q.ternary_init(Wd)
    ra0, rm0, rT0 = orc.ternary_init(W)
    assert bits_equal(host(a0), ra0) and bits_equal(host(m0), rm0) and np.array_equal(host(T0), rT0)
    np.testing.assert_array_equal(host(T0).astype(np.int8), g["T_init"])
    a1, m1, T1 = q.iterative_ternary_fitting(Wd, a0, m0, T0)
    ra1, rm1, rT1, rit = orc.iterative_ternary_fitting(W, ra0, rm0, rT0)
    assert bits_equal(host(a1), ra1) and bits_equal(host(m1), rm1) and np.array_equal(host(T1), rT1)
    assert int(q.last_itf_iters.item()) == rit
    np.testing.assert_array_equal(host(T1).astype(np.int8), g["T_itf"])
    check_scales(host(a1).ravel(), g["a_itf"], "a_itf")
    ga, gm = q.build_optimal_grid(Wd, T1)
    rga, rgm = orc.build_optimal_grid(W, rT1)
    assert bits_equal(host(ga), rga) and bits_equal(host(gm), rgm)
    Tr = q.flexible_round(Wd, ga, gm)
    assert np.array_equal(host(Tr), orc.flexible_round(W, rga, rgm))
    a2, m2 = q.activation_aware_grid_alignment(Wd, T1, cuda(X))
    ra2, rm2 = orc.activation_aware_grid_alignment(W, rT1, X)
    assert bits_equal(host(a2), ra2) and bits_equal(host(m2), rm2)
    check_scales(host(a2).ravel(), g["a_aga"], "a_aga")
    af, mf, Tf = q.quantize(Wd, cuda(X))
    raf, rmf, rTf, _ = orc.atq_quantize(W, X)
    assert bits_equal(host(af), raf) and bits_equal(host(mf), rmf) and np.array_equal(host(Tf), rTf)


def test_atq_edges_vs_reference(pt2q):
    g = load_golden("atq_edges")
    q = pt2q.AsymmetricTernaryQuantizer()
    Z = torch.zeros(64, 128, device=DEV)
    a, m, T = q.quantize(Z)
    np.testing.assert_array_equal(host(T).astype(np.int8), g["zero_T"])
    np.testing.assert_array_equal(host(a).ravel(), g["zero_alpha"])
    np.testing.assert_array_equal(host(m).ravel(), g["zero_mu"])
    assert int(q.last_itf_iters.item()) == 0
    a, m, T = q.quantize(Z, cuda(synth.activations(220, 64, 128)))
    np.testing.assert_array_equal(host(T).astype(np.int8), g["zerox_T"])
    np.testing.assert_array_equal(host(a).ravel(), g["zerox_alpha"])
    Wc = g["const_W"]
    a, m, T = q.quantize(cuda(Wc))
    np.testing.assert_array_equal(host(T).astype(np.int8), g["const_T"])
    ra, rm, rT, _ = orc.atq_quantize(Wc)
    assert bits_equal(host(a), ra) and bits_equal(host(m), rm)
    Wr = synth.weights(130, 32, 128)
    T = q.flexible_round(cuda(Wr), cuda(g["round_alpha"]), cuda(g["round_mu"]))
    np.testing.assert_array_equal(host(T).astype(np.int8), g["round_T"])


@pytest.mark.parametrize("b", [128, 1000])
def test_atq_round_at_thresholds(pt2q, b):
    """flexible_round (quantizer.py:127-131) on quotients within 40 ulp of ±0.5: the HIP round
    decides RN(d / as) against ±0.5 with no division (atq.hip round_code); every code must equal
    the oracle's correctly rounded division.  b = 128: the row kernel; b = 1000: the wide one."""
    rng = np.random.default_rng(b)
    n = 256
    alpha = np.exp(rng.uniform(np.log(1e-6), np.log(10.0), n)).astype(np.float32)
    mu = np.where(np.arange(n) % 2 == 0, 0.0, rng.standard_normal(n) * 0.01).astype(np.float32)
    d = np.repeat((alpha * np.float32(0.5))[:, None], b, axis=1)
    k = rng.integers(-40, 41, (n, b))
    for step in range(1, 41):
        sel = np.abs(k) >= step
        d[sel] = np.nextafter(d[sel], np.where(k[sel] > 0, np.inf, -np.inf).astype(np.float32))
    d *= np.where(rng.random((n, b)) < 0.5, -1, 1).astype(np.float32)
    W = (d + mu[:, None]).astype(np.float32)
    q = pt2q.AsymmetricTernaryQuantizer()
    T = q.flexible_round(cuda(W), cuda(alpha[:, None]), cuda(mu[:, None]))
    ref = orc.flexible_round(W, alpha[:, None], mu[:, None])
    assert np.array_equal(host(T), ref)
    assert 0.2 < (ref == 0).mean() < 0.8  # both sides of the thresholds are exercised


@pytest.mark.parametrize("b", [128, 300, 512, 1000])
def test_atq_one_signed_codes_and_general_t(pt2q, b):
    """Grid counts at their extremes: an ITF whose second grid sees codes almost all of one sign
    (|sum t| near b, past the 256 a 512-multiplier packing could carry), and build_optimal_grid
    on a caller T that is not ternary (quantizer.py:71-108 accepts any T): both vs the oracle,
    bit-exact."""
    n = 96
    rng = np.random.default_rng(b)
    W = rng.uniform(1.0, 1.1, (n, b)).astype(np.float32)
    T0 = np.ones((n, b), np.float32)
    zc = rng.choice(b, 6, replace=False)
    W[:, zc] = 0.0
    T0[:, zc] = -1.0
    T0[(rng.random((n, b)) < 0.1) & (T0 > 0)] = 0.0  # the first round makes these +1 as well
    W[: n // 2] *= -1.0  # half the rows one-signed the other way
    T0[: n // 2] *= -1.0
    q = pt2q.AsymmetricTernaryQuantizer()
    Wd = cuda(W)
    ga, gm = q.build_optimal_grid(Wd, cuda(T0))
    rga, rgm = orc.build_optimal_grid(W, T0)
    assert bits_equal(host(ga), rga) and bits_equal(host(gm), rgm)
    _, _, rTa, _ = orc.iterative_ternary_fitting(W, rga, rgm, T0, max_iter=1)
    assert np.abs(rTa.sum(axis=1)).min() > 0.8 * b  # what the second (packed) grid must carry
    a1, m1, T1 = q.iterative_ternary_fitting(Wd, ga, gm, cuda(T0))
    ra1, rm1, rT1, rit = orc.iterative_ternary_fitting(W, rga, rgm, T0)
    assert np.array_equal(host(T1), rT1)
    assert bits_equal(host(a1), ra1) and bits_equal(host(m1), rm1)
    assert int(q.last_itf_iters.item()) == rit >= 2
    Tg = rng.standard_normal((n, b)).astype(np.float32)  # not ternary
    ga, gm = q.build_optimal_grid(Wd, cuda(Tg))
    rga, rgm = orc.build_optimal_grid(W, Tg)
    assert bits_equal(host(ga), rga) and bits_equal(host(gm), rgm)


def test_atq_per_channel_b1000_vs_reference(pt2q):
    """b = 1000 > 512: the streaming one-lane-per-row kernel (atq_wide_*), per-method stages
    and the fused quantize, vs the oracle (bit-exact) and the reference's fixture."""
    g = load_golden("atq_256x1000")
    W = synth.weights(int(g["wseed"]), 256, 1000)
    X = synth.activations(int(g["xseed"]), 300, 1000)
    q = pt2q.AsymmetricTernaryQuantizer()
    Wd = cuda(W)
    af, mf, Tf = q.quantize(Wd, cuda(X))
    raf, rmf, rTf, rit = orc.atq_quantize(W, X)
    assert bits_equal(host(af), raf) and bits_equal(host(mf), rmf) and np.array_equal(host(Tf), rTf)
    assert int(q.last_itf_iters.item()) == rit
    np.testing.assert_array_equal(host(Tf).astype(np.int8), g["T"])
    check_scales(host(af).ravel(), g["alpha"], "alpha")
    check_scales(host(mf).ravel(), g["mu"], "mu")


@pytest.mark.parametrize("n,b", [(200, 1500), (64, 777), (130, 4100)])
def test_atq_wide_stages_vs_oracle(pt2q, n, b):
    W = synth.weights(140 + b, n, b)
    X = synth.activations(240 + b, 128, b)
    q = pt2q.AsymmetricTernaryQuantizer()
    Wd = cuda(W)
    a0, m0, T0 = q.ternary_init(Wd)
    ra0, rm0, rT0 = orc.ternary_init(W)
    assert bits_equal(host(a0), ra0) and bits_equal(host(m0), rm0) and np.array_equal(host(T0), rT0)
    a1, m1, T1 = q.iterative_ternary_fitting(Wd, a0, m0, T0)
    ra1, rm1, rT1, rit = orc.iterative_ternary_fitting(W, ra0, rm0, rT0)
    assert bits_equal(host(a1), ra1) and bits_equal(host(m1), rm1) and np.array_equal(host(T1), rT1)
    assert int(q.last_itf_iters.item()) == rit
    ga, gm = q.build_optimal_grid(Wd, T1)
    rga, rgm = orc.build_optimal_grid(W, rT1)
    assert bits_equal(host(ga), rga) and bits_equal(host(gm), rgm)
    assert np.array_equal(host(q.flexible_round(Wd, ga, gm)), orc.flexible_round(W, rga, rgm))
    a2, m2 = q.activation_aware_grid_alignment(Wd, T1, cuda(X))
    ra2, rm2 = orc.activation_aware_grid_alignment(W, rT1, X)
    assert bits_equal(host(a2), ra2) and bits_equal(host(m2), rm2)


def test_atq_wide_zero_block(pt2q):
    """All-zero wide block: ITF exits at iteration 0 (quantizer.py:164) -> alpha = mu = 0."""
    q = pt2q.AsymmetricTernaryQuantizer()
    a, m, T = q.quantize(torch.zeros(70, 900, device=DEV))
    assert int(q.last_itf_iters.item()) == 0
    assert not host(T).any() and not host(a).any() and not host(m).any()


def test_per_channel_config5_shape(pt2q):
    """BASELINE config 5 shape class: per-channel (block_size = m) 5120 x 5120, N = 4096, SSR on
    (a single block: blk = all columns in order), bit-exact vs the oracle."""
    n = m = 5120
    N = 4096
    W = synth.weights(5120, n, m)
    X = synth.activations(5121, N, m)
    orc.set_threads(16)
    Xd = cuda(X).to(torch.bfloat16)
    out = pt2q.quantize_layer(cuda(W), Xd, block_size=m, use_ssr=True)
    ref = _oracle_m(W, oracle_x(Xd), m, True)
    _assert_layer_bitexact(out, ref)
    np.testing.assert_array_equal(host(out.perm), np.arange(m))


def test_atq_wide_block_vs_oracle(pt2q):
    """b = 512 (the widest register-resident block; per-channel runs use the same kernel)."""
    W = synth.weights(110, 256, 512)
    X = synth.activations(210, 300, 512)
    q = pt2q.AsymmetricTernaryQuantizer()
    a, m, T = q.quantize(cuda(W), cuda(X))
    ra, rm, rT, _ = orc.atq_quantize(W, X)
    assert bits_equal(host(a), ra) and bits_equal(host(m), rm) and np.array_equal(host(T), rT)


@pytest.mark.parametrize("name", ["ssr_4096x4096", "ssr_1024x1000_subset"])
def test_ssr_vs_oracle_and_reference(pt2q, name):
    g = load_golden(name)
    n, m = int(g["n"]), int(g["m"])
    W = synth.weights(int(g["wseed"]), n, m)
    rem = g["rem"] if "rem" in g else np.arange(m, dtype=np.int64)
    Wd = cuda(W)
    sim = pt2q.compute_column_similarity_to_mean(Wd, cuda(rem))
    assert bits_equal(host(sim), orc.ssr_similarity(W, rem))
    blk, newrem = pt2q.select_next_block_ssr(Wd, cuda(rem), 128)
    np.testing.assert_array_equal(host(blk), g["blk"])
    np.testing.assert_array_equal(host(newrem), g["newrem"])


@pytest.mark.parametrize("n,m,b,dup", [(256, 700, 128, 7), (512, 4096, 128, 3),
                                       (64, 300, 256, 2), (128, 11008, 128, 5)])
def test_ssr_topk_ties_vs_oracle(pt2q, n, m, b, dup):
    """Exact similarity ties: repeated columns and all-zero columns tie bitwise, so the pick
    and its order rest on the position tie-break (value desc, position asc)."""
    W = synth.weights(40 + m, n, m)
    W[:, 1::dup] = W[:, :1]  # every dup-th column equals column 0
    W[:, 5::11] = 0.0
    rem = np.arange(m, dtype=np.int64)[(np.arange(m) % 13) != 4]
    blk, newrem = pt2q.select_next_block_ssr(cuda(W), cuda(rem), b)
    rblk, rnew = orc.select_next_block_ssr(W, rem, b)
    np.testing.assert_array_equal(host(blk), rblk)
    np.testing.assert_array_equal(host(newrem), rnew)


@pytest.mark.parametrize("n,m", [(4096, 700), (11008, 600), (320, 500)])
def test_ssr_similarity_quotient_paths(pt2q, n, m):
    """The similarity kernel divides by the column norm through an exact reciprocal quotient
    when every element and the norm are in range, else by the division itself (wave-uniform):
    columns with tiny (< 2^-60) or huge (> 2^60) elements and tiny-norm columns take the
    fallback; every similarity must stay bit-identical to the oracle's plain division."""
    W = synth.weights(70 + n, n, m)
    W[:, 3] *= 1e-25          # every element below 2^-60 (and a tiny norm)
    W[7, 10] = 3e18           # one element above 2^60
    W[:5, 20] = 1e-20         # a few tiny elements in an otherwise normal column
    W[:, 30] = 0.0            # an all-zero column (norm clamped to 1e-8)
    W[:, 40] *= 1e-12         # small norm, elements still in range
    W[::2, 50:90] = 0.0       # pruned columns: zeros keep the reciprocal path (nonzero-min gate)
    W[1, 60] = 1e-30          # ... except beside a tiny nonzero element
    W[:, 95] *= 1e13          # norm above 2^40: the division
    W[:, 96] = 0.0
    W[5, 96] = 1e-30          # a lone tiny element: quotient ~1, division path
    rem = np.arange(m, dtype=np.int64)[(np.arange(m) % 7) != 2]
    rem = np.concatenate([rem, np.array([2, 9], dtype=np.int64)])
    rem.sort()
    sim = pt2q.compute_column_similarity_to_mean(cuda(W), cuda(rem))
    assert bits_equal(host(sim), orc.ssr_similarity(W, rem))


def test_fill_synthetic_matches_numpy(pt2q):
    a = pt2q.fill_synthetic((300, 257), 1234, std=0.02)
    np.testing.assert_array_equal(host(a), synth.weights(1234, 300, 257))
    b = pt2q.fill_synthetic((64, 1000), 99, std=1.0, outliers=True)
    np.testing.assert_array_equal(host(b), synth.activations(99, 64, 1000))


@pytest.mark.parametrize("count", [1001, 4096 * 3])
def test_pack_unpack_matches_reference_layout(pt2q, count):
    """1001 codes: the per-byte kernel; 12288 (a multiple of 16): the 16-codes-per-thread kernel."""
    T = (synth.centered24(5, count).astype(np.int64) % 3 - 1).astype(np.int8)
    packed, shape = pt2q.pack_ternary(cuda(T))
    # utils.py:202-217 layout: {-1,0,1} -> {0,1,2}, element 4q+s at bits 2s of byte q
    flat = np.concatenate([T + 1, np.zeros((-len(T)) % 4, np.int8)]).astype(np.uint8).reshape(-1, 4)
    want = flat[:, 0] | (flat[:, 1] << 2) | (flat[:, 2] << 4) | (flat[:, 3] << 6)
    np.testing.assert_array_equal(host(packed), want)
    np.testing.assert_array_equal(host(pt2q.unpack_ternary(packed, shape)), T)


# ------------------------------------------------------------------ whole layers

def _oracle_m(W, X, bs, ssr, percdamp=0.01):
    return orc.quantize_layer_m(W, X, block_size=bs, use_ssr=ssr, percdamp=percdamp)


def _assert_layer_bitexact(out, ref):
    np.testing.assert_array_equal(host(out.perm), ref["perm"])
    np.testing.assert_array_equal(host(out.T), ref["T"])
    assert bits_equal(host(out.alpha), ref["alpha"])
    assert bits_equal(host(out.mu), ref["mu"])
    np.testing.assert_array_equal(host(out.iters), ref["iters"])


@pytest.mark.parametrize("name", [n for n in golden_names("layer_m_") if n != "layer_m_notspd"])
def test_layer_m_vs_reference_and_oracle(pt2q, name):
    g = load_golden(name)
    W, X = layer_inputs(g)
    bs, ssr = int(g["block_size"]), bool(g["use_ssr"])
    out = pt2q.quantize_layer(cuda(W), cuda(X), block_size=bs, use_ssr=ssr)
    assert out.spd
    _assert_layer_bitexact(out, _oracle_m(W, X, bs, ssr))
    if name in NEAR_TIE_LAYERS:
        _check_layer_sets(g, {"perm": host(out.perm), "T": host(out.T), "alpha": host(out.alpha)}, bs)
        return
    np.testing.assert_array_equal(host(out.perm), g["perm"])
    np.testing.assert_array_equal(host(out.T), g["T"])
    check_scales(host(out.alpha), g["alpha"], "alpha")


def test_pt2llm_quantizer_surface(pt2q):
    """main.py:102-230 call shape: nn.Linear + 3-D activations -> CPU dict."""
    g = load_golden("layer_m_c1_ssr")
    W, X = layer_inputs(g)
    lin = torch.nn.Linear(W.shape[1], W.shape[0], bias=False)
    lin.weight.data = torch.from_numpy(W.copy())
    q = pt2q.PT2LLMQuantizer(model=None, tokenizer=None, device="cuda")
    res = q.quantize_layer(lin, "layer_0.q_proj", torch.from_numpy(X.reshape(2, -1, X.shape[1])))
    assert set(res) == {"alpha", "mu", "T", "perm"}
    assert res["T"].dtype == torch.int8 and res["perm"].dtype == torch.int64
    assert res["T"].device.type == "cpu"
    np.testing.assert_array_equal(res["T"].numpy(), g["T"])
    np.testing.assert_array_equal(res["perm"].numpy(), g["perm"])


@pytest.mark.parametrize("name", golden_names("layer_g_"))
def test_layer_g_vs_reference_and_oracle(pt2q, name):
    g = load_golden(name)
    W, X = layer_inputs(g)
    m = W.shape[1]
    lin = torch.nn.Linear(m, W.shape[0], bias=False).to(DEV)
    lin.weight.data = cuda(W)
    gq = pt2q.GPTQ(lin, int(g["block_size"]), 0.01)
    for c in np.array_split(X, int(g["nbatch"])):
        gq.add_batch(cuda(c))
    alpha, mu, T, perm = gq.quantize(use_ssr=bool(g["use_ssr"]))
    Hs = np.zeros((m, m), np.float32)
    for c in np.array_split(X, int(g["nbatch"])):
        orc.gram_accumulate(Hs, c)
    ref = orc.quantize_layer_g(W, Hs, X.shape[0], block_size=int(g["block_size"]),
                               use_ssr=bool(g["use_ssr"]))
    np.testing.assert_array_equal(host(perm), ref["perm"])
    np.testing.assert_array_equal(host(T), ref["T"])
    assert bits_equal(host(alpha), ref["alpha"]) and bits_equal(host(mu), ref["mu"])
    np.testing.assert_array_equal(host(T).astype(np.int8), g["T"])
    np.testing.assert_array_equal(host(perm), g["perm"])
    # gptq.py:201-230 reconstruction
    Wq = gq.get_quantized_weight()
    bs = int(g["block_size"])
    want = np.empty_like(W)
    for k in range(ref["alpha"].shape[1]):
        cols = ref["perm"][k * bs:(k + 1) * bs]
        want[:, cols] = ref["alpha"][:, k:k + 1] * ref["T"][:, cols] + ref["mu"][:, k:k + 1]
    assert bits_equal(host(Wq), want)


def test_layer_graph_replay_matches_eager(pt2q):
    """The hipGraph-captured layer (bench path) replays to the same bits as the oracle."""
    W = synth.weights(41, 1024, 768)
    X = synth.activations(42, 1536, 768)
    Wd, Xd = cuda(W), cuda(X)
    lg = pt2q.LayerGraph(Wd, Xd)
    out = lg.replay()
    torch.cuda.synchronize()
    assert lg.spd()
    ref = _oracle_m(W, X, 128, True)
    _assert_layer_bitexact(out, ref)
    # new inputs in place -> replay recomputes
    W2 = synth.weights(43, 1024, 768)
    Wd.copy_(cuda(W2))
    out = lg.replay()
    torch.cuda.synchronize()
    _assert_layer_bitexact(out, _oracle_m(W2, X, 128, True))


def test_layer_not_spd_pinv_fallback(pt2q):
    g = load_golden("layer_m_notspd")
    W, X = layer_inputs(g)
    out = pt2q.quantize_layer(cuda(W), cuda(X), block_size=128, use_ssr=True,
                              percdamp=float(g["percdamp"]))
    assert not out.spd
    np.testing.assert_array_equal(host(out.perm), g["perm"])
    b0 = g["perm"][:128]
    np.testing.assert_array_equal(host(out.T)[:, b0], g["T"][:, b0])


@pytest.mark.parametrize("n,m,N,ssr,bs", [
    (1024, 1024, 2048, True, 128),
    (768, 3072, 512, True, 128),     # GPT-2 mlp.c_proj shape, 24 blocks
    (2304, 768, 1024, False, 128),   # GPT-2 c_attn shape, sequential blocks
    (640, 1000, 700, True, 256),     # ragged m, wider blocks
    (1000, 640, 700, True, 128),     # n % 16 != 0: the block ATQ's per-element form (no 16-byte stage)
    (1008, 520, 600, True, 128),     # n % 16 == 0 with a ragged last block (16-byte stage, then b = 8)
])
def test_layer_m_bitexact_larger(pt2q, n, m, N, ssr, bs):
    W = synth.weights(1000 + n, n, m)
    X = synth.activations(2000 + m, N, m)
    out = pt2q.quantize_layer(cuda(W), cuda(X), block_size=bs, use_ssr=ssr)
    _assert_layer_bitexact(out, _oracle_m(W, X, bs, ssr))


def test_layer_m_fp16_inputs(pt2q):
    """fp16 layer + activations (configs C3/C4): W is used as its exact fp32 upcast, the Gram of
    the fp16 activations follows the 16-bit MFMA arithmetic (orc.gram16)."""
    W = synth.weights(31, 512, 640)
    X = synth.activations(32, 1024, 640)
    Wh, Xh = cuda(W).half(), cuda(X).half()
    out = pt2q.quantize_layer(Wh, Xh)
    ref = _oracle_m(host(Wh.float()), host(Xh), 128, True)
    _assert_layer_bitexact(out, ref)


def test_layer_headline_shape_bitexact(pt2q):
    """Llama-2-7B q_proj shape (4096x4096, 32 blocks), N=2048: GPU == oracle bit-for-bit."""
    orc.set_threads(16)
    W = synth.weights(4096, 4096, 4096)
    X = synth.activations(4097, 2048, 4096)
    out = pt2q.quantize_layer(cuda(W), cuda(X))
    ref = _oracle_m(W, X, 128, True)
    _assert_layer_bitexact(out, ref)
    # size-independent properties
    p = host(out.perm)
    assert np.array_equal(np.sort(p), np.arange(4096))
    T = host(out.T)
    assert set(np.unique(T)) <= {-1, 0, 1}


@pytest.mark.parametrize("n,m,N,bs,ssr", [(384, 640, 1024, 256, True),    # blocks wider than 128
                                          (256, 300, 512, 512, True),     # per-channel: bs >= m
                                          (200, 700, 800, 700, False)])
def test_gptq_wide_blocks_vs_oracle(pt2q, n, m, N, bs, ssr):
    """Variant G with blocks wider than 128 columns: S = H_bbᵀH_bb on the f32 MFMA
    GEMM, S1 / d in the aga_s1 order; bit-exact vs the oracle's s1_from_hess_block."""
    W = synth.weights(600 + n, n, m)
    X = synth.activations(601 + m, N, m, outliers=False)
    lin = torch.nn.Linear(m, n, bias=False).to(DEV)
    lin.weight.data = cuda(W)
    gq = pt2q.GPTQ(lin, bs, 0.01)
    for c in np.array_split(X, 2):
        gq.add_batch(cuda(c))
    alpha, mu, T, perm = gq.quantize(use_ssr=ssr)
    Hs = np.zeros((m, m), np.float32)
    for c in np.array_split(X, 2):
        orc.gram_accumulate(Hs, c)
    ref = orc.quantize_layer_g(W, Hs, N, block_size=bs, use_ssr=ssr)
    np.testing.assert_array_equal(host(perm), ref["perm"])
    np.testing.assert_array_equal(host(T), ref["T"])
    assert bits_equal(host(alpha), ref["alpha"]) and bits_equal(host(mu), ref["mu"])


@pytest.mark.parametrize("n,m,bs", [(300, 700, 128), (256, 1024, 256), (64, 200, 37)])
def test_error_feedback_entry_vs_oracle(pt2q, n, m, bs):
    """pt2q_error_feedback (main.py:187-214 for one block, standalone C entry) vs the oracle's
    orc_error_feedback: bit-exact W after the update; rem in arbitrary (non-sorted) order."""
    rng = np.random.default_rng(n + m)
    W = synth.weights(700 + n, n, m)
    cols = rng.permutation(m)
    blk, rem = cols[:bs].astype(np.int64), cols[bs:].astype(np.int64)
    E = synth.weights(701 + n, n, bs) * np.float32(0.1)
    X = synth.activations(702 + m, 2 * m, m)
    H, _ = orc.prepare_hessian(orc.gram(X), 2 * m)
    Hinv, spd = orc.cholesky_inverse(H)
    assert spd
    Wd = cuda(W)
    pt2q.error_feedback(Wd, cuda(blk), cuda(rem), cuda(E), cuda(Hinv))
    ref = orc.error_feedback(W, blk, rem, E, Hinv)
    assert bits_equal(host(Wd), ref)
    assert bits_equal(host(Wd)[:, blk], W[:, blk])  # the block's own columns are untouched


def test_reference_call_shapes_with_cpu_tensors(pt2q):
    """The reference runs these on CPU tensors; here they compute on the GPU and hand results
    back on the caller's device, identical to the GPU-tensor call."""
    W = synth.weights(810, 256, 384)
    X = synth.activations(811, 300, 384)
    q = pt2q.AsymmetricTernaryQuantizer()
    a_c, m_c, T_c = q.quantize(torch.from_numpy(W[:, :128].copy()), torch.from_numpy(X[:, :128].copy()))
    a_g, m_g, T_g = q.quantize(cuda(W[:, :128]), cuda(X[:, :128]))
    assert a_c.device.type == "cpu" and T_c.device.type == "cpu"
    assert bits_equal(a_c.numpy(), host(a_g)) and np.array_equal(T_c.numpy(), host(T_g))
    rem = torch.arange(384)
    blk, new = pt2q.select_next_block_ssr(torch.from_numpy(W), rem, 128)
    assert blk.device.type == "cpu" and new.device.type == "cpu"
    rblk, rnew = orc.select_next_block_ssr(W, rem.numpy(), 128)
    np.testing.assert_array_equal(blk.numpy(), rblk)
    np.testing.assert_array_equal(new.numpy(), rnew)
    lin = torch.nn.Linear(384, 256, bias=False)
    lin.weight.data = torch.from_numpy(W.copy())
    gq = pt2q.GPTQ(lin, 128, 0.01)
    gq.add_batch(torch.from_numpy(X.copy()))
    alpha, mu, T, perm = gq.quantize()
    assert alpha.device.type == "cpu" and perm.device.type == "cpu"
    Hs = orc.gram(X)
    ref = orc.quantize_layer_g(W, Hs, X.shape[0])
    np.testing.assert_array_equal(perm.numpy(), ref["perm"])
    np.testing.assert_array_equal(T.numpy(), ref["T"])
    assert gq.get_quantized_weight().device.type == "cpu"


@pytest.mark.parametrize("n,m,count,ssr,dt", [(256, 512, 3, True, torch.float32), (384, 700, 5, True, torch.float16),
                                             (512, 384, 2, False, torch.float32), (1024, 1024, 16, True, torch.float16),
                                             (4096, 4096, 3, True, torch.float16), (1000, 512, 3, True, torch.float16),
                                             (11008, 4096, 3, True, torch.float16),
                                             (4096, 11008, 2, True, torch.float16)])
def test_blocks_group_equals_per_linear(pt2q, n, m, count, ssr, dt):
    """pt2q_quantize_blocks_group (one launch per block step for all linears, grid.z = linear)
    == quantize_blocks on each linear alone, bit for bit: every linear has its own W, raw Gram
    and H^-1 (and some share them, as q/k/v do); ragged m, fp16 weights, sequential blocks, a
    full group of 16, and the 7B step's MLP shapes as the bench groups them (gate/up 11008 x
    4096: n > 4096 takes the split similarity kernel ssr_sim_split_kernel; down 4096 x 11008)."""
    Ws, Gs, Hs = [], [], []
    for z in range(count):
        X = pt2q.fill_synthetic((2 * m + 64 * z, m), 300 + 7 * z, outliers=True, device="cuda").half()
        G = pt2q.gram(X) if z % 3 != 2 else Gs[-1]  # every third linear shares its input's Gram
        Hinv, spd = pt2q.hessian_inverse(G, X.shape[0]) if z % 3 != 2 else (Hs[-1], True)
        assert spd
        Gs.append(G)
        Hs.append(Hinv)
        Ws.append(pt2q.fill_synthetic((n, m), 900 + z, std=0.02, device="cuda").to(dt))
    got = pt2q.engine.quantize_blocks_group(Ws, Gs, Hs, 128, ssr)
    for z in range(count):
        want = pt2q.quantize_blocks(Ws[z], Gs[z], Hs[z], 128, ssr)
        for a, b in ((got[z].perm, want.perm), (got[z].T, want.T), (got[z].alpha, want.alpha),
                     (got[z].mu, want.mu), (got[z].iters, want.iters)):
            assert bits_equal(host(a), host(b)), z


@pytest.mark.parametrize("n,m", [(11008, 4096), (4096, 11008)])
def test_blocks_group_vs_oracle_at_mlp_shapes(pt2q, n, m):
    """The grouped block loop the 7B bench times (pt2q_quantize_blocks_group at the MLP shapes,
    fp16 weights, N = 2048) pinned to the oracle directly, not only through the per-linear path:
    two linears sharing one Gram and H^-1 (gate/up read the same input), each vs
    orc.quantize_blocks fed the device G and H^-1 -- codes, permutation, scales and ITF counts
    bit for bit (main.py:158-215, reorder.py:107-143)."""
    X = pt2q.fill_synthetic((2048, m), 4100 + m, outliers=True, device="cuda").half()
    G = pt2q.gram(X)
    Hinv, spd = pt2q.hessian_inverse(G, X.shape[0])
    assert spd
    Ws = [pt2q.fill_synthetic((n, m), 910 + z, std=0.02, device="cuda").half() for z in range(2)]
    got = pt2q.engine.quantize_blocks_group(Ws, [G, G], [Hinv, Hinv], 128, True)
    torch.cuda.synchronize()
    orc.set_threads(16)
    Gh, Hh = host(G), host(Hinv)
    for z in range(2):
        ref = orc.quantize_blocks(host(Ws[z].float()), Gh, Hh, 128, True, 1)
        np.testing.assert_array_equal(host(got[z].perm), ref["perm"])
        np.testing.assert_array_equal(host(got[z].T), ref["T"])
        assert bits_equal(host(got[z].alpha), ref["alpha"]) and bits_equal(host(got[z].mu), ref["mu"])
        np.testing.assert_array_equal(host(got[z].iters), ref["iters"])


@pytest.mark.parametrize("m,N,batch,dt", [(256, 1000, 3, torch.float16), (512, 2048, 5, torch.bfloat16),
                                          (4096, 8192, 3, torch.float16), (768, 64, 130, torch.float16),
                                          (1280, 192, 2, torch.float16), (1024, 4160, 2, torch.bfloat16),
                                          (11008, 1024, 2, torch.float16), (8192, 256, 3, torch.bfloat16),
                                          (13824, 128, 2, torch.float16), (768, 2048, 5, torch.float32),
                                          (3072, 512, 3, torch.float32), (1000, 300, 4, torch.float32),
                                          (200, 64, 130, torch.float32), (514, 100, 3, torch.float32),
                                          (3072, 2048, 12, torch.float32)])
def test_gram_batched_equals_per_item(pt2q, m, N, batch, dt):
    """pt2q_gram_batched (one data-parallel launch for every item, 256 x 256 tiles, each tile one
    chain over all rows) == pt2q_gram on each item alone, bit for bit; ragged N, chains of 2 / 6 /
    130 stages (prologue only, steady + draining ring), m = 11008, bf16, and more items than one
    launch takes (130 > 128).  m = 8192 / 11008 / 13824 run the searched tile orders
    (gram_order.inc: every item's whole runs, then every item's partial-run tiles); fp32 items
    (GPT-2 widths at C2's 2048 rows, a ragged m, 130 items) take the LDS-DMA f32 chain GEMM
    (gemmx_gram_kernel), m % 4 != 0 (514) the generic batched f32 GEMM."""
    Xs = [pt2q.fill_synthetic((N, m), 40 + z, outliers=True, device="cuda").to(dt) for z in range(batch)]
    G = torch.empty((batch, m, m), dtype=torch.float32, device="cuda")
    pt2q.engine.gram_batched(Xs, G)
    for z in (0, batch // 2, batch - 1):
        assert bits_equal(host(G[z]), host(pt2q.gram(Xs[z]))), z


def test_stage_timing_brackets_the_block_loop(pt2q):
    """pt2q_stage_timing (bench.py's live stage rooflines): a grouped block loop on one stream
    records SSR, ATQ and EF intervals whose sum stays within the wall of the call; disabled, it
    records nothing.  The results are the untimed call's, bit for bit."""
    lib = pt2q._lib
    n, m, count = 1024, 1024, 4
    Ws, Gs, Hs = [], [], []
    for z in range(count):
        X = pt2q.fill_synthetic((4 * m, m), 500 + z, outliers=True, device="cuda").half()
        G = pt2q.gram(X)
        Hinv, spd = pt2q.hessian_inverse(G, X.shape[0])
        assert spd
        Gs.append(G)
        Hs.append(Hinv)
        Ws.append(pt2q.fill_synthetic((n, m), 600 + z, std=0.02, device="cuda").half())
    want = pt2q.engine.quantize_blocks_group(Ws, Gs, Hs, 128, True)
    torch.cuda.synchronize()
    lib.stage_timing(True)
    try:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        got = pt2q.engine.quantize_blocks_group(Ws, Gs, Hs, 128, True)
        ev1.record()
        torch.cuda.synchronize()
    finally:
        lib.stage_timing(False)
    t = lib.stage_timing_read()
    B = m // 128
    assert t["records"] == 2 + 3 * B, t  # setup + per block (SSR, ATQ, EF) + outputs
    assert t["ssr"] > 0 and t["atq"] > 0 and t["ef"] > 0, t
    wall = ev0.elapsed_time(ev1)
    assert sum(t[k] for k in lib.TIMERS) <= wall * 1.01 + 0.05, (t, wall)
    for z in range(count):
        for a, b in ((got[z].perm, want[z].perm), (got[z].T, want[z].T), (got[z].alpha, want[z].alpha)):
            assert bits_equal(host(a), host(b)), z
    lib.stage_timing(True)
    lib.stage_timing(False)
    pt2q.engine.quantize_blocks_group(Ws, Gs, Hs, 128, True)
    assert lib.stage_timing_read()["records"] == 0
