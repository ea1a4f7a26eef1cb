"""The bench workload and every BASELINE.json config shape, HIP path vs the CPU oracle, plus the
16-bit reference fixtures (VERDICT r1 "do this" #1 and #2).

Large shapes are checked stage by stage so that the oracle finishes in seconds:
  * the Gram on sampled column blocks: G[S, S] of the device Gram vs the oracle's 16-bit MFMA
    arithmetic (orc.gram16) on X[:, S] -- every output element's chain depends only on its two
    columns, so a column subset reproduces those entries exactly;
  * the damped Hessian's inverse: device (public path) vs orc.cholesky_inverse, fed the device G;
  * the whole block loop: orc.quantize_blocks fed the device G and H⁻¹ vs the fused
    pt2q_quantize_layer outputs (codes, permutation, scales, ITF iterations: bit-exact);
  * size-independent properties: perm is a permutation of range(m), codes in {-1, 0, 1}, every
    block's ITF count < max_iter, every scale finite.
Reference: main.py:102-230 (variant M), configs C2-C5 of BASELINE.json."""
import numpy as np
import pytest
import torch

import synth
from conftest import golden_names, layer_inputs16, load_golden, unpack2
from oracle import oracle as orc
from test_gpu_parity import bits_equal, host
from test_oracle_golden import NEAR_TIE_LAYERS, _check_layer, _check_layer_sets, check_scales

pytestmark = pytest.mark.gpu

DEV = "cuda"


def sample_cols(m, width=64, count=4):
    """`count` blocks of `width` columns spread over [0, m): first, last and interior blocks, so
    the sampled G[S, S] covers diagonal and far off-diagonal tiles and both matrix edges."""
    starts = sorted({0, m - width, *(int(m * f) // 8 * 8 for f in np.linspace(0, 1, count)[1:-1])})
    return np.concatenate([np.arange(s, min(s + width, m)) for s in starts])


def host_x(Xd):
    """Device activations as the oracle takes them (fp16 numpy / bf16 torch / f32 numpy)."""
    return Xd.cpu() if Xd.dtype == torch.bfloat16 else host(Xd)


def check_layer_staged(pt2q, Wd, Xd, bs=128, ssr=True, check_hinv=True):
    n, m = Wd.shape
    N = Xd.shape[0]
    ws = pt2q.LayerWorkspace(n, m, bs, Wd.device)
    out = pt2q.quantize_layer(Wd, Xd, block_size=bs, use_ssr=ssr, workspace=ws)
    assert out.spd
    G = ws.gram_view(m).clone()
    torch.cuda.synchronize()
    orc.set_threads(16)
    # 1) Gram on sampled column blocks
    S = sample_cols(m)
    Xs = Xd[:, torch.from_numpy(S).to(Xd.device)].contiguous()
    Gs_ref = orc.gram16(host_x(Xs)) if Xd.dtype != torch.float32 else orc.gram(host(Xs))
    Gh = host(G)
    assert bits_equal(Gh[np.ix_(S, S)], Gs_ref), "sampled Gram tiles differ from the oracle"
    assert np.array_equal(Gh, Gh.T)
    # 2) H⁻¹ (public path) vs the oracle, both from the device Gram
    B = -(-m // bs) if bs < m else 1
    if B > 1:
        Hinv, spd = pt2q.hessian_inverse(G, N)
        assert spd
        Hinv = host(Hinv)
        if check_hinv:
            Hr, _ = orc.prepare_hessian(Gh, N)
            Hinv_r, spd_r = orc.cholesky_inverse(Hr)
            assert spd_r and bits_equal(Hinv, Hinv_r), "H^-1 differs from the oracle"
    else:
        Hinv = np.zeros((1, 1), np.float32)  # one block: no error feedback, H⁻¹ unused
    # 3) the block loop fed the same G and H⁻¹
    ref = orc.quantize_blocks(host(Wd.float()), Gh, Hinv, bs, ssr, 1)
    np.testing.assert_array_equal(host(out.perm), ref["perm"])
    np.testing.assert_array_equal(host(out.T), ref["T"])
    assert bits_equal(host(out.alpha), ref["alpha"]) and bits_equal(host(out.mu), ref["mu"])
    np.testing.assert_array_equal(host(out.iters), ref["iters"])
    # 4) properties
    p = host(out.perm)
    assert np.array_equal(np.sort(p), np.arange(m))
    assert set(np.unique(host(out.T))) <= {-1, 0, 1}
    assert (host(out.iters) < 100).all()
    assert np.isfinite(host(out.alpha)).all() and np.isfinite(host(out.mu)).all()
    return out


def test_headline_bench_workload(pt2q):
    """The exact bench workload: fp16 4096 x 4096 (Llama-2-7B q_proj), N = 262144 rows, SSR,
    same synthetic generator and seeds as bench.py's single-layer extra; plus the hipGraph
    replay the bench times equals the eager launch bit-for-bit."""
    n = m = 4096
    N = 262144
    Wd = pt2q.fill_synthetic((n, m), 1000, std=0.02).half()
    Xd = pt2q.fill_synthetic((N, m), 2000 + m, std=1.0, outliers=True).half()
    out = check_layer_staged(pt2q, Wd, Xd)
    g = pt2q.LayerGraph(Wd, Xd)
    r = g.replay()
    torch.cuda.synchronize()
    assert g.spd()
    for a, b in ((r.T, out.T), (r.perm, out.perm), (r.alpha, out.alpha), (r.mu, out.mu)):
        assert bits_equal(host(a), host(b))


@pytest.mark.parametrize("m", [4096, 11008])
def test_gram16_full_length_vs_oracle_and_f64(pt2q, m):
    """the bench's own Gram launches at full length (fp16, N = 262144 rows; m =
    4096: gram16x_kernel, 128 x 256 tiles; m = 11008: gram16w_kernel, 256 x 256 tiles) on sampled
    column blocks: bit-exact to the oracle's 16-bit MFMA arithmetic, and at least as accurate
    as the fp32 k-ascending chain (the reference's fp32 arithmetic, main.py:128) against an f64
    Gram of the same columns -- error of each entry scaled by sqrt(G_ii G_jj)."""
    N = 262144
    Xd = pt2q.fill_synthetic((N, m), 2000 + m, std=1.0, outliers=True).half()
    G = pt2q.gram(Xd)
    torch.cuda.synchronize()
    S = sample_cols(m)
    Xs = host(Xd[:, torch.from_numpy(S).to(Xd.device)].contiguous())
    del Xd
    Gs = host(G)[np.ix_(S, S)]
    del G
    orc.set_threads(16)
    assert bits_equal(Gs, orc.gram16(Xs)), "sampled full-length Gram tiles differ from the oracle"
    X64 = Xs.astype(np.float64)
    G64 = X64.T @ X64
    scale = np.sqrt(np.outer(np.diag(G64), np.diag(G64)))
    err16 = np.abs(Gs - G64) / scale
    err32 = np.abs(orc.gram(Xs.astype(np.float32)) - G64) / scale
    assert err16.max() <= err32.max(), (float(err16.max()), float(err32.max()))
    assert err16.max() < 1e-4


CONFIGS = [
    # C2 GPT-2-small (Conv1D weights transposed to n x m), N = 2048, SSR on
    ("c2_attn_c_proj", 768, 768, 2048, torch.float32, 128),
    ("c2_c_fc", 3072, 768, 2048, torch.float32, 128),
    ("c2_c_attn", 2304, 768, 2048, torch.float32, 128),
    ("c2_mlp_c_proj", 768, 3072, 2048, torch.float32, 128),
    # C3 OPT-1.3B fp16
    ("c3_qkvo", 2048, 2048, 2048, torch.float16, 128),
    ("c3_fc1", 8192, 2048, 2048, torch.float16, 128),
    ("c3_fc2", 2048, 8192, 2048, torch.float16, 128),
    # C4 Llama-2-7B fp16 MLP
    ("c4_gate_up", 11008, 4096, 2048, torch.float16, 128),
    ("c4_down", 4096, 11008, 2048, torch.float16, 128),
    # C5 Llama-2-13B bf16 per-channel (block = m), 4096-sample Hessian
    ("c5_qkvo", 5120, 5120, 4096, torch.bfloat16, 5120),
    ("c5_gate_up", 13824, 5120, 4096, torch.bfloat16, 5120),
    ("c5_down", 5120, 13824, 4096, torch.bfloat16, 13824),
]


@pytest.mark.parametrize("name,n,m,N,dt,bs", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_config_layers(pt2q, name, n, m, N, dt, bs):
    seed = sum(map(ord, name))
    Wd = pt2q.fill_synthetic((n, m), seed, std=0.02).to(dt)
    Xd = pt2q.fill_synthetic((N, m), seed + 1, std=1.0, outliers=True).to(dt)
    out = check_layer_staged(pt2q, Wd, Xd, bs=bs)
    if bs >= m:
        np.testing.assert_array_equal(host(out.perm), np.arange(m))  # one block, in order


@pytest.mark.parametrize("name", golden_names("layer_m16_"))
def test_layer_16bit_vs_reference(pt2q, name):
    """16-bit W / X on the device (16-bit MFMA Gram) vs the reference's fp32-upcast run of the
    same values (codes / perm exact, scales within 1e-5) and vs the oracle (bit-exact)."""
    g = load_golden(name)
    W, X16 = layer_inputs16(g)
    dt = torch.float16 if str(g["dtype"]) == "fp16" else torch.bfloat16
    Wd = torch.from_numpy(W).to(DEV).to(dt)
    Xd = (torch.from_numpy(X16) if isinstance(X16, np.ndarray) else X16).to(DEV)
    bs = int(g["block_size"])
    out = pt2q.quantize_layer(Wd, Xd, block_size=bs, use_ssr=True)
    res = {"perm": host(out.perm), "T": host(out.T), "alpha": host(out.alpha), "mu": host(out.mu)}
    if name in NEAR_TIE_LAYERS:
        _check_layer_sets(g, res, bs)
    else:
        _check_layer(g, res)
    orc.set_threads(16)
    ref = orc.quantize_layer_m(W, X16, block_size=bs, use_ssr=True)
    np.testing.assert_array_equal(res["T"], ref["T"])
    assert bits_equal(res["alpha"], ref["alpha"]) and bits_equal(res["mu"], ref["mu"])


@pytest.mark.parametrize("name", golden_names("loop16_"))
def test_block_loop_16bit_vs_reference(pt2q, name):
    """Whole 16-bit layers on the device vs the reference's block loop run with the engine's
    H⁻¹ (gen_golden.gen_loop16): 24 / 16 blocks, codes and permutation bit-exact."""
    g = load_golden(name)
    W, X16 = layer_inputs16(g)
    Wd = torch.from_numpy(W).to(DEV).half()
    Xd = torch.from_numpy(X16).to(DEV)
    out = pt2q.quantize_layer(Wd, Xd, block_size=128, use_ssr=True)
    np.testing.assert_array_equal(host(out.perm), g["perm"])
    np.testing.assert_array_equal(host(out.T), unpack2(g["T2"], W.shape[1]))
    check_scales(host(out.alpha), g["alpha"], "alpha")
    check_scales(host(out.mu), g["mu"], "mu")


@pytest.mark.parametrize("n,m,dt,tdt", [(333, 5120, torch.bfloat16, torch.int8), (70, 5120, torch.bfloat16, torch.float32),
                                        (77, 4104, torch.float16, torch.int8), (50, 1000, torch.float32, torch.int8),
                                        (40, 13824, torch.bfloat16, torch.int8)])
def test_per_channel_row_kernels_edges(pt2q, n, m, dt, tdt):
    """The per-channel block loop (block_size = m) on both row kernels of atq_pc.hip -- 5120 bf16
    columns: rows held in registers; otherwise streamed through the LDS ring (ragged last chunk
    at m = 4104 / 1000, f16 / f32 W) -- with rows that are not a multiple of the workgroup's, an
    all-zero row, one-signed rows and int8 / fp32 codes: every output vs the oracle, bit-exact,
    and equal to the old streaming wide kernel (PT2Q_ATQ_PC=0 is read at load, so the oracle
    stands in for it here)."""
    Wd = pt2q.fill_synthetic((n, m), n + m, std=0.02)
    Wd[3] = 0.0
    Wd[5] = Wd[5].abs() + 0.01  # one-signed rows
    Wd[6] = -Wd[6].abs() - 0.01
    Wd = Wd.to(dt)
    Xd = pt2q.fill_synthetic((512, m), n + m + 1, std=1.0, outliers=True).to(dt)
    G = pt2q.gram(Xd)
    out = pt2q.engine.quantize_blocks(Wd, G, None, block_size=m, t_dtype=tdt)
    torch.cuda.synchronize()
    orc.set_threads(16)
    ref = orc.quantize_blocks(host(Wd.float()), host(G), np.zeros((1, 1), np.float32), m, True, 1)
    np.testing.assert_array_equal(host(out.perm), np.arange(m))
    np.testing.assert_array_equal(host(out.T.float()), ref["T"].astype(np.float32))
    assert bits_equal(host(out.alpha), ref["alpha"]) and bits_equal(host(out.mu), ref["mu"])
    np.testing.assert_array_equal(host(out.iters), ref["iters"])


@pytest.mark.parametrize("m,dt", [(5120, torch.bfloat16), (2048, torch.float16)])
def test_per_channel_zero_block(pt2q, m, dt):
    """All-zero per-channel block: ITF stops at iteration 0 (quantizer.py:164); the init grid
    (alpha = mu = 0, codes 0) is what every row returns, on both row kernels."""
    Wd = torch.zeros((37, m), device=DEV, dtype=dt)
    G = pt2q.gram(pt2q.fill_synthetic((256, m), 7, std=1.0).to(dt))
    out = pt2q.engine.quantize_blocks(Wd, G, None, block_size=m)
    torch.cuda.synchronize()
    assert int(host(out.iters)[0]) == 0
    assert not host(out.T).any() and not host(out.alpha).any() and not host(out.mu).any()


@pytest.mark.parametrize("m,batch", [(5120, 3), (1000, 2), (300, 2), (100, 3), (13824, 2), (4104, 5), (516, 1)])
def test_s1_batched_equals_per_item_and_given(pt2q, m, batch):
    """pt2q_s1_from_gram_batched (S1 = S·1, d = 1ᵀS1 of several Grams in one launch pair) ==
    pt2q_s1_from_gram per item, bit for bit; a per-channel block loop fed the formed S1 / d
    (PT2Q_FLAG_S1_GIVEN) == the same loop forming them itself (quantizer.py:215-218)."""
    Gs = torch.stack([pt2q.gram(pt2q.fill_synthetic((384, m), 31 + z, std=1.0, outliers=True).half())
                      for z in range(batch)]).contiguous()
    S1d = pt2q.engine.s1_from_gram_batched(Gs)
    for z in range(batch):
        S1 = torch.empty(m, device=DEV)
        d = torch.empty(1, device=DEV)
        rc = pt2q._lib.lib().pt2q_s1_from_gram(pt2q._lib.ptr(Gs[z]), m, m, pt2q._lib.ptr(S1), pt2q._lib.ptr(d),
                                               pt2q._lib.stream_of(Gs.device))
        assert rc == 0
        assert bits_equal(host(S1d[z, :m]), host(S1)) and bits_equal(host(S1d[z, m:]), host(d))
    if m > 512:
        Wd = pt2q.fill_synthetic((96, m), 77, std=0.02).to(torch.bfloat16)
        z = batch - 1
        a = pt2q.engine.quantize_blocks(Wd, Gs[z], None, block_size=m)
        b = pt2q.engine.quantize_blocks(Wd, Gs[z], None, block_size=m, s1d=S1d[z])
        for x, y in ((a.T, b.T), (a.alpha, b.alpha), (a.mu, b.mu), (a.iters, b.iters)):
            assert bits_equal(host(x.float()), host(y.float()))


@pytest.mark.parametrize("m,dt,ns,tdt", [
    (5120, torch.bfloat16, (333, 80, 600, 16), torch.int8),      # register rows, mixed row counts
    (5120, torch.bfloat16, (70, 45), torch.float32),             # fp32 codes
    (4104, torch.float16, (77, 130, 33), torch.int8),            # streamed rows, ragged last chunk
    (13824, torch.bfloat16, (40, 24), torch.int8),               # the C5 down projection's width
    (1000, torch.float32, (50, 17), torch.int8)])
def test_perchannel_group_equals_per_linear(pt2q, m, dt, ns, tdt):
    """pt2q_quantize_perchannel_group: every linear of the group (row counts differ, one of them
    all-zero so its launch takes the grouped repair, another with NO AGA) == quantize_blocks on
    that linear alone (block_size = m, the same S1 / d): codes, alpha, mu, perm, ITF count."""
    eng = pt2q.engine
    Ws, s1ds = [], []
    G = pt2q.gram(pt2q.fill_synthetic((384, m), m + 5, std=1.0, outliers=True).to(dt))
    S1d = eng.s1_from_gram_batched(G.unsqueeze(0).contiguous())[0]
    for z, n in enumerate(ns):
        W = pt2q.fill_synthetic((n, m), 1000 * z + n + m, std=0.02)
        if z == 1:
            W.zero_()  # every row's init codes zero: the whole-block repair (quantizer.py:164)
        Ws.append(W.to(dt))
        s1ds.append(None if z == len(ns) - 1 and len(ns) > 2 else S1d)
    outs = eng.quantize_perchannel_group(Ws, s1ds, t_dtype=tdt)
    torch.cuda.synchronize()
    for z, (W, s1, out) in enumerate(zip(Ws, s1ds, outs)):
        if s1 is None:
            ref = eng.quantize_blocks(W, None, None, block_size=m, aga=pt2q._lib.AGA_NONE, t_dtype=tdt)
        else:
            ref = eng.quantize_blocks(W, G, None, block_size=m, t_dtype=tdt, s1d=s1)
        for x, y in ((out.T, ref.T), (out.alpha, ref.alpha), (out.mu, ref.mu), (out.perm, ref.perm),
                     (out.iters, ref.iters)):
            assert bits_equal(host(x.float()), host(y.float())), z
    assert int(host(outs[1].iters)[0]) == 0 and not host(outs[1].T).any()


def test_perchannel_group_of_sixteen_vs_oracle(pt2q):
    """A full group (16 linears, the C5 q/k/v/o and gate/up row counts scaled down) vs the oracle,
    each with its own Gram's S1 / d, in one launch sequence."""
    eng = pt2q.engine
    m, dt = 5120, torch.bfloat16
    Gs = torch.stack([pt2q.gram(pt2q.fill_synthetic((256, m), 500 + z, std=1.0, outliers=True).to(dt))
                      for z in range(4)]).contiguous()
    S1d = eng.s1_from_gram_batched(Gs)
    Ws = [pt2q.fill_synthetic((48 + 16 * (z % 3), m), 900 + z, std=0.02).to(dt) for z in range(16)]
    outs = eng.quantize_perchannel_group(Ws, [S1d[z % 4] for z in range(16)])
    torch.cuda.synchronize()
    orc.set_threads(16)
    for z in (0, 5, 10, 15):
        ref = orc.quantize_blocks(host(Ws[z].float()), host(Gs[z % 4]), np.zeros((1, 1), np.float32), m, True, 1)
        np.testing.assert_array_equal(host(outs[z].T.float()), ref["T"].astype(np.float32))
        assert bits_equal(host(outs[z].alpha), ref["alpha"]) and bits_equal(host(outs[z].mu), ref["mu"])
        np.testing.assert_array_equal(host(outs[z].iters), ref["iters"])


@pytest.mark.parametrize("m,batch", [(5120, 2), (13824, 1), (1000, 2), (548, 1), (544, 1), (576, 3), (4104, 1)])
def test_s1_from_upper_equals_full(pt2q, m, batch):
    """pt2q_s1_from_upper_batched reads only the upper triangle (the lower one is NaN here) and
    gives S1 / d bit-identical to pt2q_s1_from_gram_batched on the full symmetric Gram: column
    tiles above the diagonal block, the two diagonal tiles (mixed), row tiles after it, ragged
    last blocks (548: a 36-row last block, 544: one diagonal tile)."""
    eng = pt2q.engine
    Gs = torch.stack([pt2q.gram(pt2q.fill_synthetic((384, m), 61 + z, std=1.0, outliers=True).half())
                      for z in range(batch)]).contiguous()
    want = eng.s1_from_gram_batched(Gs)
    low = torch.tril(torch.ones(m, m, dtype=torch.bool, device=DEV), diagonal=-1)
    Gu = Gs.masked_fill(low, float("nan"))
    got = eng.s1_from_gram_batched(Gu, upper_only=True)
    assert bits_equal(host(got), host(want))


@pytest.mark.parametrize("m,dt,N", [(5120, torch.bfloat16, 1024), (768, torch.float16, 1024),
                                    (13824, torch.bfloat16, 1000), (1024, torch.float16, 328)])
def test_gram_batched_upper(pt2q, m, dt, N):
    """pt2q_gram_batched_upper: the upper triangle (diagonal included) equals the full batched
    Gram's bit for bit, the strictly lower part is left untouched.  Off-diagonal tiles are formed
    transposed there (gram16.hip), so this also pins G[j][i] == G[i][j]; N = 1000 / 328 end in a
    ragged stage (N % 32 != 0), 328 rows are fewer than the chain's 2 x 5 ring stages."""
    eng = pt2q.engine
    Xs = [pt2q.fill_synthetic((N, m), 71 + z, std=1.0, outliers=True).to(dt) for z in range(3)]
    full = torch.empty((3, m, m), device=DEV)
    eng.gram_batched(Xs, full)
    up = torch.full((3, m, m), 7.0, device=DEV)
    eng.gram_batched(Xs, up, upper_only=True)
    upper = torch.triu(torch.ones(m, m, dtype=torch.bool, device=DEV))
    assert bits_equal(host(up[:, upper]), host(full[:, upper]))
    assert bool((up[:, ~upper] == 7.0).all())
