"""Calibration capture + shared Grams (reference main.py:232-308).

The streamed Gram must equal the Gram of the concatenated rows bit-for-bit (oracle), shared
quantisation must equal per-linear quantize_layer, and the model-level loop must reproduce the
reference's capture-concatenate-quantise-writeback loop exactly (emulated here with the same
hooks the reference registers, main.py:262-275, and per-linear quantize_layer)."""
import numpy as np
import pytest
import torch

import synth
from test_gpu_parity import bits_equal, cuda, host, oracle_gram
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("splits,m,dt", [((100, 37, 200), 96, torch.float32),
                                         ((1000, 3000, 16384), 2048, torch.float16),
                                         ((64, 192, 2048), 256, torch.bfloat16),
                                         # ragged 16-bit batches: the accumulator carries the
                                         # (< 8) remainder rows into the next batch's first group
                                         ((13, 100, 7, 1, 333, 5), 256, torch.float16),
                                         ((3, 2, 1, 1, 701), 200, torch.bfloat16),
                                         ((5, 64, 3), 96, torch.float32)])
@pytest.mark.parametrize("buffer_rows", [32768, 0, 104])
def test_gram_continue_equals_concatenated(pt2q, splits, m, dt, buffer_rows):
    """The streamed Gram == the Gram of the concatenated rows, bit for bit: staged through the
    default buffer, per batch (buffer_rows=0: remainder rows carried), and through a 104-row buffer
    that fills and flushes mid-batch many times (chains continued at multiples of 8 rows)."""
    X = synth.activations(21 + m, sum(splits), m)
    Xd = cuda(X).to(dt)
    acc = pt2q.GramAccumulator(m, "cuda", buffer_rows=buffer_rows)
    s = 0
    for k in splits:
        acc.add(Xd[s:s + k])
        s += k
    assert acc.nsamples == X.shape[0]
    assert bits_equal(host(acc.G), oracle_gram(Xd))


def test_quantize_shared_equals_per_linear(pt2q):
    n1, n2, m, N = 384, 256, 320, 600
    X = cuda(synth.activations(31, N, m))
    Ws = [cuda(synth.weights(32, n1, m)), cuda(synth.weights(33, n2, m))]
    G = pt2q.gram(X)
    outs = pt2q.quantize_shared(Ws, G, N, 128, True)
    for W, o in zip(Ws, outs):
        r = pt2q.quantize_layer(W, X, 128, True)
        for a, b in ((o.alpha, r.alpha), (o.mu, r.mu), (o.T, r.T), (o.perm, r.perm)):
            assert bits_equal(host(a), host(b))


def _tiny_llama():
    transformers = pytest.importorskip("transformers")
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=384,
                                   num_hidden_layers=2, num_attention_heads=4,
                                   num_key_value_heads=4, max_position_embeddings=256)
    torch.manual_seed(0)
    return transformers.LlamaForCausalLM(cfg).cuda().eval()


def test_model_loop_matches_reference_loop(pt2q):
    """PT2LLMQuantizer.quantize (Gram capture, shared Hessians) vs the reference's loop shape:
    capture every input, torch.cat, quantize_layer per linear, _dequantize_weight write-back."""
    torch.manual_seed(1)
    samples = [torch.randint(0, 512, (1, 64)) for _ in range(3)]

    model_a = _tiny_llama()
    q = pt2q.PT2LLMQuantizer(model_a, None, "llama", block_size=128, use_ssr=True)
    got = q.quantize(samples)

    model_b = _tiny_llama()
    want = {}
    with torch.no_grad():
        for idx, layer in enumerate(model_b.model.layers):
            acts, hooks = {}, []
            lins = pt2q.find_linear_layers(layer)
            for name, lin in lins.items():
                hooks.append(lin.register_forward_hook(
                    lambda mod, inp, out, name=name: acts.setdefault(name, []).append(inp[0].detach())))
            for s in samples:
                model_b(s.cuda())
            for h in hooks:
                h.remove()
            for name, lin in lins.items():
                X = torch.cat(acts[name], dim=0)
                out = pt2q.quantize_layer(lin.weight.data, X, 128, True)
                p = {"alpha": out.alpha, "mu": out.mu, "T": out.T, "perm": out.perm}
                want[f"layer_{idx}.{name}"] = p
                lin.weight.data = pt2q.calibration.dequantize_weight_reference(p, 128).to(lin.weight.dtype)
    assert set(got) == set(want) and len(got) == 14
    for k in want:
        for f in ("alpha", "mu", "T", "perm"):
            assert bits_equal(host(got[k][f]), host(want[k][f])), (k, f)
    # the model was written back identically
    for pa, pb in zip(model_a.parameters(), model_b.parameters()):
        assert torch.equal(pa, pb)


@pytest.mark.parametrize("lanes", [2, 3])
def test_unit_pipeline_equals_sequential(pt2q, lanes):
    """engine.UnitPipeline (unit i+1's Gram on a low-priority stream while unit i's tail runs)
    must give exactly the results of quantize_unit one unit after another: mixed input widths,
    shared-input units with several linears, fp16 and fp32 activations, and more units per width
    than Gram slots so every slot is rewritten while later units are in flight."""
    units = []
    for i, (m, ns, N, dt) in enumerate([(512, (384, 256), 1024, torch.float16),
                                        (768, (512,), 2048, torch.float16),
                                        (512, (640,), 1024, torch.float32),
                                        (512, (256, 256, 128), 1536, torch.float16),
                                        (768, (256,), 2048, torch.float16),
                                        (512, (384,), 1024, torch.float16)]):
        X = cuda(synth.activations(600 + i, N, m)).to(dt)
        Ws = [cuda(synth.weights(700 + 10 * i + k, n, m)).to(dt) for k, n in enumerate(ns)]
        units.append((Ws, X))
    pipe = pt2q.UnitPipeline("cuda", 128, True, lanes=lanes)
    runs = [pipe.run(Ws, X) for Ws, X in units]
    got = [r.finish() for r in runs]
    for (Ws, X), outs in zip(units, got):
        want = pt2q.quantize_unit(Ws, X, block_size=128, use_ssr=True)
        assert len(outs) == len(want)
        for o, r in zip(outs, want):
            for a, b in ((o.alpha, r.alpha), (o.mu, r.mu), (o.T, r.T), (o.perm, r.perm), (o.iters, r.iters)):
                assert bits_equal(host(a), host(b))


@pytest.mark.parametrize("batched,chunk,group,inv_streams", [(False, 32, 1, 1), (True, 32, 1, 1), (True, 1, 1, 1),
                                                             (True, 32, 16, 1), (True, 2, 2, 1), (True, 1, 16, 3)])
def test_grams_first_schedule_equals_sequential(pt2q, batched, chunk, group, inv_streams):
    """sharding.GramsFirst (every Gram of the step first into packed per-width slots, then --
    batched -- every width's Hessian inverses in batched launches, then the block loops on the
    pipeline lanes, per unit or -- group > 1 -- grouped across units by shape) through
    quantize_units_sharded == quantize_unit per unit; inv_streams > 1 spreads the inverse chunks
    over streams with scratch of their own."""
    import importlib
    sharding = importlib.import_module("pt2q.sharding")
    specs = [(512, (384, 256), 1024, torch.float16), (768, (512,), 2048, torch.float16),
             (512, (640,), 1024, torch.float32), (768, (256,), 1536, torch.float16)]
    units, data = [], {}
    for i, (m, ns, N, dt) in enumerate(specs):
        X = cuda(synth.activations(800 + i, N, m)).to(dt)
        Ws = {f"p{k}": cuda(synth.weights(900 + 10 * i + k, n, m)).to(dt) for k, n in enumerate(ns)}
        units.append((f"u{i}", [(f"p{k}", n, m) for k, n in enumerate(ns)], N))
        data[f"u{i}"] = (X, Ws)
    pipe = pt2q.UnitPipeline("cuda", 128, True, lanes=3)
    gf = sharding.GramsFirst(pipe, "cuda", batched=batched, chunk=chunk, group=group, inv_streams=inv_streams)
    res, mine = sharding.quantize_units_sharded(units, lambda u: data[u[0]], pack=False,
                                                grams_first=gf)
    res2, _ = sharding.quantize_units_sharded(units, lambda u: data[u[0]], pack=False,
                                              grams_first=gf)  # second step reuses the slots
    for k in res:
        for f in res[k]:
            assert bits_equal(host(res[k][f]), host(res2[k][f])), (k, f)
    assert mine == list(range(len(units))) or sorted(mine) == list(range(len(units)))
    for name, lins, _ in units:
        X, Ws = data[name]
        want = pt2q.quantize_unit([Ws[p] for p, _, _ in lins], X, block_size=128, use_ssr=True)
        for (p, _, _), r in zip(lins, want):
            o = res[f"{name}.{p}"]
            for k, b in (("alpha", r.alpha), ("mu", r.mu), ("T", r.T), ("perm", r.perm)):
                assert bits_equal(host(o[k]), host(b)), (name, p, k)


def _units_and_data(pt2q, specs, seed):
    units, data = [], {}
    for i, (m, ns, N, dt) in enumerate(specs):
        X = cuda(synth.activations(seed + i, N, m)).to(dt)
        Ws = {f"p{k}": cuda(synth.weights(seed + 100 + 10 * i + k, n, m)).to(dt) for k, n in enumerate(ns)}
        units.append((f"u{i}", [(f"p{k}", n, m) for k, n in enumerate(ns)], N))
        data[f"u{i}"] = (X, Ws)
    return units, data


@pytest.mark.parametrize("bs,batched", [(1024, True), (1 << 14, True), (1 << 14, False)])
def test_grams_first_per_channel_equals_quantize_layer(pt2q, bs, batched):
    """the per-channel (block >= m, C5) grams-first step runs no Hessian inverse
    -- H^-1 feeds only the error feedback (main.py:198-214), which one block never reaches -- and
    its results equal pt2q_quantize_layer (which skips the inverse the same way) bit for bit:
    bf16 640 x 1024 linears, a shared-input unit of two, batched Grams, the per-linear block
    loops issued on the lanes with their status read once at finish."""
    import importlib
    sharding = importlib.import_module("pt2q.sharding")
    specs = [(1024, (640, 512), 4096, torch.bfloat16), (1024, (640,), 4096, torch.bfloat16)]
    units, data = _units_and_data(pt2q, specs, 1200)
    pipe = pt2q.UnitPipeline("cuda", bs, True, lanes=3)
    gf = sharding.GramsFirst(pipe, "cuda", batched=batched)
    res, _ = sharding.quantize_units_sharded(units, lambda u: data[u[0]], pack=False, grams_first=gf)
    assert gf.groups and all(grp["Hinv"] is None for grp in gf.groups.values())  # no inverse buffer
    assert not gf.inv_done and not gf.scratch  # ... and no batched factorisation ran
    for name, lins, _ in units:
        X, Ws = data[name]
        for p, _, _ in lins:
            r = pt2q.quantize_layer(Ws[p], X, bs, True)
            o = res[f"{name}.{p}"]
            for k, b in (("alpha", r.alpha), ("mu", r.mu), ("T", r.T), ("perm", r.perm)):
                assert bits_equal(host(o[k]), host(b)), (name, p, k)
    Ws = [data["u0"][1]["p0"], data["u0"][1]["p1"]]
    shared = pt2q.quantize_shared(Ws, pt2q.gram(data["u0"][0]), 4096, bs, True)
    for W, o in zip(Ws, shared):
        r = pt2q.quantize_layer(W, data["u0"][0], bs, True)
        assert o.spd and bits_equal(host(o.T), host(r.T)) and bits_equal(host(o.alpha), host(r.alpha))


@pytest.mark.parametrize("group", [1, 16])
def test_grams_first_pinv_fallback(pt2q, group):
    """a unit whose Hessian is not positive definite (its Gram negated after the Gram
    phase) takes the reference's pinv fallback (main.py:140-141) through GramsFirst.tails /
    _GroupedRun.finish (group > 1) or the lanes (group 1), with the SAME damping as every other
    path, and equals quantize_unit on that Gram; the SPD units beside it are untouched."""
    import importlib
    sharding = importlib.import_module("pt2q.sharding")
    specs = [(512, (384, 256), 1024, torch.float16), (512, (256,), 1024, torch.float16)]
    units, data = _units_and_data(pt2q, specs, 1300)
    pipe = pt2q.UnitPipeline("cuda", 128, True, percdamp=0.02, lanes=2)
    gf = sharding.GramsFirst(pipe, "cuda", batched=True, group=group)
    assert gf.percdamp == 0.02
    gf.begin([(i, u[1][0][2], u[2]) for i, u in enumerate(units)])
    for i, u in enumerate(units):
        gf.gram(i, data[u[0]][0])
    gf.flush()
    g, z = gf.slot[0]
    gf.groups[g]["G"][z].neg_()
    Gneg = gf.groups[g]["G"][z].clone()
    gf.inverses()
    jobs = [(i, [data[u[0]][1][p] for p, _, _ in u[1]], u[2]) for i, u in enumerate(units)]
    runs = gf.tails(jobs) if gf.grouped else [gf.tail(i, Ws, N) for i, Ws, N in jobs]
    outs = [r.finish() for r in runs]
    gf.check()
    assert [o.spd for o in outs[0]] == [False, False] and outs[1][0].spd
    want0 = pt2q.quantize_unit(jobs[0][1], G=Gneg, nsamples=1024, percdamp=0.02)
    want1 = pt2q.quantize_unit(jobs[1][1], X=data["u1"][0], percdamp=0.02)
    for got, want in ((outs[0], want0), (outs[1], want1)):
        for o, r in zip(got, want):
            for a, b in ((o.alpha, r.alpha), (o.mu, r.mu), (o.T, r.T), (o.perm, r.perm)):
                assert bits_equal(host(a), host(b))
