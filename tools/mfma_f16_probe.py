"""Generate inputs for / analyse outputs of tools/mfma_f16_probe (dev tool).
  python tools/mfma_f16_probe.py gen DIR ; <run probe DIR on the GPU> ; python tools/mfma_f16_probe.py ana DIR
Exact arithmetic in int64 fixed point (scale 2^SC); inputs are kept in a range where that is exact."""
import sys
import numpy as np

SC = 48
TILES = 384


def rnd_f32(v):
    """round-to-nearest-even of the exact value v * 2^-SC (int64 array) to f32 (as float64)."""
    v = np.asarray(v, dtype=np.int64)
    s = np.sign(v)
    a = np.abs(v).astype(np.uint64)
    out = np.zeros(v.shape, dtype=np.float64)
    nz = a > 0
    L = np.zeros(v.shape, dtype=np.int64)
    L[nz] = np.floor(np.log2(a[nz].astype(np.float64))).astype(np.int64) + 1
    # fix log2 rounding
    for _ in range(2):
        too_big = nz & (L < 64) & (a >= (np.uint64(1) << np.minimum(L, 63).astype(np.uint64)))
        L[too_big] += 1
        too_small = nz & (L > 1) & (a < (np.uint64(1) << (L - 1).astype(np.uint64)))
        L[too_small] -= 1
    sh = np.maximum(L - 24, 0).astype(np.uint64)
    q = a >> sh
    rem = a - (q << sh)
    half = np.where(sh > 0, np.uint64(1) << np.maximum(sh, np.uint64(1)) - np.uint64(1), np.uint64(0))
    up = (sh > 0) & ((rem > half) | ((rem == half) & ((q & np.uint64(1)) == 1)))
    q = q + up.astype(np.uint64)
    out = s * q.astype(np.float64) * np.exp2(sh.astype(np.float64) - SC)
    return out


def to_fix(x):
    y = np.asarray(x, dtype=np.float64) * 2.0 ** SC
    assert np.all(y == np.round(y)) and np.all(np.abs(y) < 2 ** 62)
    return y.astype(np.int64)


REGIMES = [  # (active k list, C mode)
    ([0, 1], 0), ([0, 1, 2, 3], 0), (list(range(8)), 0), ([0, 8], 0), ([0], 1), ([0, 1], 1),
    (list(range(4)), 1), (list(range(8)), 1), ([0, 8], 1), ([0, 4], 0), ([0, 2], 0), ([1, 2], 0),
]


def gen2(d):
    """Targeted regimes: only the listed k slots are non-zero; C = 0 (mode 0) or random (1)."""
    rng = np.random.default_rng(2)
    A = np.zeros((TILES, 32, 16), np.float16)
    B = np.zeros((TILES, 16, 32), np.float16)
    C = np.zeros((TILES, 32, 32), np.float32)
    for t in range(TILES):
        ks, cm = REGIMES[t % len(REGIMES)]
        for k in ks:
            A[t][:, k] = rng.standard_normal(32) * np.exp2(rng.integers(-4, 4, 32))
            B[t][k, :] = rng.standard_normal(32) * np.exp2(rng.integers(-4, 4, 32))
        if cm:
            C[t] = (rng.standard_normal((32, 32)) * np.exp2(rng.integers(-4, 4, (32, 32)))).astype(np.float32)
    C = (np.round(C.astype(np.float64) * 2.0 ** 40) / 2.0 ** 40).astype(np.float32)
    with open(f"{d}/probe_in.bin", "wb") as f:
        np.array([TILES], np.int32).tofile(f)
        A.tofile(f); B.tofile(f); C.tofile(f)
    np.savez(f"{d}/probe_inputs.npz", A=A, B=B, C=C)


def gen3(d):
    """Broad validation set: exponent extremes, fp16 subnormals, f32-subnormal accumulators,
    Gram-like chains (C = large running sum, products of activation pairs)."""
    rng = np.random.default_rng(3)
    A = np.zeros((TILES, 32, 16), np.float32)
    B = np.zeros((TILES, 16, 32), np.float32)
    C = np.zeros((TILES, 32, 32), np.float64)
    def spread(shape, lo, hi):
        return rng.standard_normal(shape) * np.exp2(rng.integers(lo, hi, shape))
    for t in range(TILES):
        reg = t % 8
        if reg == 0:   # full fp16 range incl. subnormals
            A[t] = spread((32, 16), -24, 15); B[t] = spread((16, 32), -24, 15)
            C[t] = spread((32, 32), -40, 40)
        elif reg == 1:  # subnormal-heavy activations
            A[t] = spread((32, 16), -24, -12); B[t] = spread((16, 32), -24, -8)
            C[t] = spread((32, 32), -50, -20) * (rng.random((32, 32)) < 0.7)
        elif reg == 2:  # f32-subnormal accumulators and results
            A[t] = spread((32, 16), -24, -18); B[t] = spread((16, 32), -24, -18)
            C[t] = spread((32, 32), -149, -120)
        elif reg == 3:  # Gram-like: C = big running sums, products of activations
            x = (rng.standard_normal((16, 32)) * np.where(rng.random(32) < 0.05, 20, 1)).astype(np.float16)
            A[t] = x.T.astype(np.float32)[:, :16] if False else x[:, :32].T[:, :16].astype(np.float32)
            B[t] = x.astype(np.float32)
            C[t] = np.abs(rng.standard_normal((32, 32))) * np.exp2(rng.integers(0, 22, (32, 32)))
        elif reg == 4:  # same as 3 with signed C (off-diagonal sums)
            x = rng.standard_normal((16, 32)).astype(np.float16)
            A[t] = x.T[:, :16].astype(np.float32); B[t] = x.astype(np.float32)
            C[t] = rng.standard_normal((32, 32)) * np.exp2(rng.integers(-4, 18, (32, 32)))
        elif reg == 5:  # large magnitudes
            A[t] = spread((32, 16), 5, 16); B[t] = spread((16, 32), 5, 16)
            C[t] = spread((32, 32), 20, 50)
        elif reg == 6:  # sparse products (zeros mixed in), random C
            A[t] = spread((32, 16), -6, 6) * (rng.random((32, 16)) < 0.4)
            B[t] = spread((16, 32), -6, 6) * (rng.random((16, 32)) < 0.4)
            C[t] = spread((32, 32), -10, 10)
        else:           # exact cancellation of C by the products
            A[t] = spread((32, 16), -3, 3); B[t] = spread((16, 32), -3, 3)
            a16 = A[t].astype(np.float16).astype(np.float64); b16 = B[t].astype(np.float16).astype(np.float64)
            C[t] = -(a16 @ b16) * (1 + rng.standard_normal((32, 32)) * 1e-6)
    A = np.clip(A, -65504, 65504).astype(np.float16)
    B = np.clip(B, -65504, 65504).astype(np.float16)
    C = C.astype(np.float32)
    with open(f"{d}/probe_in.bin", "wb") as f:
        np.array([TILES], np.int32).tofile(f)
        A.tofile(f); B.tofile(f); C.tofile(f)
    np.savez(f"{d}/probe_inputs.npz", A=A, B=B, C=C)


def gen_bf16(d):
    """bf16 operands: the s1/s3 value sets re-rounded to bf16, plus a wide-exponent regime."""
    import torch
    rng = np.random.default_rng(4)
    A = rng.standard_normal((TILES, 32, 16)) * np.exp2(rng.integers(-30, 30, (TILES, 32, 16)))
    B = rng.standard_normal((TILES, 16, 32)) * np.exp2(rng.integers(-30, 30, (TILES, 16, 32)))
    C = rng.standard_normal((TILES, 32, 32)) * np.exp2(rng.integers(-40, 40, (TILES, 32, 32)))
    for t in range(TILES):
        reg = t % 4
        if reg == 1:   # activations-like
            A[t] = rng.standard_normal((32, 16)); B[t] = rng.standard_normal((16, 32))
            C[t] = rng.standard_normal((32, 32)) * 30
        elif reg == 2:  # C dominant
            A[t] *= 2.0 ** -20; B[t] *= 2.0 ** -20
        elif reg == 3:  # Gram-like
            x = rng.standard_normal((16, 32)) * np.where(rng.random(32) < 0.05, 20, 1)
            A[t] = x.T[:, :16]; B[t] = x
            C[t] = np.abs(rng.standard_normal((32, 32))) * np.exp2(rng.integers(0, 22, (32, 32)))
    Ab = torch.from_numpy(A.astype(np.float32)).bfloat16()
    Bb = torch.from_numpy(B.astype(np.float32)).bfloat16()
    C = C.astype(np.float32)
    with open(f"{d}/probe_in.bin", "wb") as f:
        np.array([TILES], np.int32).tofile(f)
        Ab.view(torch.int16).numpy().tofile(f); Bb.view(torch.int16).numpy().tofile(f); C.tofile(f)
    np.savez(f"{d}/probe_inputs.npz", A=Ab.view(torch.int16).numpy().view(np.uint16),
             B=Bb.view(torch.int16).numpy().view(np.uint16), C=C)


def gen(d):
    rng = np.random.default_rng(1)
    A = np.zeros((TILES, 32, 16), np.float16)
    B = np.zeros((TILES, 16, 32), np.float16)
    C = np.zeros((TILES, 32, 32), np.float32)
    for t in range(TILES):
        reg = t % 6
        if reg == 0:   # plain random
            A[t] = rng.standard_normal((32, 16)); B[t] = rng.standard_normal((16, 32))
            C[t] = rng.standard_normal((32, 32)).astype(np.float32)
        elif reg == 1:  # wide exponent spread in the products
            A[t] = rng.standard_normal((32, 16)) * np.exp2(rng.integers(-9, 5, (32, 16)))
            B[t] = rng.standard_normal((16, 32)) * np.exp2(rng.integers(-9, 5, (16, 32)))
            C[t] = (rng.standard_normal((32, 32)) * np.exp2(rng.integers(-6, 6, (32, 32)))).astype(np.float32)
        elif reg == 2:  # C = 0
            A[t] = rng.standard_normal((32, 16)); B[t] = rng.standard_normal((16, 32))
        elif reg == 3:  # C large, small products (alignment / sticky)
            A[t] = rng.standard_normal((32, 16)) * 2.0 ** -6; B[t] = rng.standard_normal((16, 32)) * 2.0 ** -6
            C[t] = (rng.standard_normal((32, 32)) * 64).astype(np.float32)
        elif reg == 4:  # cancellation: products of opposite signs, near-equal magnitudes
            a = rng.standard_normal((32, 16)); A[t] = a
            b = rng.standard_normal((16, 32)); b[1::2] = -b[0::2]; B[t] = b
            C[t] = (rng.standard_normal((32, 32)) * 1e-3).astype(np.float32)
        else:           # sums of many tiny products onto 1.0 (pure tie / sticky cases)
            A[t] = np.float16(2.0 ** -12) * rng.integers(1, 4, (32, 16)); B[t] = np.float16(2.0 ** -12)
            C[t] = 1.0 + rng.integers(0, 4, (32, 32)) * 2.0 ** -23
    # keep values exactly representable in fixed point
    C = np.where(np.abs(C) < 2.0 ** -16, 0, C).astype(np.float32)
    C = (np.round(C.astype(np.float64) * 2.0 ** SC) / 2.0 ** SC).astype(np.float32)
    with open(f"{d}/probe_in.bin", "wb") as f:
        np.array([TILES], np.int32).tofile(f)
        A.tofile(f); B.tofile(f); C.tofile(f)
    np.savez(f"{d}/probe_inputs.npz", A=A, B=B, C=C)


def ana(d):
    z = np.load(f"{d}/probe_inputs.npz")
    A, B, C = z["A"].astype(np.float64), z["B"].astype(np.float64), z["C"].astype(np.float64)
    D = np.fromfile(f"{d}/probe_out.bin", np.float32).reshape(TILES, 32, 32).astype(np.float64)
    P = A[:, :, :, None] * B[:, None, :, :]          # (t, i, k, j) exact in f64
    P = np.moveaxis(P, 2, 3)                          # (t, i, j, k)
    Pf = to_fix(P)
    Cf = to_fix(C)
    models = {}
    models["fused16"] = rnd_f32(Cf + Pf.sum(-1))
    models["dot_then_add"] = rnd_f32(Cf + to_fix(rnd_f32(Pf.sum(-1))))
    for g in (1, 2, 4, 8):
        acc = Cf.copy()
        for k0 in range(0, 16, g):
            acc = to_fix(rnd_f32(acc + Pf[..., k0:k0 + g].sum(-1)))
        models[f"chain_g{g}"] = acc.astype(np.float64) / 2.0 ** SC
        acc = Cf.copy()
        for k0 in reversed(range(0, 16, g)):
            acc = to_fix(rnd_f32(acc + Pf[..., k0:k0 + g].sum(-1)))
        models[f"chain_g{g}_rev"] = acc.astype(np.float64) / 2.0 ** SC
    # group of 8 rounded as a dot, then added
    acc = Cf.copy()
    for k0 in (0, 8):
        acc = to_fix(rnd_f32(acc + to_fix(rnd_f32(Pf[..., k0:k0 + 8].sum(-1)))))
    models["g8dot_then_add"] = acc.astype(np.float64) / 2.0 ** SC
    nreg = len(REGIMES) if len(sys.argv) > 3 else 6
    for reg in range(nreg):
        sel = np.arange(TILES) % nreg == reg
        line = [f"reg{reg}"]
        for name, M in models.items():
            line.append(f"{name}={np.mean(M[sel] == D[sel]):.4f}")
        print(" ".join(line))
    print("ALL", {k: round(float(np.mean(v == D)), 5) for k, v in models.items()})


if __name__ == "__main__":
    {"gen": gen, "gen2": gen2, "gen3": gen3, "genbf": gen_bf16, "ana": ana}[sys.argv[1]](sys.argv[2])
