"""Analyse tools/probe_mfma_f16.hip output: which accumulation semantics does the f16/bf16 MFMA
implement?  H1 = sequential fp32 fma chain; H2 = exact sum of the 16 products + C, one RN
rounding per instruction; H3 = exact products, pairwise fp32 tree, then + C."""
import numpy as np
from fractions import Fraction

K = 128
raw = open("gpurun_out/mfma_f16_inputs.bin", "rb").read()
o = 0
A = np.frombuffer(raw, np.float16, 32 * K, o).astype(np.float64).reshape(32, K); o += 2 * 32 * K
B = np.frombuffer(raw, np.float16, K * 32, o).astype(np.float64).reshape(K, 32); o += 2 * K * 32
Ab = (np.frombuffer(raw, np.uint16, 32 * K, o).astype(np.uint32) << 16).view(np.float32).astype(np.float64).reshape(32, K); o += 2 * 32 * K
Bb = (np.frombuffer(raw, np.uint16, K * 32, o).astype(np.uint32) << 16).view(np.float32).astype(np.float64).reshape(K, 32); o += 2 * K * 32
C = np.frombuffer(raw, np.float32, 1024, o).reshape(32, 32)
res = np.fromfile("gpurun_out/mfma_f16_probe.bin", np.float32).reshape(4, 32, 32)


def rn32(fr):
    # correct rounding of a Fraction to fp32 via exact comparison
    f = np.float32(float(fr))  # float() is correctly rounded to double; double->float may double-round
    # fix double rounding: check neighbours
    best = f
    for cand in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        if abs(Fraction(float(cand)) - fr) < abs(Fraction(float(best)) - fr) or (
                abs(Fraction(float(cand)) - fr) == abs(Fraction(float(best)) - fr) and (cand.view(np.uint32) & 1) == 0):
            best = cand
    return best


def check(Am, Bm, D, kk, name):
    n_h1 = n_h2 = n_h3 = 0
    for i in range(32):
        for j in range(32):
            acc1 = np.float32(C[i, j]); acc2 = np.float32(C[i, j]); acc3 = np.float32(C[i, j])
            for g in range(0, kk, 16):
                prods = [Fraction(Am[i, k]) * Fraction(Bm[k, j]) for k in range(g, g + 16)]
                for p in prods:
                    acc1 = rn32(Fraction(float(acc1)) + p)
                acc2 = rn32(Fraction(float(acc2)) + sum(prods))
                t = [rn32(p) for p in prods]
                while len(t) > 1:
                    t = [rn32(Fraction(float(t[q])) + Fraction(float(t[q + 1]))) for q in range(0, len(t), 2)]
                acc3 = rn32(Fraction(float(acc3)) + Fraction(float(t[0])))
            d = D[i, j]
            n_h1 += acc1 == d; n_h2 += acc2 == d; n_h3 += acc3 == d
    print(f"{name} K={kk}: matches H1 chain {n_h1}/1024, H2 exact-sum-1-rounding {n_h2}/1024, H3 tree {n_h3}/1024")


check(A, B, res[0], 16, "f16")
check(Ab, Bb, res[1], 16, "bf16")
check(A, B, res[2], 128, "f16")
check(Ab, Bb, res[3], 128, "bf16")


def err(Am, Bm, D, kk, name):
    ex = C.astype(np.float64) + Am[:, :kk] @ Bm[:kk, :]
    rel = np.abs(D - ex) / np.maximum(np.abs(ex), 1e-30)
    ulp = np.abs(D - ex) / np.spacing(np.abs(ex).astype(np.float32)).astype(np.float64)
    print(f"{name} K={kk}: max rel err {rel.max():.3e}, median |err| in ulps {np.median(ulp):.2f}, max {ulp.max():.1f}")


err(A, B, res[0], 16, "f16")
err(Ab, Bb, res[1], 16, "bf16")
err(A, B, res[2], 128, "f16")
