"""PT2Q CPU oracle — Python (ctypes + numpy) wrapper around oracle/pt2q_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  Every function restates one step of the
reference (file:line cited per function) under the PT2Q arithmetic contract.
Parity of this restatement with the reference itself is pinned by tests/golden/*.npz
(generated from /root/reference by tests/golden/gen_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libpt2q_oracle.so")
_lib = None

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
L = ctypes.c_long
I = ctypes.c_int
F = ctypes.c_float


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        h = ctypes.CDLL(_SO)
        sig = {
            "orc_ternary_init": (None, [f32p, L, I, I, f32p, f32p, f32p, L]),
            "orc_build_optimal_grid": (None, [f32p, L, f32p, L, I, I, f32p, f32p]),
            "orc_flexible_round": (None, [f32p, L, f32p, f32p, I, I, f32p, L]),
            "orc_itf": (I, [f32p, L, I, I, I, f32p, f32p, f32p, L]),
            "orc_aga": (None, [f32p, L, f32p, L, I, I, f32p, F, f32p, f32p]),
            "orc_s1_from_x": (None, [f32p, L, L, I, f32p, f32p]),
            "orc_atq_quantize": (I, [f32p, L, I, I, I, f32p, F, I, f32p, f32p, f32p, L]),
            "orc_ssr_similarity": (None, [f32p, L, I, i64p, I, f32p]),
            "orc_ssr_select": (I, [f32p, L, I, i64p, I, I, i64p, i64p, f32p]),
            "orc_gram": (None, [f32p, L, L, I, f32p, L]),
            "orc_gram_accumulate": (None, [f32p, L, L, I, f32p, L]),
            "orc_gram16": (None, [u16p, L, L, I, f32p, L, I, I]),
            "orc_mfma16_tiles": (None, [I, u16p, u16p, f32p, f32p, I]),
            "orc_prepare_hessian": (F, [f32p, L, I, L, F, f32p, L]),
            "orc_cholesky_upper": (I, [f32p, L, I, f32p, L]),
            "orc_trtri_upper": (None, [f32p, L, I, f32p, L]),
            "orc_lauum_upper": (None, [f32p, L, I, f32p, L]),
            "orc_cholesky_inverse": (I, [f32p, L, I, f32p, L]),
            "orc_quantize_blocks": (I, [f32p, L, I, I, I, I, I, f32p, L, f32p, L, I,
                                        f32p, f32p, i8p, i64p, i32p]),
            "orc_error_feedback": (None, [f32p, L, I, i64p, I, i64p, I, f32p, f32p, L]),
            "orc_matvec16": (None, [f32p, L, I, I, f32p, f32p]),
            "orc_rowsum_seq": (None, [f32p, L, I, I, f32p]),
            "orc_set_threads": (None, [I]),
            "orc_get_threads": (I, []),
            "orc_fp_rule_mismatches": (L, [I, L, ctypes.c_uint64]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def set_threads(t):
    lib().orc_set_threads(int(t))


def get_threads():
    return int(lib().orc_get_threads())


# ------------------------------------------------------------------ ATQ (quantizer.py)

def fp_rule_mismatches(rule, count, seed=1):
    """Mismatches of a GPU arithmetic shortcut against the oracle's own operation (C, fmaf):
    rule 0 = the division-free ITF round (atq.hip round_code), rule 1 = the reciprocal-corrected
    division of the SSR similarity (ssr.hip div_rcp)."""
    return int(lib().orc_fp_rule_mismatches(rule, count, seed))


def ternary_init(W):
    """quantizer.py:32-69. Returns alpha (n,1), mu (n,1), T (n,b) float32."""
    W = _f32(W)
    n, b = W.shape
    a = np.empty(n, np.float32); m = np.empty(n, np.float32); T = np.empty((n, b), np.float32)
    lib().orc_ternary_init(W, b, n, b, a, m, T, b)
    return a[:, None], m[:, None], T


def build_optimal_grid(W, T):
    """quantizer.py:71-108."""
    W = _f32(W); T = _f32(T)
    n, b = W.shape
    a = np.empty(n, np.float32); m = np.empty(n, np.float32)
    lib().orc_build_optimal_grid(W, b, T, b, n, b, a, m)
    return a[:, None], m[:, None]


def flexible_round(W, alpha, mu):
    """quantizer.py:110-134."""
    W = _f32(W)
    n, b = W.shape
    T = np.empty((n, b), np.float32)
    lib().orc_flexible_round(W, b, _f32(np.reshape(alpha, -1)), _f32(np.reshape(mu, -1)), n, b, T, b)
    return T


def iterative_ternary_fitting(W, alpha, mu, T, max_iter=100):
    """quantizer.py:136-175 (whole-block torch.equal stop). Returns alpha, mu, T, iters."""
    W = _f32(W)
    n, b = W.shape
    a = _f32(np.reshape(alpha, -1)).copy(); m = _f32(np.reshape(mu, -1)).copy(); T = _f32(T).copy()
    it = lib().orc_itf(W, b, n, b, int(max_iter), a, m, T, b)
    return a[:, None], m[:, None], T, int(it)


def matvec16(A, x):
    """y[i] = DOT16(A[i], x): the contract order of the ATQ row products (fixture generator)."""
    A = _f32(A)
    y = np.empty(A.shape[0], np.float32)
    lib().orc_matvec16(A, A.shape[1], A.shape[0], A.shape[1], _f32(x).reshape(-1), y)
    return y


def rowsum_seq(A):
    """y[i] = l-ascending sum of A[i] (S1 = S·1 in the contract order; fixture generator)."""
    A = _f32(A)
    y = np.empty(A.shape[0], np.float32)
    lib().orc_rowsum_seq(A, A.shape[1], A.shape[0], A.shape[1], y)
    return y


def s1_from_x(X):
    """S = XᵀX (quantizer.py:207), S1 = S·1 (:216), d = 1ᵀS1 (:218)."""
    X = _f32(X)
    if X.ndim == 3:
        X = X.reshape(-1, X.shape[-1])
    N, b = X.shape
    S1 = np.empty(b, np.float32); d = np.empty(1, np.float32)
    lib().orc_s1_from_x(X, b, N, b, S1, d)
    return S1, float(d[0])


def activation_aware_grid_alignment(W, T, X=None, S1=None, d=None):
    """quantizer.py:177-248 (either X, or precomputed S1/d)."""
    W = _f32(W); T = _f32(T)
    n, b = W.shape
    if S1 is None:
        S1, d = s1_from_x(X)
    a = np.empty(n, np.float32); m = np.empty(n, np.float32)
    lib().orc_aga(W, b, T, b, n, b, _f32(S1), float(d), a, m)
    return a[:, None], m[:, None]


def atq_quantize(W, X=None, max_iter=100):
    """quantizer.py:250-277. Returns alpha, mu, T, itf_iters."""
    W = _f32(W)
    n, b = W.shape
    if X is not None:
        S1, d = s1_from_x(X)
        aga = 1
    else:
        S1, d, aga = np.zeros(b, np.float32), 0.0, 0
    a = np.empty(n, np.float32); m = np.empty(n, np.float32); T = np.empty((n, b), np.float32)
    it = lib().orc_atq_quantize(W, b, n, b, aga, S1, float(d), int(max_iter), a, m, T, b)
    return a[:, None], m[:, None], T, int(it)


def dequantize(alpha, mu, T):
    """quantizer.py:279-293: alpha*T + mu (two roundings)."""
    return (np.float32(1) * alpha * T + mu).astype(np.float32)


# ------------------------------------------------------------------ SSR (reorder.py)

def ssr_similarity(W, remaining):
    """reorder.py:36-61 on W (n x m)."""
    Wt = _f32(np.asarray(W, np.float32).T)
    n = Wt.shape[1]
    rem = np.ascontiguousarray(remaining, dtype=np.int64)
    sim = np.empty(len(rem), np.float32)
    lib().orc_ssr_similarity(Wt, n, n, rem, len(rem), sim)
    return sim


def select_next_block_ssr(W, remaining, block_size):
    """reorder.py:107-143. Returns (block_indices, new_remaining) int64."""
    Wt = _f32(np.asarray(W, np.float32).T)
    n = Wt.shape[1]
    rem = np.ascontiguousarray(remaining, dtype=np.int64)
    r = len(rem)
    blk = np.empty(max(r, 1), np.int64); newrem = np.empty(max(r, 1), np.int64)
    sim = np.empty(max(r, 1), np.float32)
    bs = lib().orc_ssr_select(Wt, n, n, rem, r, int(block_size), blk, newrem, sim)
    return blk[:bs].copy(), newrem[: r - bs].copy()


# ------------------------------------------------------------------ Hessian / inverse

def gram(X):
    """XᵀX (main.py:128; gptq.py:75) as k-ascending fmaf chains."""
    X = _f32(X)
    if X.ndim == 3:
        X = X.reshape(-1, X.shape[-1])
    N, m = X.shape
    G = np.empty((m, m), np.float32)
    lib().orc_gram(X, m, N, m, G, m)
    return G


def _bits16(X):
    """(uint16 bits, is_bf16) of an fp16 array, or of bf16 data given as a torch tensor or as
    uint16 bits tagged by the caller."""
    if hasattr(X, "dtype") and str(X.dtype) == "torch.bfloat16":
        import torch
        return np.ascontiguousarray(X.contiguous().view(torch.int16).numpy().view(np.uint16)), True
    return np.ascontiguousarray(np.asarray(X, dtype=np.float16)).view(np.uint16), False


def gram16(X, G=None, bf16_bits=False):
    """XᵀX of 16-bit X (numpy fp16, torch bf16, or raw bf16 bits with bf16_bits=True) under the
    gfx950 16-bit MFMA arithmetic (pt2q_oracle.c orc_gram16); with G given, continues G's chains
    by this batch (pt2q_gram accumulate=2).  main.py:128."""
    if bf16_bits:
        Xb, bf = np.ascontiguousarray(X, np.uint16), True
    else:
        Xb, bf = _bits16(X)
    if Xb.ndim == 3:
        Xb = Xb.reshape(-1, Xb.shape[-1])
    N, m = Xb.shape
    cont = G is not None
    G = np.zeros((m, m), np.float32) if G is None else np.ascontiguousarray(G, np.float32).copy()
    lib().orc_gram16(np.ascontiguousarray(Xb), m, N, m, G, m, int(cont), int(bf))
    return G


def mfma16_tiles(A, B, C, bf16=False):
    """The oracle's model of one v_mfma_f32_32x32x16_{f16,bf16} per tile: A (t,32,16) and
    B (t,16,32) as uint16 bits, C (t,32,32) f32."""
    A = np.ascontiguousarray(A).view(np.uint16); B = np.ascontiguousarray(B).view(np.uint16)
    C = _f32(C)
    D = np.empty_like(C)
    lib().orc_mfma16_tiles(A.shape[0], A, B, C, D, int(bf16))
    return D


def gram_accumulate(H, X):
    """GPTQ.add_batch gptq.py:59-76: H += XᵀX (in place)."""
    X = _f32(X)
    if X.ndim == 3:
        X = X.reshape(-1, X.shape[-1])
    N, m = X.shape
    assert H.dtype == np.float32 and H.flags.c_contiguous
    lib().orc_gram_accumulate(X, m, N, m, H, m)
    return H


def prepare_hessian(G, nsamples, percdamp=0.01):
    """main.py:129-133 / gptq.py:94-98. Returns (H_damped, damp)."""
    G = _f32(G)
    m = G.shape[0]
    H = np.empty_like(G)
    damp = lib().orc_prepare_hessian(G, m, m, int(nsamples), float(percdamp), H, m)
    return H, float(damp)


def cholesky_upper(H):
    H = _f32(H)
    m = H.shape[0]
    U = np.empty_like(H)
    info = lib().orc_cholesky_upper(H, m, m, U, m)
    return U, int(info)


def cholesky_inverse(H):
    """main.py:136-141: Cholesky + cholesky_inverse; on failure torch.linalg.pinv (fp32)."""
    H = _f32(H)
    m = H.shape[0]
    Hinv = np.empty_like(H)
    st = lib().orc_cholesky_inverse(H, m, m, Hinv, m)
    if st != 0:
        import torch
        return torch.linalg.pinv(torch.from_numpy(H)).numpy(), False
    return Hinv, True


def error_feedback(W, blk, rem, E, Hinv):
    """main.py:187-214 for one block on W (n x m, returned updated copy); E is (n x bs)."""
    Wt = _f32(np.asarray(W, np.float32).T).copy()
    n = Wt.shape[1]
    blk = np.ascontiguousarray(blk, np.int64); rem = np.ascontiguousarray(rem, np.int64)
    Hinv = _f32(Hinv)
    lib().orc_error_feedback(Wt, n, n, blk, len(blk), rem, len(rem), _f32(np.asarray(E).T), Hinv, Hinv.shape[1])
    return Wt.T.copy()


# ------------------------------------------------------------------ whole layer

def quantize_blocks(W, A, Hinv, block_size=128, use_ssr=True, aga_src=1, max_iter=100):
    """Block loop of main.py:158-215 / gptq.py:124-187 on W (n x m).
    aga_src: 0 none, 1 activations (A = raw Gram XᵀX), 2 Hessian block (A = damped H)."""
    W = _f32(W)
    n, m = W.shape
    Wt = _f32(W.T).copy()
    B = -(-m // block_size) if block_size < m else 1
    at = np.empty((B, n), np.float32); mt = np.empty((B, n), np.float32)
    Tt = np.zeros((m, n), np.int8)
    perm = np.empty(m, np.int64)
    iters = np.zeros(B, np.int32)
    A = _f32(A) if A is not None else np.zeros((1, 1), np.float32)
    kb = lib().orc_quantize_blocks(Wt, n, n, m, int(block_size), int(bool(use_ssr)), int(aga_src),
                                   A, A.shape[-1], _f32(Hinv), m, int(max_iter), at, mt, Tt, perm, iters)
    assert kb == B, (kb, B)
    return {"alpha": at.T.copy(), "mu": mt.T.copy(), "T": Tt.T.copy(), "perm": perm,
            "iters": iters, "W_final": Wt.T.copy()}


def is16(X):
    """fp16 numpy data or a torch bf16 tensor: the 16-bit Gram arithmetic applies."""
    return (isinstance(X, np.ndarray) and X.dtype == np.float16) or str(getattr(X, "dtype", "")) == "torch.bfloat16"


def gram_any(X):
    """The Gram the engine computes for activations of X's dtype: the 16-bit MFMA model for
    fp16 / bf16 (gram16), the f32 fmaf chain otherwise (gram)."""
    return gram16(X) if is16(X) else gram(X)


def quantize_layer_m(W, X, block_size=128, use_ssr=True, percdamp=0.01, max_iter=100):
    """PT2LLMQuantizer.quantize_layer main.py:102-230 (variant M).  X may be fp16 (numpy) or
    bf16 (torch): its Gram then follows the 16-bit MFMA arithmetic, as on the device."""
    if not is16(X):
        X = _f32(X)
    if X.ndim == 3:
        X = X.reshape(-1, X.shape[-1])
    G = gram_any(X)
    H, _ = prepare_hessian(G, X.shape[0], percdamp)
    Hinv, spd = cholesky_inverse(H)
    out = quantize_blocks(W, G, Hinv, block_size, use_ssr, 1, max_iter)
    out["spd"] = spd
    return out


def sum_partials(parts):
    """Rank-ordered fold ((P0 + P1) + P2) + ... in fp32 (the intra-layer split's reduction)."""
    acc = _f32(parts[0]).copy()
    for p in parts[1:]:
        acc = (acc + _f32(p)).astype(np.float32)
    return acc


def row_slices(N, world):
    """The calibration-row split of the intra-layer split: rank r takes rows
    [r*N//world, (r+1)*N//world) (sharding.row_slice)."""
    return [(r * N // world, (r + 1) * N // world) for r in range(world)]


def quantize_layer_split(W, X, world, block_size=128, use_ssr=True, percdamp=0.01, max_iter=100):
    """main.py:102-230 (variant M) with the Gram of main.py:128 data-parallel over `world` ranks
    (SURVEY §8e(ii)): each rank's rows form their own Gram chain from +0, the partial Grams are
    folded in rank order, the rest is the single-rank layer on that G with nsamples = N."""
    if not is16(X):
        X = _f32(X)
    if X.ndim == 3:
        X = X.reshape(-1, X.shape[-1])
    G = sum_partials([gram_any(X[a:b]) for a, b in row_slices(X.shape[0], world)])
    H, _ = prepare_hessian(G, X.shape[0], percdamp)
    Hinv, spd = cholesky_inverse(H)
    out = quantize_blocks(W, G, Hinv, block_size, use_ssr, 1, max_iter)
    out["spd"] = spd
    out["G"] = G
    return out


def quantize_layer_g(W, Hsum, nsamples, block_size=128, use_ssr=True, percdamp=0.01, max_iter=100):
    """GPTQ.quantize gptq.py:78-199 (variant G) given the accumulated H = Σ XᵢᵀXᵢ."""
    H, _ = prepare_hessian(Hsum, nsamples, percdamp)
    Hinv, spd = cholesky_inverse(H)
    out = quantize_blocks(W, H, Hinv, block_size, use_ssr, 2, max_iter)
    out["T"] = out["T"].astype(np.float32)
    out["spd"] = spd
    return out


def ternary_weight(alpha, mu, T, perm, block_size, compat, dtype=np.float16):
    """The dense weight a TernaryLinear multiplies by, rounded to the layer dtype.

    compat=True: model.py:97-110 (_dequantize: contiguous blocks of T) followed by the column
    re-index of forward (model.py:88-90), folded into one effective weight:
    out = x[..., perm] @ W[:, inv_perm]ᵀ  ==  x @ W_eff^T with W_eff[:, j] = W[:, inv_perm[inv_perm[j]]].
    compat=False: the correct reconstruction gptq.py:201-230 (block k <-> columns perm[k·b:(k+1)·b]).
    alpha/mu are rounded to `dtype` first (the reference stores them in the layer dtype), then
    alpha*t + mu is formed in fp32 and rounded to `dtype` (t in {-1,0,1} makes alpha*t exact)."""
    a = np.asarray(alpha, np.float32).astype(dtype).astype(np.float32)
    m_ = np.asarray(mu, np.float32).astype(dtype).astype(np.float32)
    T = np.asarray(T).astype(np.float32)
    perm = np.asarray(perm, np.int64)
    n, m = T.shape
    bs = block_size if block_size < m else m
    W = np.zeros((n, m), np.float32)
    for k in range(a.shape[1]):
        s, e = k * bs, min((k + 1) * bs, m)
        cols = np.arange(s, e) if compat else perm[s:e]
        W[:, cols] = (a[:, k:k + 1] * T[:, cols] + m_[:, k:k + 1]).astype(dtype).astype(np.float32)
    if compat:
        inv = np.argsort(perm)
        W = W[:, inv[inv]]
    return W


def ternary_linear(x, alpha, mu, T, perm, bias, block_size, compat, dtype=np.float16):
    """TernaryLinear.forward (model.py:75-95): fp32 accumulation of the dtype-rounded operands,
    output rounded to dtype.  Floating-point: compared with a tolerance."""
    W = ternary_weight(alpha, mu, T, perm, block_size, compat, dtype)
    xf = np.asarray(x, np.float32).astype(dtype).astype(np.float64)
    y = xf.reshape(-1, xf.shape[-1]) @ W.astype(np.float64).T
    if bias is not None:
        y = y + np.asarray(bias, np.float32).astype(dtype).astype(np.float64)
    return y.astype(np.float32).astype(dtype).reshape(*np.shape(x)[:-1], W.shape[0])
