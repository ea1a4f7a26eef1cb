import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
GOLDEN = os.path.join(TESTS, "golden")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU case")


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))


def layer_inputs(g):
    """Regenerate (W, X) of a full-layer fixture from its seeds (tests/synth.py)."""
    import synth
    n, m, N = int(g["n"]), int(g["m"]), int(g["N"])
    W = synth.weights(int(g["wseed"]), n, m)
    X = synth.activations(int(g["xseed"]), N, m, outliers=bool(g.get("outliers", True)))
    if "zero_col" in g:
        X[:, int(g["zero_col"])] = 0.0
    if "dtype" in g:  # 16-bit fixture: the fp32 upcast of the 16-bit tensors (what the reference ran)
        W, X = round16(W, str(g["dtype"])), round16(X, str(g["dtype"]))
    return W, X


def round16(a, dtype):
    if dtype == "fp16":
        return a.astype(np.float16).astype(np.float32)
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).bfloat16().float().numpy()


def unpack2(T2, m):
    """tests/golden/gen_golden.py pack2 inverse: n x ceil(2m/8) bytes -> int8 codes n x m."""
    bits = np.unpackbits(T2, axis=1)[:, :2 * m].reshape(T2.shape[0], m, 2)
    return (bits[..., 0].astype(np.int16) * 2 + bits[..., 1] - 1).astype(np.int8)


def layer_inputs16(g):
    """16-bit fixture inputs as the engine takes them: W (fp32 upcast, exact) and X as fp16 numpy
    or bf16 torch -- the oracle then applies the 16-bit MFMA Gram arithmetic (orc.gram16)."""
    W, X = layer_inputs(g)
    if str(g["dtype"]) == "fp16":
        return W, X.astype(np.float16)
    import torch
    return W, torch.from_numpy(X).bfloat16()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def pt2q():
    """The product package (HIP path). Loaded by file path: the directory name is not an identifier."""
    import pt2q_loader
    return pt2q_loader.load()
