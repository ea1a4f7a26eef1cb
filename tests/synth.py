"""Counter-based synthetic inputs shared by tests, fixtures and the HIP generator.

Every value is c * scale with c = (splitmix64(splitmix64(seed) + index) >> 40) - 2**23, an
integer exactly representable in fp32, times an fp32 scale: ONE IEEE rounding, so numpy, the C
oracle and the HIP kernel `pt2q_fill_synthetic` produce bit-identical tensors without any
transfer.  Weights: uniform with std `std` (default 0.02, LLM-like).  Activations: unit-variance
uniform with ~1 % outlier feature channels scaled x20 (realistic Hessian conditioning).
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_C1 = np.uint64(0x9E3779B97F4A7C15)
_C2 = np.uint64(0xBF58476D1CE4E5B9)
_C3 = np.uint64(0x94D049BB133111EB)
OUTLIER_SALT = 0x5BD1E995


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _C1
        z = (z ^ (z >> np.uint64(30))) * _C2
        z = (z ^ (z >> np.uint64(27))) * _C3
    return z ^ (z >> np.uint64(31))


def centered24(seed, count):
    base = splitmix64(np.uint64(seed))
    idx = np.arange(count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = splitmix64(base + idx)
    return ((h >> np.uint64(40)).astype(np.int64) - (1 << 23)).astype(np.float32)


def scale_for_std(std):
    return np.float32(std * np.sqrt(3.0) / float(1 << 23))


def weights(seed, n, m, std=0.02):
    """(n, m) fp32, uniform, std `std`."""
    return (centered24(seed, n * m) * scale_for_std(std)).reshape(n, m)


def outlier_mask(seed, m, every=100):
    h = splitmix64(splitmix64(np.uint64(seed ^ OUTLIER_SALT)) + np.arange(m, dtype=np.uint64))
    return (h % np.uint64(every)) == 0


def activations(seed, N, m, outliers=True):
    """(N, m) fp32, unit variance, ~1 % outlier channels x20."""
    c = centered24(seed, N * m).reshape(N, m)
    s = scale_for_std(1.0)
    scales = np.full(m, s, dtype=np.float32)
    if outliers:
        scales[outlier_mask(seed, m)] = np.float32(s * np.float32(20.0))
    return c * scales[None, :]
