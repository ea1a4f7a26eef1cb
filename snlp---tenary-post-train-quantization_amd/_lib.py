"""ctypes binding of libpt2q.so (include/pt2q.h) for PyTorch-ROCm device tensors.

The library is the product: there is no CPU or eager-PyTorch fallback.  If the shared object
is missing this module raises at import, and every op requires tensors on a HIP device.
"""
import ctypes
import os

import torch

_DIR = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.path.join(_DIR, "libpt2q.so")

PT2Q_OK = 0
PT2Q_E_NOT_SPD = 2
PT2Q_E_STALL = 6
STATUS_BYTES = 256  # the status word at the head of a workspace (include/pt2q.h)
STALL_BITS = {0x1: "Gram partial-tile hand-off", 0x2: "ATQ S1/d hand-off", 0x4: "top-k pick hand-off"}
F32, F16, BF16, I8 = 0, 1, 2, 3
FLAG_SSR = 0x1
FLAG_S1_GIVEN = 0x2
AGA_NONE, AGA_ACT, AGA_HESS = 0x0, 0x10, 0x20
AGA_MASK = 0x30
STAGE_INIT, STAGE_GRID, STAGE_ROUND, STAGE_ITF, STAGE_AGA, STAGE_FULL = range(6)
# stage-timer classes (pt2q_stage_timing, include/pt2q.h PT2Q_TIMER_*)
TIMERS = ("setup", "ssr", "atq", "ef", "out", "gram", "inverse")

_DT = {torch.float32: F32, torch.float16: F16, torch.bfloat16: BF16, torch.int8: I8}


class Pt2qError(RuntimeError):
    pass


if not os.path.exists(SO_PATH):
    raise ImportError(
        f"libpt2q.so not found at {SO_PATH}: build it with `python -c \"import __graft_entry__ as g; "
        f"g.build()\"` (hipcc --offload-arch=gfx950). There is no CPU fallback.")

_h = ctypes.CDLL(SO_PATH)
P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
F = ctypes.c_float
SZ = ctypes.c_size_t

_SIGS = {
    "pt2q_version": (ctypes.c_char_p, []),
    "pt2q_strerror": (ctypes.c_char_p, [I]),
    "pt2q_layer_workspace_bytes": (SZ, [I, I, I, I]),
    "pt2q_cholesky_workspace_bytes": (SZ, [I]),
    "pt2q_blocks_workspace_bytes": (SZ, [I, I, I, I]),
    "pt2q_stage_timing": (I, [I]),
    "pt2q_stage_timing_read": (I, [P, I, P]),
    "pt2q_quantize_blocks_group_supported": (I, [I, I, I, I]),
    "pt2q_ssr_workspace_bytes": (SZ, [I, I]),
    "pt2q_gram_workspace_bytes": (SZ, [I]),
    "pt2q_gram": (I, [P, I, I64, I, I64, P, I64, I, P, SZ, P]),
    "pt2q_gram_batched": (I, [I, P, I, I64, I, I64, P, P]),
    "pt2q_gram_batched_upper": (I, [I, P, I, I64, I, I64, P, P]),
    "pt2q_prepare_hessian": (I, [P, I64, I, I64, F, P, I64, P, P]),
    "pt2q_cholesky_inverse": (I, [P, I64, I, P, I64, P, SZ, P, P]),
    "pt2q_hessian_inverse_batched_workspace_bytes": (SZ, [I, I]),
    "pt2q_hessian_inverse_batched": (I, [P, I, I, I64, F, P, P, P, SZ, P, P]),
    "pt2q_quantize_blocks": (I, [P, I, I64, I, I, I, I, P, I64, P, I64, I, P, P, P, I, P, P, P,
                                 SZ, P]),
    "pt2q_quantize_blocks_group_workspace_bytes": (SZ, [I, I, I, I, I]),
    "pt2q_quantize_blocks_group": (I, [I, P, I, I64, I, I, I, I, P, I64, P, I64, I, P, P, P, I, P, P, P,
                                       SZ, P]),
    "pt2q_quantize_perchannel_group_workspace_bytes": (SZ, [I]),
    "pt2q_quantize_perchannel_group": (I, [I, P, I, I64, P, I, P, I, P, P, P, I, P, P, P, SZ, P]),
    "pt2q_quantize_layer": (I, [P, I, I64, I, I, P, I, I64, I64, I, I, F, I, P, P, P, I, P, P, P,
                                P, SZ, P]),
    "pt2q_atq_stage": (I, [I, P, I64, I, I, P, P, P, I64, P, P, I, P, P, SZ, P]),
    "pt2q_s1_from_gram": (I, [P, I64, I, P, P, P]),
    "pt2q_s1_from_gram_batched": (I, [P, I64, I, I, I64, P, P]),
    "pt2q_s1_from_upper_batched": (I, [P, I64, I, I, I64, P, P]),
    "pt2q_ssr_select": (I, [P, I64, I, I, P, I, I, P, P, P, P, SZ, P]),
    "pt2q_dequantize": (I, [P, P, P, I, P, I, I, I, P, P]),
    "pt2q_error_feedback_workspace_bytes": (SZ, [I, I, I]),
    "pt2q_error_feedback": (I, [P, I64, I, I, P, I, P, I, P, I64, P, I64, P, SZ, P]),
    "pt2q_pack_ternary": (I, [P, I64, P, P]),
    "pt2q_unpack_ternary": (I, [P, I64, P, P]),
    "pt2q_fill_synthetic": (I, [P, I64, ctypes.c_uint64, F, I64, I, F, P]),
    "pt2q_sum_partials": (I, [P, I64, I, I64, P, P]),
    "pt2q_ternary_linear_positions": (SZ, [I]),
    "pt2q_ternary_pack": (I, [P, I64, I, I, P, I, P, P, P]),
    "pt2q_ternary_linear_workspace_bytes": (SZ, [I, I, I]),
    "pt2q_ternary_linear": (I, [P, I, I, I64, I, I, P, P, P, P, I, I, P, P, I, I64, P, SZ, P]),
}
for _name, (_res, _args) in _SIGS.items():
    _fn = getattr(_h, _name)
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = tuple(_SIGS)


def lib():
    return _h


def version():
    return _h.pt2q_version().decode()


def check(rc, what=""):
    if rc != PT2Q_OK:
        raise Pt2qError(f"{what}: {_h.pt2q_strerror(rc).decode()} (status {rc})")


def status_view(ws):
    """The int32 status word at the head of a workspace tensor (device; no synchronisation)."""
    return ws[:4].view(torch.int32)


def raise_stall(status: int, what=""):
    if status:
        parts = ", ".join(v for k, v in STALL_BITS.items() if status & k) or hex(status)
        raise Pt2qError(f"{what}: {_h.pt2q_strerror(PT2Q_E_STALL).decode()} [{parts}] "
                        f"(status {PT2Q_E_STALL})")


def check_status(ws, what=""):
    """Raise if a kernel of the last call on this workspace gave up a cross-workgroup wait
    (synchronises with the device: one 4-byte read)."""
    raise_stall(int(status_view(ws).item()), what)


def dtype_code(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise Pt2qError("pt2q kernels need tensors on a HIP device (MI355X); got "
                        f"{getattr(t, 'device', type(t))}")
    return t.device


def compute_device(*tensors):
    """The HIP device the kernels run on for the reference-surface classes: the inputs' own
    device if any is on a GPU, else the current HIP device (a reference-style caller passing CPU
    tensors gets its results back on the CPU -- the arithmetic still runs in libpt2q on the GPU).
    With no HIP device present this raises: there is no CPU path."""
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
    if not torch.cuda.is_available():
        raise Pt2qError("pt2q kernels need an MI355X (HIP device); none is visible and there is "
                        "no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def stage_timing(enable: bool):
    """Enable (clearing the log) or disable the library's per-stage HIP-event brackets."""
    check(_h.pt2q_stage_timing(1 if enable else 0), "pt2q_stage_timing")


def stage_timing_read():
    """{class: ms} summed over the bracketed intervals since stage_timing(True) (waits for the
    recorded events), plus "records": the number of intervals."""
    arr = (ctypes.c_double * len(TIMERS))()
    cnt = ctypes.c_int(0)
    check(_h.pt2q_stage_timing_read(ctypes.cast(arr, P), len(TIMERS), ctypes.cast(ctypes.pointer(cnt), P)), "pt2q_stage_timing_read")
    out = {k: arr[i] for i, k in enumerate(TIMERS)}
    out["records"] = cnt.value
    return out


def ptr_array(tensors):
    """A host array of device pointers (the pointer-array arguments of the grouped entries)."""
    arr = (ctypes.c_void_p * len(tensors))(*[None if t is None else t.data_ptr() for t in tensors])
    return ctypes.cast(arr, ctypes.c_void_p), arr  # keep `arr` alive across the call


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
