"""CPU-side checks of the drop-in boundary: libpt2q.so loads, exports exactly what include/pt2q.h
declares, and rejects bad arguments before touching a device."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "pt2q.h")
SO = os.path.join(ROOT, "snlp---tenary-post-train-quantization_amd", "libpt2q.so")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(pt2q_\w+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("pt2q_gram", "pt2q_prepare_hessian", "pt2q_cholesky_inverse", "pt2q_quantize_blocks",
              "pt2q_quantize_layer", "pt2q_atq_stage", "pt2q_ssr_select", "pt2q_dequantize"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(SO), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(SO)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header(pt2q):
    assert set(pt2q._lib.EXPORTED) == set(declared_symbols())
    assert pt2q._lib.version().startswith("pt2q-mi355x")


def test_host_only_entry_points(pt2q):
    lib = pt2q._lib.lib()
    ws = lib.pt2q_layer_workspace_bytes(4096, 4096, 128, 0x11)
    # Wt + Tt + 4 Hessian-sized buffers dominate
    assert ws > 4 * 4096 * 4096 * 4 + 4096 * 4096 * 5
    assert lib.pt2q_layer_workspace_bytes(0, 4096, 128, 0) == 0
    assert lib.pt2q_strerror(2).decode().startswith("Hessian not positive definite")


def test_argument_errors_without_device(pt2q):
    lib = pt2q._lib.lib()
    E_ARG = 1
    assert lib.pt2q_gram(None, 0, 10, 10, 10, None, 10, 0, None, 0, None) == E_ARG
    assert lib.pt2q_quantize_layer(None, 0, 1, 1, 1, None, 0, 1, 1, 128, 0, 0.01, 100, None, None,
                                   None, 3, None, None, None, None, 0, None) == E_ARG
    assert lib.pt2q_atq_stage(0, None, 1, 1, 1, None, None, None, 1, None, None, 100, None, None, 0,
                              None) == E_ARG


def test_ops_refuse_cpu_tensors(pt2q):
    import torch
    with pytest.raises(pt2q._lib.Pt2qError):
        pt2q.gram(torch.zeros(4, 4))
