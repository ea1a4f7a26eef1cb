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


def test_argument_bounds_without_device(pt2q):
    """Lengths that would overflow the kernels' 32-bit row counts and leading dimensions shorter
    than a row are rejected before any device work (fake non-null pointers are never touched)."""
    lib = pt2q._lib.lib()
    E_ARG = 1
    p = ctypes.c_void_p(4096)
    F16, I8 = 1, 3
    assert lib.pt2q_gram(p, F16, 2**31, 64, 64, p, 64, 0, None, 0, None) == E_ARG
    assert lib.pt2q_gram(p, F16, 100, 64, 32, p, 64, 0, None, 0, None) == E_ARG
    assert lib.pt2q_gram(p, F16, 100, 64, 64, p, 63, 0, None, 0, None) == E_ARG

    def layer(ldw=64, N=100, ldx=64):
        return lib.pt2q_quantize_layer(p, 0, ldw, 16, 64, p, F16, N, ldx, 32, 0x11, 0.01, 100, p, p,
                                       p, I8, p, None, p, p, 1 << 30, None)
    assert layer(ldw=63) == E_ARG
    assert layer(ldx=32) == E_ARG
    assert layer(N=2**31) == E_ARG
    assert lib.pt2q_quantize_blocks(p, 0, 63, 16, 64, 32, 0x11, p, 64, p, 64, 100, p, p, p, I8, p,
                                    None, p, 1 << 30, None) == E_ARG
    assert lib.pt2q_quantize_blocks(p, 0, 64, 16, 64, 32, 0x11, p, 32, p, 64, 100, p, p, p, I8, p,
                                    None, p, 1 << 30, None) == E_ARG
    assert lib.pt2q_ssr_select(p, 63, 16, 64, p, 64, 32, p, p, None, p, 1 << 30, None) == E_ARG


def test_workspace_sizes(pt2q):
    lib = pt2q._lib.lib()
    st = pt2q._lib.STATUS_BYTES
    assert st == 256
    assert lib.pt2q_strerror(pt2q._lib.PT2Q_E_STALL).decode().startswith("a cross-workgroup wait")
    # every workspace-taking call reserves the status word first
    assert lib.pt2q_gram_workspace_bytes(4096) >= st + 272 * 4
    assert lib.pt2q_ssr_workspace_bytes(4096, 4096) > st + 4096 * 4096 * 5
    # variant G blocks wider than 128 columns carry the gathered H_bb and S = H_bbᵀH_bb
    m = 1000
    g = lib.pt2q_layer_workspace_bytes(200, m, m, 0x20)
    a = lib.pt2q_layer_workspace_bytes(200, m, m, 0x10)
    assert g - a >= 2 * m * m * 4
    # ternary inference: a prefill-sized call needs only its own split (1) of partial sums, not
    # the decode bound of 16 (4096 tokens through an 11008 x 4096 projection: <= ~215 MB)
    P = lib.pt2q_ternary_linear_positions(4096)
    pre = lib.pt2q_ternary_linear_workspace_bytes(4096, 11008, 4096)
    assert pre <= 4096 * P * 2 + 4096 * 11008 * 4 + 512
    dec = lib.pt2q_ternary_linear_workspace_bytes(1, 4096, 4096)
    assert dec >= P * 2 + 2 * 4096 * 4  # decode splits K


def test_ops_refuse_cpu_tensors(pt2q):
    import torch
    with pytest.raises(pt2q._lib.Pt2qError):
        pt2q.gram(torch.zeros(4, 4))


def test_reference_surface_fails_loudly_without_gpu(pt2q):
    """The class surface takes CPU tensors (the reference's call shape) but computes on the GPU;
    on a machine without one it raises instead of falling back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    with pytest.raises(pt2q._lib.Pt2qError):
        pt2q.AsymmetricTernaryQuantizer().quantize(torch.zeros(4, 128))
    with pytest.raises(pt2q._lib.Pt2qError):
        pt2q.select_next_block_ssr(torch.zeros(4, 300), torch.arange(300), 128)


def test_group_support_query_and_block_workspace(pt2q):
    """pt2q_quantize_blocks_group_supported restates every E_UNSUPPORTED condition of the grouped
    entry (host only), and engine.group_supported asks it rather than restating them."""
    lib = pt2q._lib.lib()
    ACT, SSR, HESS = pt2q._lib.AGA_ACT, pt2q._lib.FLAG_SSR, pt2q._lib.AGA_HESS
    ok = lib.pt2q_quantize_blocks_group_supported
    assert ok(4096, 4096, 128, SSR | ACT) == 1
    assert ok(11008, 4096, 128, SSR | ACT) == 1 and ok(4096, 11008, 128, SSR | ACT) == 1
    assert ok(4096, 4096, 256, SSR | ACT) == 0       # blocks > 128 columns
    assert ok(4096, 128, 128, SSR | ACT) == 0        # one block: no error feedback to group
    assert ok(4096, 4096, 128, SSR | HESS) == 0      # variant G (H_bb AGA) per linear
    assert ok(4098, 4096, 128, SSR | ACT) == 0       # n % 4
    assert ok(4096, 4098, 128, SSR | ACT) == 0       # m % 4: EF coefficient rows 16-byte aligned
    assert ok(16384, 40000, 128, SSR | ACT) == 0     # Wt >= 2 GiB: past the EF buffer range
    assert pt2q.engine.group_supported(4096, 4096, 128) and not pt2q.engine.group_supported(4096, 4098, 128)
    # the per-linear block loop's own workspace: status word + loop buffers, far below the
    # layer figure (which adds the Gram, Hessian, inverse and their scratch)
    n, m = 5120, 13824
    b = lib.pt2q_blocks_workspace_bytes(n, m, 1 << 14, SSR | ACT)
    assert pt2q._lib.STATUS_BYTES + m * 5120 * 5 < b < lib.pt2q_layer_workspace_bytes(n, m, 1 << 14, SSR | ACT)
    assert lib.pt2q_blocks_workspace_bytes(0, m, 128, 0) == 0


def test_stage_timing_host_side(pt2q):
    """pt2q_stage_timing with no bracketed launches: enabling clears the log, reading sums
    nothing and makes no device call (so it runs here without a GPU)."""
    lib = pt2q._lib
    lib.stage_timing(True)
    lib.stage_timing(False)
    t = lib.stage_timing_read()
    assert t["records"] == 0 and all(t[k] == 0.0 for k in lib.TIMERS)
    assert lib.TIMERS.index("ef") == 3 and lib.TIMERS.index("inverse") == 6  # PT2Q_TIMER_* order


def test_quantize_blocks_hinv_optional_only_per_channel(pt2q):
    """Hinv may be NULL only for one block (b >= m: nothing reads it); with several blocks the
    call is refused before any device work (fake non-null pointers are never touched)."""
    lib = pt2q._lib.lib()
    p = ctypes.c_void_p(4096)
    E_ARG, I8 = 1, 3
    assert lib.pt2q_quantize_blocks(p, 0, 64, 16, 64, 32, 0x11, p, 64, None, 64, 100, p, p, p, I8, p,
                                    None, p, 1 << 30, None) == E_ARG


def test_gram_order_tables_cover_every_tile_once():
    """csrc/gram_order.inc (tools/gram_order_search.c): each searched batched-Gram tile order is a
    permutation of the T (T + 1) / 2 upper tiles of its width, and its runs of 32 (one XCD's
    concurrent tiles) read fewer distinct X panels per k-row than the super-block order they
    replace -- the order decides only which workgroup computes which tile, so this (and the
    bit-exact batched-Gram GPU tests) is its whole contract."""
    src = open(os.path.join(ROOT, "snlp---tenary-post-train-quantization_amd", "csrc", "gram_order.inc")).read()
    tab = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{4})", src)]
    Ts = [int(v) for v in re.search(r"go_T\[GO_COUNT\] = \{([^}]*)\}", src).group(1).split(",")]
    offs = [int(v) for v in re.search(r"go_off\[GO_COUNT\] = \{([^}]*)\}", src).group(1).split(",")]
    claimed = {int(T): (int(c), int(c0)) for T, c, c0 in
               re.findall(r"T = (\d+): \d+ tiles, \d+ runs; distinct panels per k-row (\d+) \(super-block order (\d+)\)", src)}
    assert len(Ts) == len(offs) == len(claimed) and offs[0] == 0
    for T, o in zip(Ts, offs):
        nt = T * (T + 1) // 2
        tiles = [(e & 0xFF, e >> 8) for e in tab[o:o + nt]]
        assert sorted(tiles) == sorted((a, b) for b in range(T) for a in range(b + 1)), T
        panels = sum(len({p for t in tiles[r:r + 32] for p in t}) for r in range(0, nt, 32))
        assert panels == claimed[T][0] < claimed[T][1], T
    assert len(tab) == offs[-1] + Ts[-1] * (Ts[-1] + 1) // 2


def test_chol_lane_stream_keeps_chain_order():
    """csrc/chol_lane.inc (tools/gen_chol_lane.py): the committed stream is the generator's output,
    and replaying its items symbolically, every chain receives the terms of rows 0, 1, 2, ... in
    ascending order and row R's value is used only once chain R has all its terms and its
    division -- the PT2Q chain order, so the one-lane kernel's bits are the oracle's."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_chol_lane", os.path.join(ROOT, "tools", "gen_chol_lane.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    src = open(gen.OUT).read()
    assert gen.gen(False) in src and gen.gen(True) in src
    NB = gen.NB
    terms = [[] for _ in range(NB)]  # rows applied to each chain, in order
    final = set()
    for R, c, diag in gen.stream():
        if diag:
            assert terms[R] == list(range(R)), R  # chain R complete before its division
            final.add(R)
        assert R in final
        for j in range(4 * c, 4 * c + 4):
            if j > R:
                terms[j].append(R)
    assert all(terms[j] == list(range(j)) for j in range(NB))
    assert final == set(range(NB))
