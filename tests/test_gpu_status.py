"""Stalled cross-workgroup hand-offs fail loudly (ADVICE r1 / VERDICT r1 weak #6).

The stream-K Gram partials, the ATQ launch's S1/d hand-off and the top-k pick hand-off each
poll a flag a bounded number of times.  When a wait gives up, the kernel sets a bit in the call's
status word (the head of its workspace, include/pt2q.h PT2Q_STATUS_BYTES) and the Python layer
raises Pt2qError instead of returning results computed from stale data.  The cap is a load-time
setting (PT2Q_DEBUG_SPIN_CAP; 0 makes every hand-off report a stall), so the forced-stall runs
happen in a child process."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r'''
import sys, torch
sys.path.insert(0, ROOT)
import pt2q_loader
pt2q = pt2q_loader.load()
X = pt2q.fill_synthetic((16384, 4096), 5, outliers=True).half()
W = pt2q.fill_synthetic((1024, 4096), 6, std=0.02)
def attempt(tag, fn):
    try:
        fn()
        torch.cuda.synchronize()
        print(tag, "NO-RAISE", flush=True)
    except pt2q._lib.Pt2qError as e:
        print(tag, "RAISED", e, flush=True)
attempt("gram", lambda: pt2q.gram(X))
attempt("layer", lambda: pt2q.quantize_layer(W, X))
g = pt2q.LayerGraph(W, X)
g.replay()
attempt("graph", g.spd)
'''


def run_child(cap):
    env = dict(os.environ)
    if cap is None:
        env.pop("PT2Q_DEBUG_SPIN_CAP", None)
    else:
        env["PT2Q_DEBUG_SPIN_CAP"] = str(cap)
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_forced_stall_raises():
    """Spin cap 0: the Gram's continuing pieces and the ATQ rows report their hand-off as
    stalled, and every entry point raises."""
    out = run_child(0)
    assert "gram RAISED" in out and "Gram partial-tile hand-off" in out, out
    assert "layer RAISED" in out, out
    assert "graph RAISED" in out, out


def test_default_cap_no_stall(pt2q):
    """The default cap never trips on a healthy run (same workload, in process)."""
    X = pt2q.fill_synthetic((16384, 4096), 5, outliers=True).half()
    W = pt2q.fill_synthetic((1024, 4096), 6, std=0.02)
    G = pt2q.gram(X)
    out = pt2q.quantize_layer(W, X)
    assert out.spd and int(out.status.item()) == 0
    assert G.shape == (4096, 4096)
