"""bench.py's measured paths on a small model (GPU): the transfer-inclusive step (extra.h2d,
bench.H2DStep: inputs from pinned host memory, packed results back to pinned host memory) must
produce exactly the resident step's results, and the live stage timing must bracket every stage
of the step it measures."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _small_step():
    import bench
    a = bench.parse(["--model", "llama-2-7b", "--layers", "2", "--hidden", "512", "--inter", "768",
                     "--tokens", "2048", "--no-cpu-baseline"])
    bench._load_runtime(False)
    bench.resolve(a)
    return bench, bench.ModelStep(a, 0, 1, torch.device("cuda", 0), torch.float16)


def test_h2d_step_equals_resident_step():
    bench, ms = _small_step()
    want = ms.step()  # {unit.linear: {T2, alpha, mu, perm, shape}} on the device
    h = bench.H2DStep(ms)
    manifest = h.step()
    got = bench.sharding._unflatten(manifest, h.host_res[:h.d2h_bytes])
    assert sorted(got) == sorted(want) and len(got) == 14
    for k, r in want.items():
        for f in ("T2", "alpha", "mu", "perm"):
            assert torch.equal(got[k][f], r[f].cpu()), (k, f)
    assert h.h2d_bytes > 0 and got[next(iter(got))]["T2"].device.type == "cpu"


def test_stage_busy_brackets_every_stage():
    bench, ms = _small_step()
    ms.step()
    busy = ms.stage_busy()
    for k in ("gram", "inverse", "ssr", "atq", "ef", "setup", "out"):
        assert busy[k] > 0, (k, busy)
    assert busy["records"] > 0
    # one lane: the busy times of the tail phase fit inside its wall
    tails = sum(busy[k] for k in ("setup", "ssr", "atq", "ef", "out"))
    assert tails <= busy["phase_wall_ms"]["tails"] * 1.02 + 0.5
    assert len(ms.gf.pipe.lanes) == 3  # restored after the one-lane measurement


def test_shards_union_equals_whole_step():
    """bench --shard: every rank's LPT shard of a 2-rank step run alone on this GPU (shard_only,
    no gather) gives, linear for linear, exactly the one-GPU step's results, and each non-root
    shard reports the bytes its gather would send."""
    import bench
    a = bench.parse(["--model", "llama-2-7b", "--layers", "2", "--hidden", "512", "--inter", "768",
                     "--tokens", "2048", "--no-cpu-baseline"])
    bench._load_runtime(False)
    bench.resolve(a)
    dev = torch.device("cuda", 0)
    want = bench.ModelStep(a, 0, 1, dev, torch.float16).step()
    got = {}
    for r in range(2):
        ms = bench.ModelStep(a, r, 2, dev, torch.float16, shard_only=True)
        res = ms.step()
        assert (ms.gather_bytes > 0) == (r > 0)
        if r:
            assert ms.gather_bytes == sum(e[4] for e in bench.sharding._manifest(res))
        assert not set(res) & set(got)
        got.update(res)
    assert sorted(got) == sorted(want) and len(got) == 14
    for k, r in want.items():
        for f in ("T2", "alpha", "mu", "perm"):
            assert torch.equal(got[k][f], r[f]), (k, f)


def test_shard_mode_line():
    """`bench.py --gpus 2 --shard all` (one process): the whole step, then both shards, one JSON
    line with the projection fields."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--shard", "all",
                        "--layers", "2", "--hidden", "512", "--inter", "768", "--tokens", "2048",
                        "--steps", "1", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["world"] == 2 and len(d["shards"]) == 2
    assert sum(s["linears"] for s in d["shards"]) == 14
    assert d["t1_ms"] > 0 and 0 < d["projected_efficiency"] < 2
    assert set(d["share_ratio"]) == {"gram", "inverse", "tails"}
    assert d["gather_bytes_to_rank0"] == d["shards"][1]["gather_send_bytes"] > 0


@pytest.mark.gpu
def test_two_rank_launch_shared_gpu():
    """`bench.py --gpus 2 --share-gpu` (TEST ONLY: both ranks on cuda:0, gloo gather -- RCCL refuses
    two ranks on one device): the launcher starts its own torch.distributed.run child, each rank
    quantises its LPT shard and rank 0 gathers every linear's device results; the line reports
    both ranks and the whole job's columns."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu",
                        "--layers", "2", "--hidden", "512", "--inter", "768", "--tokens", "2048",
                        "--steps", "1", "--warmup", "1", "--no-extra", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and len(d["ranks"]) == 2
    assert d["gathered_linears"] == 14 and sum(r["linears"] for r in d["ranks"]) == 14
    assert d["value"] > 0
