"""Parity at the bench's own headline workload (BASELINE configs[3]): ONE 1000-frame 3-gain
fused stack, ~50 M points, land filter + ST-DBSCAN + per-frame clusters + tracker — bit-exact
against the oracle (4_temporal_object_tracker.py run_pipeline :941-991).

The oracle's outputs for the two seeded stacks the bench alternates (std0 = SynthConfig(
n_frames=1000), std1 = seed 1 / target seed 124) are committed as per-frame / per-object digests
by tests/golden/make_bigstack.py (the oracle needs minutes on this size; the digests are
compared here in seconds, tests/_digest.py).

* the bench's submit path: FrameStackPipeline(lanes=3, async_host=True) with std0 / std1
  alternating, so every lane's second stack differs from its first (K1 capacity, K9 label-bit
  and segment-count speculation from the previous run miss inside the checked runs);
* the frame-sharded path at its real per-rank share: 8 ranks x 125 frames (gloo, sharing the
  one GPU), rank 0 digests the gathered result.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from _digest import compare, device_digest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
GOLD = Path(__file__).resolve().parent / "golden"


def _gold(name):
    return json.loads((GOLD / f"bigstack_{name}.json").read_text())


def _cfg(name):
    from rpt.synth import SynthConfig

    return SynthConfig(**_gold(name)["synth"])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("lanes", [3, 5])
def test_bench_stacks_lanes3_match_oracle(gpu, lanes):
    """The bench's submit path with `lanes` stacks in flight (5: the N=1 default): every run's
    labels, per-frame cluster rows and tracks against the oracle digests; two runs more than
    lanes, alternating the two stacks, so lanes switch workloads."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth

    names = ["std0", "std1"]
    cfgs = [_cfg(n) for n in names]
    dss = [DeviceSynth(c, gpu) for c in cfgs]
    echoes = [d.echo() for d in dss]
    torch.cuda.synchronize(gpu)
    c0 = cfgs[0]
    assert all(np.array_equal(d.geo.cos_t, dss[0].geo.cos_t) for d in dss)
    pipe = FrameStackPipeline(c0.gains, c0.rows, c0.bins, PathParams(), gpu, async_host=True,
                              lanes=lanes)
    pipe.set_geometry(np.full(c0.rows, c0.scale, np.float32), dss[0].geo.cos_t,
                      dss[0].geo.sin_t, c0.n_frames * len(c0.gains))
    # every lane busy, then two more runs: the lanes that take them switch workloads (a run takes
    # whichever lane is free)
    order = [k % 2 for k in range(lanes)] + [lanes % 2, (lanes + 1) % 2]
    futs = [pipe.submit(echoes[k], keep_points=True) for k in order]
    for i, (k, f) in enumerate(zip(order, futs)):
        res = f.result().finish()
        got = device_digest(res)
        compare(got, _gold(names[k]), f"run {i} ({names[k]}, {lanes} lanes)")
        del res


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,lanes", [(8, 1), (4, 2)])
def test_sharded_share_matches_oracle(world, lanes):
    """world x (1000/world) frames: the per-rank shares of the 1000-frame stack (8 ranks = the
    configs[3] strong-scaling share); lanes 2 alternates std0 / std1 through rpt.dist.ShardLanes."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", str(ROOT / "tools" / "dist_check.py"),
           "--backend", "gloo", "--frames", str(1000 // world), "--lanes", str(lanes),
           "--digest", "std0,std1" if lanes > 1 else "std0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=840)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ok=True" in out, out[-4000:]


def _dense_invariants(gpu, n_frames, min_points):
    """Full-size invariants of the reference semantics on a dense stack the
    whole-stack oracle cannot label:
      * K5: the core flags of >= 200,000 sample points equal the oracle's exact neighbour count
        >= min_samples (oracle.sample_check) -- 180,000 random points plus EVERY point of 50
        random 16 m x 16 m patches of random frames, so whole cells (K5 decides most cells as a
        unit) are checked point by point, not one sample per cell;
      * a core sample's core neighbours all carry its label; a non-core sample carries the
        smallest label among its core neighbours, -1 without one (4_temporal_object_tracker.py
        :493-504, the BFS's result);
      * over ALL points: every core point is labelled, cluster ids ascend with each cluster's
        minimum core index (the BFS opens clusters in index order), ids are dense;
      * K9: segment counts equal the (frame, label) histogram; the centroids and mean
        intensities of the largest and of 40 random segments equal np.mean as :527-531 take it.
    """
    import oracle
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, dense_config

    cfg = dense_config(n_frames=n_frames)
    ds = DeviceSynth(cfg, gpu)
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), gpu)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      cfg.n_frames * len(cfg.gains))
    res = pipe.run(ds.echo(), keep_points=True, keep_core=True)
    n = res.n_clustered_input
    assert n > min_points
    x = res.points["x"].cpu().numpy()
    y = res.points["y"].cpu().numpy()
    v = res.points["v"].cpu().numpy()
    pf = res.points["frame"].cpu().numpy()
    core = res.points["core"].cpu().numpy()
    lab = res.labels.cpu().numpy()
    del res.points, res.labels
    xy = np.column_stack([x, y])
    t = pf.astype(np.float32)
    fstart = np.searchsorted(pf, np.arange(pf.max() + 2))

    rng = np.random.default_rng(7)
    patches = []
    for f in rng.choice(int(pf.max()) + 1, 50):
        a, b = fstart[f], fstart[f + 1]
        c = xy[a + rng.integers(0, b - a)]
        inside = (np.abs(x[a:b] - c[0]) <= 8.0) & (np.abs(y[a:b] - c[1]) <= 8.0)
        patches.append(a + np.nonzero(inside)[0])
    patch = np.concatenate(patches)
    idx = np.unique(np.concatenate([rng.choice(n, 180_000, replace=False), patch, [0, n - 1]]))
    assert len(idx) >= 200_000 and len(patch) > 15_000
    cnt, lo, hi = oracle.sample_check(xy, t, 8.0, 2.0, idx, core, lab)
    np.testing.assert_array_equal(core[idx], (cnt >= 15).astype(np.uint8))
    c = core[idx] == 1
    np.testing.assert_array_equal(lo[c], lab[idx][c])
    np.testing.assert_array_equal(hi[c], lab[idx][c])
    np.testing.assert_array_equal(lab[idx][~c], lo[~c])

    cl = lab[core == 1]
    assert (cl >= 0).all() and ((lab >= 0) | (core == 0)).all()
    ids, first = np.unique(cl, return_index=True)
    np.testing.assert_array_equal(ids, np.arange(res.n_clusters))
    assert (np.diff(first) > 0).all(), "cluster ids must ascend with their minimum core index"
    assert lab.max() == res.n_clusters - 1

    seg = res.seg
    m = lab >= 0
    key = pf[m].astype(np.int64) << 32 | lab[m].astype(np.int64)
    uk, uc = np.unique(key, return_counts=True)
    sk = seg["frame"].astype(np.int64) << 32 | seg["label"].astype(np.int64)
    o = np.argsort(sk)
    np.testing.assert_array_equal(sk[o], uk)
    np.testing.assert_array_equal(seg["count"][o], uc)
    assert seg["count"].sum() == m.sum() and len(uk) == res.n_segments
    pick = np.unique(np.concatenate([[int(np.argmax(seg["count"]))],
                                     rng.choice(res.n_segments, 40, replace=False)]))
    for s in pick:
        f, lb = int(seg["frame"][s]), int(seg["label"][s])
        a, b = fstart[f], fstart[f + 1]
        sel = lab[a:b] == lb
        cxy = np.mean(xy[a:b][sel], axis=0)
        assert (seg["cx"][s], seg["cy"][s]) == (cxy[0], cxy[1]), (f, lb)
        assert seg["mi"][s] == np.float32(np.mean(v[a:b][sel])), (f, lb)


@pytest.mark.timeout(600)
def test_dense_config4_share_invariants(gpu):
    """configs[4]'s per-GPU share at 8 GPUs: 125 dense frames (~490k points per frame, ~61 M
    points, one component chaining the stack); _dense_invariants."""
    _dense_invariants(gpu, 125, 55_000_000)


@pytest.mark.timeout(900)
def test_dense_above_2_26_points_invariants(gpu):
    """140 dense frames: ~68.7 M points enter ST-DBSCAN, past 2^26 = 67.1 M (the configs[4] share
    at fewer than 8 GPUs is above it), through the shipped (fused) K5: its per-cell (original,
    sorted) minima are u64 pairs at every size (k_slab_bucket / k_cell_box / k_core_slow), so this
    covers the index arithmetic of the default path past 2^26.  _dense_invariants."""
    _dense_invariants(gpu, 140, 1 << 26)


@pytest.mark.timeout(900)
def test_dense_above_2_26_unfused_k5_invariants():
    """The same 140 dense frames through the A/B build's separate K5 fill pass (librpt_ab.so,
    RPT_K5_FUSED=0): the only K5 form that packs a cell's (original << 6 | lane) minimum into 32
    bits below 2^26 points and switches to the 64-bit segmented minimum above it
    (csrc/stdbscan.hip k_core_fill); that branch runs here.  _dense_invariants in a child
    process (the library is chosen at load time)."""
    from rpt import _build

    assert _build.LIB_AB.exists(), "librpt_ab.so missing: run __graft_entry__.build()"
    tests = str(Path(__file__).resolve().parent)
    code = (f"import sys\nsys.path[:0] = {[tests, *sys.path]!r}\n"
            "import torch\nfrom rpt import _abi\n"
            "assert _abi.load()._name.endswith('librpt_ab.so')\n"
            "from test_bigstack_gpu import _dense_invariants\n"
            "_dense_invariants(torch.device('cuda', 0), 140, 1 << 26)\nprint('UNFUSED_OK')\n")
    env = dict(os.environ, RPT_LIB=str(_build.LIB_AB), RPT_K5_FUSED="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=840)
    assert r.returncode == 0 and "UNFUSED_OK" in r.stdout, (r.stdout + r.stderr)[-4000:]
