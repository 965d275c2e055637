"""Host-side halves of librpt (no GPU needed): C-ABI exports, CPython set-order emulation,
scipy-exact LSAP, and the C++ ObjectTracker against the reference's golden sequences."""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment

from test_oracle_golden import replay_tracker

ROOT = Path(__file__).resolve().parents[1]


def test_library_exports_every_header_symbol():
    from rpt import _abi

    lib = _abi.load()
    hdr = (ROOT / "include" / "rpt.h").read_text()
    declared = sorted(set(re.findall(r"\b(rpt_[a-z0-9_]+)\s*\(", hdr)))
    assert len(declared) >= 25
    missing = [s for s in declared if getattr(lib, s, None) is None]
    assert missing == [], f"declared in include/rpt.h but not exported: {missing}"
    assert lib.rpt_missing_symbols == []
    bound = set(_abi.EXPORTED)
    assert set(declared) <= bound, f"not bound in rpt/_abi.py: {set(declared) - bound}"
    assert lib.rpt_version() >= 100


@pytest.mark.parametrize("seed", range(40))
def test_set_order_matches_cpython(seed):
    from rpt.native_tracker import set_order

    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 3, 5, 8, 20, 60, 200, 1500]))
    hi = int(rng.choice([10, 64, 1000, 10**6]))
    vals = rng.integers(0, hi, n * 2)
    if rng.random() < 0.7:
        vals = np.insert(vals, int(rng.integers(0, len(vals) + 1)), -1)
    seq = []
    seen = set()
    for v in vals.tolist():
        if v not in seen:
            seen.add(v)
            seq.append(v)
    arr = np.array(seq, dtype=np.int32)
    ref = set(arr)          # np.int32 elements, exactly as the reference builds it
    ref.discard(-1)
    assert set_order(seq) == [int(v) for v in ref]


def test_order_clusters_stack_matches_per_frame():
    """rpt_order_clusters over a whole stack (segments in arbitrary order, bucketed by frame):
    every frame's order must equal the single-frame call's (CPython set order of its labels by
    first index, noise included)."""
    from rpt import stages

    rng = np.random.default_rng(7)
    F, per = 300, 40
    frames = np.repeat(np.arange(F, dtype=np.int32), per)
    labels = np.concatenate([rng.choice(60000, per, replace=False) for _ in range(F)])
    first = np.concatenate([np.sort(rng.choice(10**6, per, replace=False)) for _ in range(F)])
    perm = rng.permutation(len(frames))  # segments in arbitrary order
    seg = {"frame": frames[perm], "label": labels[perm].astype(np.int32),
           "first": first[perm].astype(np.int64)}
    noise = rng.integers(-1, 10**6, F).astype(np.int64)
    fo, order = stages.order_frames(F, seg, noise)
    for f in range(F):
        idx = np.nonzero(seg["frame"] == f)[0]
        sub = {"frame": np.zeros(len(idx), np.int32), "label": seg["label"][idx],
               "first": seg["first"][idx]}
        _, o1 = stages.order_frames(1, sub, noise[f:f + 1])
        np.testing.assert_array_equal(order[fo[f]:fo[f + 1]], idx[o1], err_msg=f"frame {f}")


def _tracker_state(trk):
    return [(o.object_id, o.object_type, np.vstack(o.positions).tobytes(), tuple(o.frames_seen),
             np.vstack(o.velocities).astype(np.float64).tobytes()) for o in trk.objects()]


@pytest.mark.parametrize("F,with_ids", [(0, False), (1, False), (50, True), (700, False),
                                        (1500, True)])
def test_order_and_track_matches_two_step(F, with_ids):
    """rpt_order_and_track (frames ordered on a second thread ahead of the tracker) == the
    order (rpt_order_clusters) then the tracker (rpt_tracker_run) over the gathered centroids:
    same order, same tracker state -- segments in arbitrary order, empty and unbuilt frames,
    noise, frame ids other than the slots."""
    from rpt import stages
    from rpt.pipeline import PathParams

    rng = np.random.default_rng(F + 3)
    tgt = rng.random((30, 2)) * 300 - 150
    vel = rng.normal(0, 1.5, (30, 2))
    frames, labels, firsts, cxs, cys = [], [], [], [], []
    for f in range(F):
        if rng.random() < 0.05:
            continue  # no segment: frame not built, or built with noise only
        keep = np.nonzero(rng.random(30) < 0.85)[0]
        n_extra = int(rng.integers(0, 5))
        k = len(keep) + n_extra
        pos = np.vstack([tgt[keep] + vel[keep] * f + rng.normal(0, 0.4, (len(keep), 2)),
                         rng.random((n_extra, 2)) * 400 - 200])
        frames += [f] * k
        labels += list(rng.choice(10**5, k, replace=False))
        firsts += list(rng.choice(10**6, k, replace=False))
        cxs += list(pos[:, 0])
        cys += list(pos[:, 1])
    perm = rng.permutation(len(frames))
    seg = {"frame": np.asarray(frames, np.int32)[perm], "label": np.asarray(labels, np.int32)[perm],
           "first": np.asarray(firsts, np.int64)[perm],
           "cx": np.asarray(cxs, np.float32)[perm], "cy": np.asarray(cys, np.float32)[perm]}
    noise = np.where(rng.random(F) < 0.7, rng.integers(0, 10**6, F), -1).astype(np.int64)
    built = np.nonzero((np.bincount(seg["frame"], minlength=F) > 0) | (noise >= 0))[0]
    ids = (np.arange(F, dtype=np.int64) * 3 + 1000) if with_ids else None
    p = PathParams()
    fo1, order1 = stages.order_frames(F, seg, noise)
    trk1 = stages.track_ordered(built, fo1, order1, seg, p, None if ids is None else ids[built])
    fo2, order2, trk2 = stages.order_and_track(F, built, seg, noise, p, ids)
    np.testing.assert_array_equal(fo1, fo2)
    np.testing.assert_array_equal(order1, order2)
    assert len(trk2) == len(trk1)
    assert _tracker_state(trk2) == _tracker_state(trk1)
    if F:
        assert len(trk1) > 0


def test_order_and_track_invalid():
    from rpt import _abi
    from rpt.native_tracker import NativeTracker

    lib = _abi.load()
    trk = NativeTracker()
    fr = np.array([0, 1], np.int32)
    lab = np.array([3, 4], np.int32)
    first = np.array([0, 5], np.int64)
    noise = np.full(2, -1, np.int64)
    c = np.zeros(2, np.float32)
    fo = np.empty(3, np.int64)
    order = np.empty(2, np.int64)

    def call(built, frames=fr):
        b = np.asarray(built, np.int64)
        p = lambda a, t: a.ctypes.data_as(t)  # noqa: E731
        return lib.rpt_order_and_track(2, 2, p(frames, _abi.c_i32p), p(lab, _abi.c_i32p),
                                       p(first, _abi.c_i64p), p(noise, _abi.c_i64p),
                                       p(c, _abi.c_f32p), p(c, _abi.c_f32p), len(b),
                                       p(b, _abi.c_i64p), None, trk._h, p(fo, _abi.c_i64p),
                                       p(order, _abi.c_i64p))

    assert call([0, 1]) == 0
    assert call([1, 0]) == 1  # not ascending
    assert call([0, 2]) == 1  # out of range
    assert call([0, 1], np.array([0, 2], np.int32)) == 1  # segment frame out of range


def _lsap_cases():
    rng = np.random.default_rng(0)
    for k in range(60):
        nr, nc = rng.integers(1, 30, 2)
        kind = k % 4
        if kind == 0:
            c = rng.random((nr, nc)) * 100
        elif kind == 1:
            c = rng.integers(0, 4, (nr, nc)).astype(np.float64)  # heavy ties
        elif kind == 2:
            c = np.full((nr, nc), 7.0)
        else:
            c = np.round(rng.random((nr, nc)) * 50, 1)
        yield c
    yield np.zeros((0, 3))
    yield np.array([[np.inf, 1.0], [2.0, np.inf]])


@pytest.mark.parametrize("i", range(62))
def test_lsap_matches_scipy(i):
    from rpt.native_tracker import lsap

    c = list(_lsap_cases())[i]
    ra, ca = linear_sum_assignment(c)
    rb, cb = lsap(c)
    np.testing.assert_array_equal(ra, rb)
    np.testing.assert_array_equal(ca, cb)


def test_lsap_tie_stress_matches_scipy():
    """Tracking-sized rectangular problems with heavy ties, +inf entries and tall shapes: the
    assignment must equal scipy's exactly (tie-breaking included)."""
    from rpt.native_tracker import lsap

    rng = np.random.default_rng(7)
    for k in range(400):
        nr, nc = int(rng.integers(1, 80)), int(rng.integers(1, 80))
        c = rng.integers(0, 3 + k % 5, (nr, nc)).astype(np.float64)
        if k % 3 == 0:
            c[rng.random((nr, nc)) < 0.2] = np.inf
        try:
            ra, ca = linear_sum_assignment(c)
        except ValueError:
            with pytest.raises(ValueError):
                lsap(c)
            continue
        rb, cb = lsap(c)
        np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(ca, cb)


def test_lsap_invalid():
    from rpt.native_tracker import lsap

    with pytest.raises(ValueError):
        lsap(np.array([[np.nan, 1.0]]))
    with pytest.raises(ValueError):
        lsap(np.array([[np.inf, np.inf], [1.0, np.inf]]))


class _Adapter:
    """Feed the g5 replay helper through the native tracker."""

    def __init__(self):
        from rpt.native_tracker import NativeTracker

        self.t = NativeTracker()

    def update(self, clusters, frame_id):
        cx = np.array([c[0][0] for c in clusters], np.float32)
        cy = np.array([c[0][1] for c in clusters], np.float32)
        self.t.update_arrays(frame_id, cx, cy, [c[1] for c in clusters])
        return self.t.objects()

    @property
    def objects(self):
        return {o.object_id: o for o in self.t.objects()}


def test_native_tracker_matches_reference(golden):
    g = golden("g5_tracker.npz")
    for s in range(int(g["n_seqs"])):
        trk, alive = replay_tracker(g, s, _Adapter)
        ao = g[f"s{s}_alive_off"]
        for i, a in enumerate(alive):
            assert a == list(g[f"s{s}_alive"][ao[i]:ao[i + 1]]), f"seq {s} frame {i}"
        objs = list(trk.objects.values())
        np.testing.assert_array_equal([o.object_id for o in objs], g[f"s{s}_obj_id"])
        np.testing.assert_array_equal([o.object_type for o in objs], g[f"s{s}_obj_type"])
        pos = np.vstack([np.vstack(o.positions) for o in objs]).astype(np.float32)
        np.testing.assert_array_equal(pos, g[f"s{s}_obj_pos"])
        vel = np.vstack([np.vstack(o.velocities).astype(np.float64) for o in objs])
        np.testing.assert_array_equal(vel, g[f"s{s}_obj_vel"])
        np.testing.assert_array_equal([float(o.average_velocity) for o in objs],
                                      g[f"s{s}_obj_avgv"])
        np.testing.assert_array_equal([isinstance(o.average_velocity, np.float32) for o in objs],
                                      g[f"s{s}_obj_avgv_f32"])
        np.testing.assert_array_equal([o.color for o in objs], g[f"s{s}_obj_color"])


def test_native_tracker_random_vs_oracle():
    """Longer random sequences (births, deaths, gating, f64->f32 switch) vs the pinned oracle."""
    import oracle

    rng = np.random.default_rng(11)
    for rep in range(6):
        o = oracle.Tracker()
        n = _Adapter()
        pos = rng.random((12, 2)) * 300 - 150
        vel = rng.normal(0, 2.0, (12, 2))
        for f in range(60):
            if rng.random() < 0.1:
                continue  # frame dropped (id gap)
            cl = [pos[k] + vel[k] * f + rng.normal(0, 0.5, 2) for k in range(12)
                  if rng.random() < 0.8]
            cl += [rng.random(2) * 400 - 200 for _ in range(int(rng.integers(0, 4)))]
            cl = [(np.asarray(c, np.float32), f) for c in cl]
            o.update(cl, f)
            n.update(cl, f)
        a = list(o.objects.values())
        b = list(n.objects.values())
        assert [x.object_id for x in a] == [x.object_id for x in b]
        assert [x.object_type for x in a] == [x.object_type for x in b]
        for x, y in zip(a, b):
            np.testing.assert_array_equal(np.vstack(x.positions), np.vstack(y.positions))
            assert x.frames_seen == y.frames_seen


def test_arange_edges_match_numpy():
    """rpt_arange_edges (used by the native stack driver for the land grid) == np.arange(lo,
    hi + 5.0, 5.0) on float32 bounds, incl. lengths near integral (stop - lo) / 5."""
    from rpt import _abi

    lib = _abi.load()
    rng = np.random.default_rng(7)
    out = np.empty(4096, np.float64)
    for it in range(20000):
        if it % 3 == 0:
            a = np.float32(rng.uniform(-300, 300))
            b = np.float32(rng.uniform(a, 400))
        else:
            a = np.float32(rng.uniform(-1000, 0))
            b = np.float32(a + np.float32(rng.integers(0, 100)) * np.float32(5.0) +
                           np.float32(rng.choice([0.0, 1e-5, -1e-5, 2.5])))
        exp = np.arange(a, b + 5.0, 5.0)
        n = lib.rpt_arange_edges(float(a), float(b), 5.0, out.ctypes.data_as(_abi.c_f64p), 4096)
        assert n == len(exp)
        np.testing.assert_array_equal(out[:n], exp)


def test_int32_index_limits_return_enotsup():
    """rpt_land_filter / rpt_cluster_summaries use int32 positions: n >= 2^31 - 1 is refused
    with RPT_ENOTSUP by the size check alone (no device memory is touched)."""
    from rpt import _abi

    lib = _abi.load()
    n = (1 << 31) - 1
    st = lib.rpt_land_filter(None, None, None, None, None, n, None, 1, None, 2, None, 2, None,
                             None, None, None, None, None, None, None, None)
    assert st == _abi.RPT_ENOTSUP and b"int32" in lib.rpt_last_error()
    st = lib.rpt_cluster_summaries(None, None, None, None, None, n, 1, 1, None, None, None, None,
                                   None, None, None, None, None, None)
    assert st == _abi.RPT_ENOTSUP and b"int32" in lib.rpt_last_error()
