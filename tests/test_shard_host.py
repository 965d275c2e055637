"""Rank 0's host stage of the frame-sharded path (rpt_shard_host_stage, csrc/shard.cpp) on CPU:
synthetic packed results of several ranks -- segments with rank-local labels, each rank's table
of the representatives its window sees (shared clusters appear in several tables), built flags,
first-noise indices -- against the Python restatement: the global label of a representative is
its rank among all of them (clusters are numbered by their minimum core point,
4_temporal_object_tracker.py:479-506), then per rank part the reference cluster order of every
frame (CPython set order, :519-522; rpt.stages.order_frames) and the tracker over the built frames
(:984-991; rpt.stages.track_ordered)."""
from __future__ import annotations

import numpy as np
import pytest

from rpt import _abi
from rpt.native_tracker import NativeTracker
from rpt.pipeline import PathParams
from rpt.stages import order_frames, track_ordered

MAGIC = 0x5250545332
HDR = 8


def _pack(rank, F, frame0, segs, noise, built, reps, cap):
    S, R = len(segs["count"]), len(reps)
    words = HDR + 2 * F + 5 * S + R
    out = np.zeros(cap, np.int64)
    out[:HDR] = [MAGIC, S, R, 0, words, F, frame0, int(segs["count"].sum()) + 7]
    o = HDR
    out[o:o + F] = built
    o += F
    out[o:o + F] = noise
    o += F
    out[o:o + S] = segs["count"]
    o += S
    out[o:o + S] = segs["first"]
    o += S
    out[o:o + S] = (segs["frame"].astype(np.int64) << 32) | segs["llabel"].astype(np.int64)
    o += S
    bx = segs["cx"].view(np.uint32).astype(np.uint64)
    by = segs["cy"].view(np.uint32).astype(np.uint64)
    out[o:o + S] = ((by << np.uint64(32)) | bx).view(np.int64)
    o += S
    out[o:o + S] = segs["mi"].view(np.uint32).astype(np.int64)
    o += S
    out[o:o + R] = reps
    return out


def _synth(seed, W=4, F=6):
    rng = np.random.default_rng(seed)
    # global clusters = sorted ids (rank << 40 | index); each rank sees some of them
    pool = np.sort(np.unique(np.concatenate(
        [(np.int64(q) << 40) | rng.integers(0, 5000, 12).astype(np.int64) for q in range(W)])))
    parts, truth = [], []
    for q in range(W):
        reps = np.sort(rng.choice(pool, size=min(len(pool), 20), replace=False))
        segs = {k: [] for k in ("frame", "llabel", "count", "first", "cx", "cy", "mi")}
        noise = np.full(F, -1, np.int64)
        built = (rng.random(F) > 0.2).astype(np.int64)
        first = 0
        for f in range(F):
            if not built[f]:
                continue
            labs = rng.choice(len(reps), size=rng.integers(0, 6), replace=False)
            for ll in labs:
                c = int(rng.integers(1, 40))
                segs["frame"].append(f)
                segs["llabel"].append(int(ll))
                segs["count"].append(c)
                segs["first"].append(first + int(rng.integers(0, 30)))
                segs["cx"].append(rng.normal(0, 100))
                segs["cy"].append(rng.normal(0, 100))
                segs["mi"].append(rng.random() * 200)
            if rng.random() < 0.5:
                noise[f] = first + int(rng.integers(0, 50))
            first += 60
        segs = {k: np.array(v, dtype={"frame": np.int32, "llabel": np.int32, "count": np.int64,
                                      "first": np.int64}.get(k, np.float32))
                for k, v in segs.items()}
        parts.append(_pack(q, F, q * F, segs, noise, built, reps, HDR + 27 * F + 64))
        truth.append((segs, noise, built, reps))
    return np.ascontiguousarray(np.stack(parts)), truth, F


# (the larger stacks run the producer thread that orders frames ahead of the tracker)
@pytest.mark.parametrize("seed,W,F", [(s, 4, 6) for s in range(5)] + [(5, 4, 50), (6, 2, 300)])
def test_shard_host_stage_matches_python(seed, W, F):
    lib = _abi.load()
    g, truth, F = _synth(seed, W, F)
    W, cap = g.shape
    sizes = np.zeros(4, np.int64)
    _abi.check(lib.rpt_shard_gathered_sizes(g.ctypes.data_as(_abi.c_i64p), W, cap,
                                            sizes.ctypes.data_as(_abi.c_i64p)))
    allreps = np.unique(np.concatenate([t[3] for t in truth]))
    S = sum(len(t[0]["count"]) for t in truth)
    B = sum(int(t[2].sum()) for t in truth)
    assert sizes.tolist() == [S, B, W * F, len(allreps)]

    # Python restatement
    segs, fos, orders, built = {k: [] for k in ("frame", "label", "count", "first", "cx", "cy",
                                                "mi")}, [np.zeros(1, np.int64)], [], []
    s0 = 0
    for q, (sg, noise, bl, reps) in enumerate(truth):
        glab = np.searchsorted(allreps, reps[sg["llabel"]]).astype(np.int32)
        part = {"frame": sg["frame"], "label": glab, "first": sg["first"]}
        fo, order = order_frames(F, part, noise)
        fos.append(fo[1:] + s0)
        orders.append(order + s0)
        for k, v in (("frame", sg["frame"] + q * F), ("label", glab), ("count", sg["count"]),
                     ("first", sg["first"]), ("cx", sg["cx"]), ("cy", sg["cy"]),
                     ("mi", sg["mi"])):
            segs[k].append(v)
        built.append(np.nonzero(bl)[0] + q * F)
        s0 += len(sg["count"])
    exp = {k: np.concatenate(v) for k, v in segs.items()}
    fo_e, ord_e, built_e = np.concatenate(fos), np.concatenate(orders), np.concatenate(built)
    trk_e = track_ordered(built_e, fo_e, ord_e, exp, PathParams(), built_e)

    got = {"frame": np.empty(S, np.int32), "label": np.empty(S, np.int32),
           "count": np.empty(S, np.int64), "first": np.empty(S, np.int64),
           "cx": np.empty(S, np.float32), "cy": np.empty(S, np.float32),
           "mi": np.empty(S, np.float32)}
    bi = np.empty(max(B, 1), np.int64)
    fo = np.empty(W * F + 1, np.int64)
    order = np.empty(max(S, 1), np.int64)
    p = PathParams()
    trk = NativeTracker(p.max_association_distance, p.max_missed_frames,
                        p.motion_history_frames, p.stationary_velocity_threshold)
    P = lambda a, t: a.ctypes.data_as(t)  # noqa: E731
    _abi.check(lib.rpt_shard_host_stage(
        P(g, _abi.c_i64p), W, cap, trk._h, P(got["frame"], _abi.c_i32p),
        P(got["label"], _abi.c_i32p), P(got["count"], _abi.c_i64p), P(got["first"], _abi.c_i64p),
        P(got["cx"], _abi.c_f32p), P(got["cy"], _abi.c_f32p), P(got["mi"], _abi.c_f32p),
        P(bi, _abi.c_i64p), P(fo, _abi.c_i64p), P(order, _abi.c_i64p), None, -1))
    for k in exp:
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    np.testing.assert_array_equal(bi[:B], built_e)
    np.testing.assert_array_equal(fo, fo_e)
    np.testing.assert_array_equal(order[:S], ord_e)
    a, b = trk_e.objects(), trk.objects()
    assert [o.object_id for o in a] == [o.object_id for o in b] and len(a) > 0
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.vstack(x.positions), np.vstack(y.positions))
        assert x.frames_seen == y.frames_seen

    # the per-rank label map (labels_local)
    for q, (_, _, _, reps) in enumerate(truth):
        m = np.empty(len(reps), np.int32)
        _abi.check(lib.rpt_shard_host_stage(P(g, _abi.c_i64p), W, cap, None, None, None, None,
                                            None, None, None, None, None, None, None,
                                            P(m, _abi.c_i32p), q))
        np.testing.assert_array_equal(m, np.searchsorted(allreps, reps))


def test_shard_host_stage_rejects_incomplete_parts():
    lib = _abi.load()
    g, _, _ = _synth(0)
    g = g.copy()
    g[1, 3] = 4   # rank 1's buffer overflowed: the step must be finished again first
    sizes = np.zeros(4, np.int64)
    with pytest.raises(Exception):
        _abi.check(lib.rpt_shard_gathered_sizes(g.ctypes.data_as(_abi.c_i64p), g.shape[0],
                                                g.shape[1], sizes.ctypes.data_as(_abi.c_i64p)),
                   "rpt_shard_gathered_sizes")
