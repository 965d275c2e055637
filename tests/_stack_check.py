"""Shared checks of the device stack path against the oracle (tests only)."""
from __future__ import annotations

import numpy as np

from oracle import path as op


def oracle_stack(echo, cfg, geo):
    F, G, R, B = echo.shape
    per_frame = [{gain: op.polar_scatter(echo[f, k], np.full(R, cfg.scale, np.float32),
                                         geo.cos_t, geo.sin_t)
                  for k, gain in enumerate(cfg.gains)} for f in range(F)]
    return op.build_frames(per_frame)


def check_stack_vs_oracle(res, n_frames, frames, o_frames, o_labels, o_clusters, o_trk):
    assert res.n_points == sum(len(p) for _, p, _ in frames)
    np.testing.assert_array_equal(res.labels.cpu().numpy(), o_labels)
    # per-frame cluster rows in reference order
    fo, order, seg = res.frame_order_offsets, res.frame_order, res.seg
    got = [(f, int(seg["label"][s]), int(seg["count"][s]), seg["cx"][s], seg["cy"][s],
            float(seg["mi"][s])) for f in range(n_frames) for s in order[fo[f]:fo[f + 1]]]
    exp = [(fid, c[0], c[1], c[2][0], c[2][1], c[3]) for fid, _, _ in o_frames
           for c in o_clusters.get(fid, [])]
    assert got == exp
    a = list(o_trk.objects.values())
    b = res.tracker.objects()
    assert [x.object_id for x in a] == [x.object_id for x in b]
    assert [x.object_type for x in a] == [x.object_type for x in b]
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.vstack(x.positions), np.vstack(y.positions))
        assert x.frames_seen == y.frames_seen
