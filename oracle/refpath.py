"""TEST / BASELINE INFRASTRUCTURE ONLY — st_dbscan with the reference's algorithmic STRUCTURE,
for bench.py's `cpu_baseline` leg: the reference itself cannot travel
to the GPU box, so this restatement of PointCloudWork/4_temporal_object_tracker.py:443-506
runs there instead, on the node's own host cores:

* ONE spatial index over every point of the stack (sklearn BallTree on the xy coordinates;
  :474) and a radius query for every point that ignores time (:475);
* per point, the time filter as a Python loop over its spatial neighbours with float32 frame
  ids (:485-486, :499-500 -- where the reference spends ~91 % of its time);
* the seed-set expansion (:490-504): a point popped from the set is visited once, a core
  point's filtered neighbours join the set, every popped noise point takes the cluster id.

Labels are bit-identical to ``oracle.stdbscan`` (pinned by tests/test_oracle_golden.py); only
the cost structure differs from the oracle's grid-indexed C BFS.  Single thread.  When sklearn
is missing, scipy's cKDTree provides the same whole-stack radius query (``index`` says which).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def _radius_neighbours(xy: np.ndarray, eps: float) -> Tuple[list, str]:
    try:
        from sklearn.neighbors import BallTree

        return BallTree(xy).query_radius(xy, r=eps), "sklearn.BallTree"
    except ImportError:  # pragma: no cover - the image ships sklearn
        from scipy.spatial import cKDTree

        t = cKDTree(xy.astype(np.float64))
        return [np.asarray(v, np.int64) for v in t.query_ball_point(xy.astype(np.float64), eps)], \
            "scipy.cKDTree"


def stdbscan_structure(coords, times, eps_space: float, eps_time: float, min_samples: int):
    """Labels of st_dbscan over a stacked frame set, computed the reference's way.
    Returns (labels int32 [n], index name)."""
    xy = np.ascontiguousarray(coords, dtype=np.float32)
    tf = np.ascontiguousarray(times, dtype=np.float32)
    n = len(xy)
    if n == 0:
        raise ValueError("Found array with 0 sample(s)")
    nbrs, index = _radius_neighbours(xy, eps_space)
    label = np.full(n, -1, dtype=np.int32)
    seen = np.zeros(n, dtype=bool)

    def near_in_time(i):  # per neighbour: two float32 scalar reads, a subtract, a compare
        return [j for j in nbrs[i] if abs(tf[j] - tf[i]) <= eps_time]

    cid = 0
    for i in range(n):
        if seen[i]:
            continue
        seen[i] = True
        first = near_in_time(i)
        if len(first) < min_samples:
            continue
        label[i] = cid
        pending = set(first)
        while pending:
            p = pending.pop()
            if not seen[p]:
                seen[p] = True
                more = near_in_time(p)
                if len(more) >= min_samples:
                    pending.update(more)
            if label[p] == -1:
                label[p] = cid
        cid += 1
    return label, index
