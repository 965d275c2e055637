"""TEST INFRASTRUCTURE ONLY — numpy restatement of the per-frame path of
PointCloudWork/4_temporal_object_tracker.py (reference), used as the parity checker.

Every function keeps the reference's dtype flow (float32 geometry, float64 grid edges, numpy
reduction orders) because the device path is held to bit-identical results.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

ANGLE_SCALE = 360.0 / 8196.0          # :66
INTENSITY_THRESHOLD = 10.0             # :70
POINT_STRIDE = 4                       # :71
LAND_PERSISTENCE_THRESHOLD = 0.8       # :80
LAND_GRID_RESOLUTION = 5.0             # :81
LAND_MIN_INTENSITY = 100               # :82


def trig_tables(angle_col) -> Tuple[np.ndarray, np.ndarray]:
    """Per-row float32 cos/sin exactly as :203, :217-218 evaluate them (numpy float32 SIMD
    cos/sin of deg2rad(Angle * ANGLE_SCALE), Python float weak-promoted to float32)."""
    a = np.deg2rad(np.asarray(angle_col).astype(np.float32) * ANGLE_SCALE)
    return np.cos(a[:, None])[:, 0].copy(), np.sin(a[:, None])[:, 0].copy()


def polar_scatter(echo, scale, cos_t, sin_t, threshold: float = INTENSITY_THRESHOLD,
                  stride: int = POINT_STRIDE):
    """:206-232 on an in-memory sweep: echo [rows][bins] (float32 values), scale [rows]."""
    e = np.asarray(echo).astype(np.float32)
    bins = e.shape[1]
    step = np.asarray(scale, dtype=np.float32)[:, None] / bins           # :213
    rng = step * np.arange(bins, dtype=np.float32)                        # :214
    x = rng * np.asarray(cos_t, dtype=np.float32)[:, None]                # :217
    y = rng * np.asarray(sin_t, dtype=np.float32)[:, None]                # :218
    keep = e > threshold                                                  # :221
    xs, ys, vs = x[keep], y[keep], e[keep]
    if stride > 1:                                                        # :227-230
        xs, ys, vs = xs[::stride], ys[::stride], vs[::stride]
    return xs, ys, vs


def build_frames(per_frame: Sequence[Dict[int, Tuple[np.ndarray, np.ndarray, np.ndarray]]]):
    """build_frame :312-352: concatenate per-gain points in ascending gain order; a frame whose
    gains are all empty is dropped (frame ids keep the gap).  Returns list of
    (frame_id, points f32 [n,3], gains i32 [n])."""
    out = []
    for fid, gains in enumerate(per_frame):
        xs, ys, vs, gs = [], [], [], []
        for g in sorted(gains):
            x, y, v = gains[g]
            if len(x) == 0:
                continue
            xs.append(x); ys.append(y); vs.append(v)
            gs.append(np.full(len(x), g, dtype=np.int32))
        if not xs:
            continue
        pts = np.column_stack([np.concatenate(xs), np.concatenate(ys), np.concatenate(vs)])
        out.append((fid, pts, np.concatenate(gs)))
    return out


def _digitize_clip(v, edges, hi):
    return np.clip(np.digitize(v, edges) - 1, 0, hi)


def land_filter(frames, resolution: float = LAND_GRID_RESOLUTION,
                persistence: float = LAND_PERSISTENCE_THRESHOLD,
                min_intensity: float = LAND_MIN_INTENSITY):
    """build_occupancy_grid :359-391 + identify_land_cells :394-410 + filter_land_from_frame
    :413-436.  Returns (filtered frames, count grid, intensity grid, land mask, (xe, ye))."""
    ax = np.concatenate([p[:, 0] for _, p, _ in frames])
    ay = np.concatenate([p[:, 1] for _, p, _ in frames])
    x0, x1 = ax.min(), ax.max()
    y0, y1 = ay.min(), ay.max()
    xe = np.arange(x0, x1 + resolution, resolution)
    ye = np.arange(y0, y1 + resolution, resolution)
    cnt = np.zeros((len(xe) - 1, len(ye) - 1), dtype=np.int32)
    tot = np.zeros((len(xe) - 1, len(ye) - 1), dtype=np.float64)
    for _, p, _ in frames:
        ix = _digitize_clip(p[:, 0], xe, len(xe) - 2)
        iy = _digitize_clip(p[:, 1], ye, len(ye) - 2)
        np.add.at(cnt, (ix, iy), 1)
        np.add.at(tot, (ix, iy), p[:, 2])
    frac = cnt / max(len(frames), 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        mean_i = np.where(cnt > 0, tot / cnt, 0)
    land = (frac >= persistence) & (mean_i >= min_intensity)
    out = []
    for fid, p, g in frames:
        ix = _digitize_clip(p[:, 0], xe, land.shape[0] - 1)
        iy = _digitize_clip(p[:, 1], ye, land.shape[1] - 1)
        keep = ~land[ix, iy]
        out.append((fid, p[keep], g[keep]))
    return out, cnt, tot, land, (xe, ye)


def frame_clusters(frames, labels):
    """:508-536 — per frame, the clusters in the order CPython iterates set(frame_labels) minus
    -1; centroid = np.mean(pts, axis=0) (sequential float32), mean_intensity = float(np.mean(I)).
    Returns {frame_id: [(label, num_points, centroid f32[2], mean_intensity float)]}."""
    res: Dict[int, list] = {}
    off = 0
    for fid, p, _ in frames:
        n = p.shape[0]
        lab = labels[off:off + n]
        xy = p[:, :2]
        ii = p[:, 2]
        order = set(lab)
        order.discard(-1)
        for lbl in order:
            m = lab == lbl
            c = np.mean(xy[m], axis=0)
            res.setdefault(fid, []).append((int(lbl), int(m.sum()), c, float(np.mean(ii[m]))))
        off += n
    return res


def stack_coords(frames):
    """:453-467: stacked xy float32 and frame ids float32."""
    xy = np.vstack([p[:, :2] for _, p, _ in frames]) if frames else np.zeros((0, 2), np.float32)
    t = np.concatenate([np.full(p.shape[0], fid, dtype=np.float32) for fid, p, _ in frames]) \
        if frames else np.zeros(0, np.float32)
    return xy, t


def run_path(frames, eps_space=8.0, eps_time=2.0, min_samples=15, land=True, dbscan=None):
    """Stage order of run_pipeline :941-991 after frame building: land filter when more than 10
    frames, ST-DBSCAN over the stack, per-frame clusters, tracker over every frame.
    dbscan: the labelling function (default the BFS ``stdbscan``; ``stdbscan_uf`` for stacks of
    millions of points)."""
    from . import stdbscan
    from .tracker import Tracker

    if land and len(frames) > 10:
        frames = land_filter(frames)[0]
    xy, t = stack_coords(frames)
    labels = (dbscan or stdbscan)(xy, t, eps_space, eps_time, min_samples)
    clusters = frame_clusters(frames, labels)
    trk = Tracker()
    for fid, _, _ in frames:
        trk.update([(c[2], fid) for c in clusters.get(fid, [])], fid)
    return frames, labels, clusters, trk
