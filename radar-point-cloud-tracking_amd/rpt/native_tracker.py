"""Python handle on the C++ ObjectTracker of librpt (csrc/tracker.cpp), mirroring
ObjectTracker / TrackedObject of PointCloudWork/4_temporal_object_tracker.py:111-140, 543-688.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import numpy as np

from . import _abi

TYPE_NAMES = ("unknown", "buoy", "boat")


@dataclass
class TrackedObject:
    """4_temporal_object_tracker.py:111-140 — a snapshot of one tracked object."""

    object_id: int
    object_type: str
    positions: List[np.ndarray] = field(default_factory=list)
    frames_seen: List[int] = field(default_factory=list)
    last_seen_frame: int = 0
    velocities: List[np.ndarray] = field(default_factory=list)
    color: Tuple[int, int, int] = (180, 180, 180)
    _avg_velocity: float = 0.0

    @property
    def centroid(self) -> np.ndarray:
        return self.positions[-1] if self.positions else np.array([0, 0])

    @property
    def average_velocity(self):
        return self._avg_velocity


class NativeTracker:
    """Owns an rpt_tracker; update() has the reference's semantics (clusters in list order)."""

    def __init__(self, max_association_distance: float = 50.0, max_missed_frames: int = 10,
                 motion_history_frames: int = 5, stationary_velocity_threshold: float = 1.0):
        self._lib = _abi.load()
        p = _abi.TrackerParams(max_association_distance, max_missed_frames,
                               motion_history_frames, stationary_velocity_threshold)
        self._h = self._lib.rpt_tracker_new(_abi.C.byref(p))
        if not self._h:
            raise MemoryError("rpt_tracker_new failed")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.rpt_tracker_free(h)
            self._h = None

    def update_arrays(self, frame_id: int, cx: np.ndarray, cy: np.ndarray,
                      cluster_frame_ids: Sequence[int] | None = None) -> int:
        cx = np.ascontiguousarray(cx, dtype=np.float32)
        cy = np.ascontiguousarray(cy, dtype=np.float32)
        k = len(cx)
        cf = None
        if cluster_frame_ids is not None:
            cf = np.ascontiguousarray(cluster_frame_ids, dtype=np.int64)
        r = self._lib.rpt_tracker_update(
            self._h, int(frame_id), k, cx.ctypes.data_as(_abi.c_f32p),
            cy.ctypes.data_as(_abi.c_f32p),
            cf.ctypes.data_as(_abi.c_i64p) if cf is not None else None)
        if r < 0:
            _abi.check(-r, "rpt_tracker_update")
        return r

    def run(self, frame_ids: np.ndarray, offsets: np.ndarray, cx: np.ndarray, cy: np.ndarray
            ) -> int:
        frame_ids = np.ascontiguousarray(frame_ids, dtype=np.int64)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        cx = np.ascontiguousarray(cx, dtype=np.float32)
        cy = np.ascontiguousarray(cy, dtype=np.float32)
        r = self._lib.rpt_tracker_run(self._h, len(frame_ids),
                                      frame_ids.ctypes.data_as(_abi.c_i64p),
                                      offsets.ctypes.data_as(_abi.c_i64p),
                                      cx.ctypes.data_as(_abi.c_f32p),
                                      cy.ctypes.data_as(_abi.c_f32p))
        if r < 0:
            _abi.check(-r, "rpt_tracker_run")
        return r

    def __len__(self) -> int:
        return self._lib.rpt_tracker_num_objects(self._h)

    def objects(self) -> List[TrackedObject]:
        out = []
        info = _abi.ObjectInfo()
        for i in range(len(self)):
            _abi.check(self._lib.rpt_tracker_object_info(self._h, i, _abi.C.byref(info)))
            npos, nvel = info.n_positions, info.n_velocities
            px = np.empty(npos, np.float32)
            py = np.empty(npos, np.float32)
            fr = np.empty(npos, np.int64)
            vx = np.empty(nvel, np.float64)
            vy = np.empty(nvel, np.float64)
            _abi.check(self._lib.rpt_tracker_object_history(
                self._h, i, px.ctypes.data_as(_abi.c_f32p), py.ctypes.data_as(_abi.c_f32p),
                fr.ctypes.data_as(_abi.c_i64p), vx.ctypes.data_as(_abi.c_f64p),
                vy.ctypes.data_as(_abi.c_f64p)))
            vel = [np.array([0.0, 0.0])] + [np.array([vx[k], vy[k]], dtype=np.float32)
                                            for k in range(1, nvel)]
            av = (np.float32(info.average_velocity) if info.average_velocity_is_f32
                  else (np.float64(info.average_velocity) if nvel >= 2 else 0.0))
            out.append(TrackedObject(
                object_id=int(info.object_id), object_type=TYPE_NAMES[info.object_type],
                positions=[np.array([px[k], py[k]], dtype=np.float32) for k in range(npos)],
                frames_seen=[int(f) for f in fr], last_seen_frame=int(info.last_seen_frame),
                velocities=vel, color=tuple(int(c) for c in info.color), _avg_velocity=av))
        return out


def set_order(keys: Sequence[int]) -> List[int]:
    """CPython set iteration order of `keys` (first-occurrence order), -1 removed."""
    k = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.empty(max(len(k), 1), np.int32)
    m = _abi.load().rpt_set_order(k.ctypes.data_as(_abi.c_i32p), len(k),
                                  out.ctypes.data_as(_abi.c_i32p))
    return out[:m].tolist()


def lsap(cost: np.ndarray):
    """scipy.optimize.linear_sum_assignment (rectangular, minimise) on the host, in C++."""
    c = np.ascontiguousarray(cost, dtype=np.float64)
    if c.ndim != 2:
        raise ValueError("expected a matrix (2-D array)")
    nr, nc = c.shape
    k = min(nr, nc)
    a = np.empty(k, np.int64)
    b = np.empty(k, np.int64)
    st = _abi.load().rpt_lsap(c.ctypes.data_as(_abi.c_f64p), nr, nc,
                              a.ctypes.data_as(_abi.c_i64p), b.ctypes.data_as(_abi.c_i64p))
    _abi.check(st, "rpt_lsap")
    return a, b
