"""TEST INFRASTRUCTURE ONLY — restatement of ObjectTracker / TrackedObject of
PointCloudWork/4_temporal_object_tracker.py:111-140, 543-688 with the reference's exact numpy
dtype flow (float64 while the initial float64 zero velocity is inside the 5-entry window,
float32 afterwards), scipy's linear_sum_assignment for association.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
from scipy.optimize import linear_sum_assignment

MAX_ASSOCIATION_DISTANCE = 50.0   # :89
MAX_MISSED_FRAMES = 10            # :90
MOTION_HISTORY_FRAMES = 5         # :86
STATIONARY_VELOCITY_THRESHOLD = 1.0  # :85


class Obj:
    __slots__ = ("object_id", "object_type", "positions", "frames_seen", "last_seen_frame",
                 "velocities", "color")

    def __init__(self, oid, centroid, frame_id, color):
        self.object_id = oid
        self.object_type = "unknown"
        self.positions = [np.array(centroid, copy=True)]
        self.frames_seen = [frame_id]
        self.last_seen_frame = frame_id
        self.velocities = [np.array([0.0, 0.0])]       # float64 zero (:619)
        self.color = color

    @property
    def centroid(self):
        return self.positions[-1]

    @property
    def average_velocity(self):                        # :127-133
        if len(self.velocities) < 2:
            return 0.0
        window = self.velocities[-MOTION_HISTORY_FRAMES:]
        return np.mean([np.linalg.norm(v) for v in window])

    def predict(self, ahead: int):                     # :135-140
        if not self.velocities:
            return self.centroid
        mean_v = np.mean(self.velocities[-MOTION_HISTORY_FRAMES:], axis=0)
        return self.centroid + mean_v * ahead


def golden_color(oid: int) -> Tuple[int, int, int]:     # :666-688
    h = (oid * 0.618033988749895) % 1.0
    k = int(h * 6)
    f = h * 6 - k
    q = 1 - f
    rgb = [(1, f, 0), (q, 1, 0), (0, 1, f), (0, q, 1), (f, 0, 1)]
    r, g, b = rgb[k] if k < 5 else (1, 0, q)
    return int(r * 255), int(g * 255), int(b * 255)


class Tracker:
    """update(clusters, frame_id) with clusters = [(centroid f32[2], cluster_frame_id), ...]."""

    def __init__(self):
        self.objects: dict = {}
        self.next_id = 1
        self.current_frame = 0

    def _new(self, centroid, fid):
        o = Obj(self.next_id, centroid, fid, golden_color(self.next_id))
        self.objects[self.next_id] = o
        self.next_id += 1

    def _drop_lost(self):
        for oid in [k for k, o in self.objects.items()
                    if self.current_frame - o.last_seen_frame > MAX_MISSED_FRAMES]:
            del self.objects[oid]
        return list(self.objects.values())

    def update(self, clusters: List[tuple], frame_id: int):
        self.current_frame = frame_id
        if not clusters:
            return self._drop_lost()
        if not self.objects:
            for c, fid in clusters:
                self._new(c, fid)
            return list(self.objects.values())
        live = [o for o in self.objects.values()
                if frame_id - o.last_seen_frame <= MAX_MISSED_FRAMES]
        if not live:
            for c, fid in clusters:
                self._new(c, fid)
            return list(self.objects.values())
        cost = np.zeros((len(clusters), len(live)))
        for j, o in enumerate(live):
            for i, (c, _) in enumerate(clusters):
                cost[i, j] = np.linalg.norm(c - o.predict(frame_id - o.last_seen_frame))
        rows, cols = linear_sum_assignment(cost)
        taken = set()
        for i, j in zip(rows, cols):
            if cost[i, j] <= MAX_ASSOCIATION_DISTANCE:
                o = live[j]
                c = clusters[i][0]
                gap = frame_id - o.last_seen_frame
                if gap > 0:
                    o.velocities.append((c - o.positions[-1]) / gap)
                o.positions.append(np.array(c, copy=True))
                o.frames_seen.append(frame_id)
                o.last_seen_frame = frame_id
                if len(o.velocities) < MOTION_HISTORY_FRAMES:
                    o.object_type = "unknown"
                else:
                    o.object_type = ("buoy" if o.average_velocity < STATIONARY_VELOCITY_THRESHOLD
                                     else "boat")
                taken.add(i)
        for i, (c, fid) in enumerate(clusters):
            if i not in taken:
                self._new(c, fid)
        return self._drop_lost()
