"""Device-resident per-frame path of PointCloudWork/4_temporal_object_tracker.py run_pipeline
(:941-991) over a stack of sweeps already in HBM:

  K1  polar scatter + threshold + stride + 3-gain fusion   build_frame / load_radar_csv  :312-352
  K2  occupancy grid + land mask (when > 10 frames)         :359-410, gate :954
  K3  land compaction                                        :413-436
  K4-K8 ST-DBSCAN over the stack                             :443-506
  K9  per-(frame, label) summaries                           :508-536
  host C++: cluster order (CPython set), Hungarian tracker   :519, :543-688, loop :984-991

Every arithmetic step runs in librpt (HIP kernels or host C++); torch provides the buffers and
the stream.  Host syncs per run: file offsets, grid bounds (x2), kept count, segment count.
"""
from __future__ import annotations

import time
from concurrent.futures import Future, ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _abi
from ._device import require_gpu
from .native_tracker import NativeTracker
from .stages import LAND_GRID_RESOLUTION, HipOps, order_and_track


@dataclass
class PathParams:
    eps_space: float = 8.0     # :75
    eps_time: float = 2.0      # :76
    min_samples: int = 15      # :77
    threshold: float = 10.0    # :70 (INTENSITY_THRESHOLD; the --intensity-threshold flag is unused)
    stride: int = 4            # :71
    land_filter: bool = True   # not --no-land-filter
    max_association_distance: float = 50.0
    max_missed_frames: int = 10
    motion_history_frames: int = 5
    stationary_velocity_threshold: float = 1.0


@dataclass
class StackResult:
    n_points: int                    # "Total points" (:950-951), before the land filter
    n_clustered_input: int           # points entering ST-DBSCAN
    frame_ids: np.ndarray            # built (non-empty) frames, in order
    n_land_cells: int
    n_clusters: int
    n_segments: int
    seg: Dict[str, np.ndarray]       # per (frame, label) summaries, host copies
    frame_order_offsets: Optional[np.ndarray]  # per frame slot: its clusters in reference order
    frame_order: Optional[np.ndarray]
    tracker: Optional[NativeTracker]
    first_noise: Optional[np.ndarray] = None  # per frame slot: first noise point or -1
    labels: Optional[torch.Tensor] = None
    points: Optional[Dict[str, torch.Tensor]] = None
    stage_ms: Dict[str, float] = field(default_factory=dict)
    _pending: Optional[Future] = None

    def finish(self) -> "StackResult":
        """Wait for the host stage (cluster order + tracker) when it runs asynchronously."""
        if self._pending is not None:
            fo, order, trk, host_ms = self._pending.result()
            self.frame_order_offsets, self.frame_order, self.tracker = fo, order, trk
            if self.stage_ms is not None and "polar" in self.stage_ms:
                self.stage_ms["tracker_host"] = host_ms
            self._pending = None
        return self


class FrameStackPipeline:
    """Runs the path over echo [n_frames][n_gains][rows][bins] (u8 or f32) in device memory."""

    def __init__(self, gains: Sequence[int], rows: int, bins: int, params: PathParams = None,
                 device=None, timing: bool = False, async_host: bool = False,
                 host_workers: int = 2):
        """async_host: the host stage (cluster order + tracker, sequential C++) of a run executes
        on a pool of host_workers threads while the caller goes on to the next runs' device
        work (runs are independent, so their host stages may overlap each other);
        StackResult.finish() waits for a run's host stage."""
        self.dev = require_gpu(device)
        self.gains = [int(g) for g in gains]
        if sorted(self.gains) != self.gains:
            raise ValueError("gains must be in ascending order (build_frame iterates sorted gains)")
        self.rows, self.bins = rows, bins
        self.p = params or PathParams()
        self.ops = HipOps(self.dev)
        self.timing = timing
        self._host = ThreadPoolExecutor(max_workers=host_workers) if async_host else None
        self._geo_key = None
        self.last_stats = None

    # -- per-row geometry repeated over files (Scale/Angle columns of every CSV) --
    def set_geometry(self, scale: np.ndarray, cos_t: np.ndarray, sin_t: np.ndarray,
                     n_files: int):
        """scale/cos_t/sin_t: float32 [rows] shared by all files, or [n_files*rows]."""
        def rep(a):
            a = np.ascontiguousarray(a, dtype=np.float32)
            if a.size == self.rows:
                a = np.tile(a, n_files)
            if a.size != n_files * self.rows:
                raise ValueError("geometry arrays must have rows or n_files*rows entries")
            return torch.from_numpy(a).to(self.dev)
        self.geo = (rep(scale), rep(cos_t), rep(sin_t))
        self.gain_d = torch.tensor(self.gains * (n_files // len(self.gains)), dtype=torch.int32,
                                   device=self.dev)
        self._geo_key = n_files

    def _check(self, echo):
        G = len(self.gains)
        if echo.shape[1:] != (G, self.rows, self.bins):
            raise ValueError(f"echo must be [frames][{G}][{self.rows}][{self.bins}]")
        if self._geo_key != echo.shape[0] * G:
            raise ValueError("call set_geometry(...) for this number of files first")
        dt = {torch.uint8: _abi.ECHO_U8, torch.float32: _abi.ECHO_F32}.get(echo.dtype)
        if dt is None:
            raise TypeError("echo must be uint8 or float32")
        return dt

    def run(self, echo: torch.Tensor, keep_points: bool = False) -> StackResult:
        p, ops = self.p, self.ops
        G = len(self.gains)
        F = echo.shape[0]
        dt = self._check(echo)
        echo = echo.contiguous()
        ev = []

        def mark(name):
            if self.timing:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                ev.append((name, e))
        mark("start")
        pts = ops.polar(echo, dt, self.rows, self.bins, self.geo, self.gain_d, p.threshold,
                        p.stride, G)
        N = pts.n
        built = np.nonzero(np.diff(pts.frame_off) > 0)[0]   # build_frame returns None if empty
        mark("polar")
        n_land = 0
        if p.land_filter and len(built) > 10 and N > 0:
            x0, x1, y0, y1 = ops.bounds(pts)
            xe = np.arange(x0, x1 + LAND_GRID_RESOLUTION, LAND_GRID_RESOLUTION)
            ye = np.arange(y0, y1 + LAND_GRID_RESOLUTION, LAND_GRID_RESOLUTION)
            cnt, tot = ops.land_grid(pts, xe, ye)
            pts, n_land = ops.land_apply(pts, cnt, tot, len(built), xe, ye)
        mark("land")
        n_in = pts.n
        if n_in == 0:
            raise ValueError("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 "
                             "is required.")
        t = ops.frame_times(pts, 0)
        labels, sts = ops.stdbscan(pts.x, pts.y, t, p.eps_space, p.eps_time, p.min_samples,
                                   timing=self.timing)
        n_clusters = int(sts.n_clusters)
        mark("stdbscan")
        seg, first_noise = ops.summaries(pts, labels, n_clusters)
        mark("summaries")

        def host_stage():
            t0 = time.perf_counter()
            fo, order, trk = order_and_track(F, built, seg, first_noise, p)
            return fo, order, trk, (time.perf_counter() - t0) * 1e3

        stage_ms = {}
        if self.timing:
            torch.cuda.synchronize(self.dev)
            for (a, ea), (b, eb) in zip(ev[:-1], ev[1:]):
                stage_ms[b] = ea.elapsed_time(eb)
            stage_ms.update({"dbscan_grid": sts.ms_grid, "dbscan_core": sts.ms_core,
                             "dbscan_union": sts.ms_union, "dbscan_label": sts.ms_label})
        self.last_stats = sts
        res = StackResult(n_points=N, n_clustered_input=n_in, frame_ids=built,
                          n_land_cells=n_land, n_clusters=n_clusters, n_segments=len(seg["frame"]),
                          seg=seg, frame_order_offsets=None, frame_order=None, tracker=None,
                          stage_ms=stage_ms, first_noise=first_noise)
        if self._host is not None:
            res._pending = self._host.submit(host_stage)
        else:
            fo, order, trk, host_ms = host_stage()
            res.frame_order_offsets, res.frame_order, res.tracker = fo, order, trk
            if self.timing:
                stage_ms["tracker_host"] = host_ms
        if keep_points:
            res.labels = labels
            res.points = {"x": pts.x, "y": pts.y, "v": pts.v, "gain": pts.g, "frame": pts.pf}
        return res
