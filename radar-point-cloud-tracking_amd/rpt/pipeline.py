"""Device-resident per-frame path of PointCloudWork/4_temporal_object_tracker.py run_pipeline
(:941-991) over a stack of sweeps already in HBM:

  K1  polar scatter + threshold + stride + 3-gain fusion   build_frame / load_radar_csv  :312-352
  K2  occupancy grid + land mask (when > 10 frames)         :359-410, gate :954
  K3  land compaction                                        :413-436
  K4-K8 ST-DBSCAN over the stack                             :443-506
  K9  per-(frame, label) summaries                           :508-536
  host C++: cluster order (CPython set), Hungarian tracker   :519, :543-688, loop :984-991

Every arithmetic step runs in librpt (HIP kernels or host C++): the device stages are ONE native
call (rpt_stack_run, csrc/stack.cpp) whose size readbacks (file offsets, land bounds, kept count,
grid bounds, segment count) are pinned-memory syncs inside C++; torch provides the echo and the
stream.
"""
from __future__ import annotations

import queue
import time
from concurrent.futures import Future, ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _abi
from ._device import require_gpu, stream_handle
from .native_tracker import NativeTracker
from .stages import (LAND_GRID_RESOLUTION, LAND_MIN_INTENSITY, LAND_PERSISTENCE_THRESHOLD,
                     order_and_track)


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
    t_done: float = 0.0              # perf_counter when the device work and readbacks ended
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
                 host_workers: int = 2, lanes: int = 1, round_robin: bool = False,
                 k1_gate: bool = False):
        """async_host: the host stage (cluster order + tracker, sequential C++) of a run executes
        on a pool of host_workers threads while the caller goes on to the next runs' device
        work (runs are independent, so their host stages may overlap each other);
        StackResult.finish() waits for a run's host stage.

        lanes > 1: submit() runs successive stacks on `lanes` native handles, each on its own
        HIP stream, so one stack's kernels fill the GPU while another waits on a size readback
        or runs a latency-bound stage (the library keeps its scratch and look-back state per
        stream).  A run takes whichever lane is free when a worker thread picks it up: streams
        beyond the process's hardware queues share a queue and progress slower, and a fixed
        round-robin left the last runs of the slow lanes finishing long after the others
        (round_robin=True keeps that policy for comparisons).  k1_gate (lanes > 1): the lanes'
        K1 passes (HBM-bound) take turns, each behind the previous one on the device
        (rpt_k1_gate), so they never share the HBM and always overlap other lanes' latency-bound
        stages.  Measured: the steady state of a run 0-6 % faster from box to box, the 20-step
        bench line 4-19 % slower (the turns delay the first and last stacks of a batch), hence
        off by default (profiles/r6/ab_k1_gate/)."""
        self.dev = require_gpu(device)
        self.gains = [int(g) for g in gains]
        if sorted(self.gains) != self.gains:
            raise ValueError("gains must be in ascending order (build_frame iterates sorted gains)")
        self.rows, self.bins = rows, bins
        self.p = params or PathParams()
        self.lib = _abi.load()
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self._hs = [self.lib.rpt_stack_create() for _ in range(lanes)]
        self._h = self._hs[0]
        self._gate = self.lib.rpt_k1_gate_create() if lanes > 1 and k1_gate else None
        for h in self._hs if self._gate else []:
            _abi.check(self.lib.rpt_stack_set_k1_gate(h, self._gate), "rpt_stack_set_k1_gate")
        self._streams = [torch.cuda.Stream(self.dev) for _ in range(lanes)] if lanes > 1 else None
        self._lane_pool = ThreadPoolExecutor(max_workers=lanes) if lanes > 1 else None
        self._rr = [ThreadPoolExecutor(max_workers=1) for _ in range(lanes)] \
            if lanes > 1 and round_robin else None
        self._next_lane = 0
        self._free_lanes = queue.SimpleQueue()
        for k in range(lanes):
            self._free_lanes.put(k)
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

    def run(self, echo: torch.Tensor, keep_points: bool = False,
            keep_core: bool = False) -> StackResult:
        """K1 -> land filter -> ST-DBSCAN -> K9 in one native call (rpt_stack_run), then the
        host stage (cluster order + tracker) inline or on the worker pool (async_host).
        keep_points: hand back the clustered points and their labels (res.points, res.labels);
        keep_core: also K5's core flag of every such point (res.points["core"], the full-size
        invariant tests; one more kernel and sync)."""
        return self._run_lane(self._h, stream_handle(self.dev), echo, keep_points, keep_core)

    def submit(self, echo: torch.Tensor, keep_points: bool = False,
               keep_core: bool = False) -> Future:
        """Queues a run on the next lane and returns a Future of its StackResult (lanes == 1:
        runs inline).  The echo must stay unchanged until the future is done."""
        if self._lane_pool is None:
            f = Future()
            f.set_result(self.run(echo, keep_points, keep_core))
            return f
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.dev))  # the echo's producer
        if self._rr is not None:
            lane = self._next_lane
            self._next_lane = (lane + 1) % len(self._hs)
            s = self._streams[lane]
            s.wait_event(ready)
            return self._rr[lane].submit(self._run_lane, self._hs[lane], s.cuda_stream, echo,
                                         keep_points, keep_core)

        def task():
            lane = self._free_lanes.get()
            try:
                s = self._streams[lane]
                s.wait_event(ready)
                return self._run_lane(self._hs[lane], s.cuda_stream, echo, keep_points,
                                      keep_core)
            finally:
                self._free_lanes.put(lane)

        return self._lane_pool.submit(task)

    def _run_lane(self, h, stream: int, echo: torch.Tensor, keep_points: bool,
                  keep_core: bool = False) -> StackResult:
        # librpt allocates and records events on the calling thread's current HIP device; lane
        # threads (and callers whose current device differs) must run on the pipeline's
        with torch.cuda.device(self.dev):
            return self._run_lane_dev(h, stream, echo, keep_points, keep_core)

    def _run_lane_dev(self, h, stream: int, echo: torch.Tensor, keep_points: bool,
                      keep_core: bool) -> StackResult:
        p, lib = self.p, self.lib
        G = len(self.gains)
        F = echo.shape[0]
        dt = self._check(echo)
        echo = echo.contiguous()
        sp = _abi.StackParams(F, G, self.rows, self.bins, dt, float(np.float32(p.threshold)),
                              int(p.stride), 1 if p.land_filter else 0, LAND_GRID_RESOLUTION,
                              LAND_PERSISTENCE_THRESHOLD, float(LAND_MIN_INTENSITY),
                              float(p.eps_space), float(p.eps_time), int(p.min_samples),
                              1 if self.timing else 0)
        r = _abi.StackResult()
        scale_d, cos_d, sin_d = self.geo
        # per-point gains only when the points are handed back (nothing downstream reads them)
        _abi.check(lib.rpt_stack_run(h, _abi.C.byref(sp), echo.data_ptr(),
                                     scale_d.data_ptr(), cos_d.data_ptr(), sin_d.data_ptr(),
                                     self.gain_d.data_ptr() if keep_points else None,
                                     _abi.C.byref(r), stream),
                   "rpt_stack_run")
        fo = np.empty(F + 1, np.int64)
        _abi.check(lib.rpt_stack_frame_offsets(h, 0, fo.ctypes.data_as(_abi.c_i64p)))
        built = np.nonzero(np.diff(fo) > 0)[0]   # build_frame returns None if empty
        S = int(r.n_segments)
        seg = {"frame": np.empty(S, np.int32), "label": np.empty(S, np.int32),
               "count": np.empty(S, np.int64), "first": np.empty(S, np.int64),
               "cx": np.empty(S, np.float32), "cy": np.empty(S, np.float32),
               "mi": np.empty(S, np.float32)}
        first_noise = np.empty(F, np.int64)
        ptr = lambda a, t: a.ctypes.data_as(t)  # noqa: E731
        _abi.check(lib.rpt_stack_segments(
            h, ptr(seg["frame"], _abi.c_i32p), ptr(seg["label"], _abi.c_i32p),
            ptr(seg["count"], _abi.c_i64p), ptr(seg["first"], _abi.c_i64p),
            ptr(seg["cx"], _abi.c_f32p), ptr(seg["cy"], _abi.c_f32p), ptr(seg["mi"], _abi.c_f32p),
            ptr(first_noise, _abi.c_i64p)))
        stage_ms = {}
        if self.timing:
            d = r.dbscan
            stage_ms = {"polar": r.ms_polar, "land": r.ms_land, "stdbscan": r.ms_stdbscan,
                        "summaries": r.ms_summaries, "dbscan_grid": d.ms_grid,
                        "dbscan_core": d.ms_core, "dbscan_union": d.ms_union,
                        "dbscan_label": d.ms_label}
        self.last_stats = r.dbscan
        res = StackResult(n_points=int(r.n_points), n_clustered_input=int(r.n_clustered),
                          frame_ids=built, n_land_cells=int(r.n_land_cells),
                          n_clusters=int(r.n_clusters), n_segments=S, seg=seg,
                          frame_order_offsets=None, frame_order=None, tracker=None,
                          stage_ms=stage_ms, first_noise=first_noise,
                          t_done=time.perf_counter())

        def host_stage():
            t0 = time.perf_counter()
            fo_, order, trk = order_and_track(F, built, seg, first_noise, p)
            return fo_, order, trk, (time.perf_counter() - t0) * 1e3

        if self._host is not None:
            res._pending = self._host.submit(host_stage)
        else:
            fo_, order, trk, host_ms = host_stage()
            res.frame_order_offsets, res.frame_order, res.tracker = fo_, order, trk
            if self.timing:
                stage_ms["tracker_host"] = host_ms
        if keep_points:
            n = res.n_clustered_input
            pts = {k: torch.empty(n, dtype=dt_, device=self.dev) for k, dt_ in
                   (("x", torch.float32), ("y", torch.float32), ("v", torch.float32),
                    ("gain", torch.int32), ("frame", torch.int32))}
            labels = torch.empty(n, dtype=torch.int32, device=self.dev)
            if stream != stream_handle(self.dev):  # allocations above are on torch's stream
                torch.cuda.current_stream(self.dev).synchronize()
            _abi.check(lib.rpt_stack_points(h, pts["x"].data_ptr(), pts["y"].data_ptr(),
                                            pts["v"].data_ptr(), pts["gain"].data_ptr(),
                                            pts["frame"].data_ptr(), labels.data_ptr(), stream),
                       "rpt_stack_points")
            if n and keep_core:  # K5's core flags of the same points (invariant checks)
                pts["core"] = torch.empty(n, dtype=torch.uint8, device=self.dev)
                if stream != stream_handle(self.dev):
                    torch.cuda.current_stream(self.dev).synchronize()
                _abi.check(lib.rpt_stack_core_flags(h, pts["core"].data_ptr(), stream),
                           "rpt_stack_core_flags")
            if stream != stream_handle(self.dev):  # the caller reads them on torch's stream
                torch.cuda.ExternalStream(stream, device=self.dev).synchronize()
            res.labels, res.points = labels, pts
        return res

    def __del__(self):
        pools = [getattr(self, "_lane_pool", None)] + list(getattr(self, "_rr", None) or [])
        for pool in pools:
            if pool is not None:
                pool.shutdown(wait=True)
        for h in getattr(self, "_hs", None) or []:
            if h:
                self.lib.rpt_stack_destroy(h)
        self._hs, self._h = [], None
        if getattr(self, "_gate", None):  # after every handle attached to it
            self.lib.rpt_k1_gate_destroy(self._gate)
            self._gate = None
