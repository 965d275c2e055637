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
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _abi
from ._device import require_gpu, stream_handle
from .native_tracker import NativeTracker

LAND_GRID_RESOLUTION = 5.0        # 4_temporal_object_tracker.py:81
LAND_PERSISTENCE_THRESHOLD = 0.8  # :80
LAND_MIN_INTENSITY = 100          # :82


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
    frame_order_offsets: np.ndarray  # per built frame: its clusters in reference order
    frame_order: np.ndarray
    tracker: NativeTracker
    labels: Optional[torch.Tensor] = None
    points: Optional[Dict[str, torch.Tensor]] = None
    stage_ms: Dict[str, float] = field(default_factory=dict)


class _Ws:
    """Grow-only device buffers keyed by name (reused across runs: no per-step allocation)."""

    def __init__(self, dev):
        self.dev = dev
        self.bufs: Dict[str, torch.Tensor] = {}

    def get(self, name, n, dtype):
        b = self.bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = torch.empty(max(int(n * 1.1) + 64, 64), dtype=dtype, device=self.dev)
            self.bufs[name] = b
        return b[:n]


class FrameStackPipeline:
    """Runs the path over echo [n_frames][n_gains][rows][bins] (u8 or f32) in device memory."""

    def __init__(self, gains: Sequence[int], rows: int, bins: int, params: PathParams = None,
                 device=None, timing: bool = False):
        self.dev = require_gpu(device)
        self.gains = [int(g) for g in gains]
        if sorted(self.gains) != self.gains:
            raise ValueError("gains must be in ascending order (build_frame iterates sorted gains)")
        self.rows, self.bins = rows, bins
        self.p = params or PathParams()
        self.lib = _abi.load()
        self.ws = _Ws(self.dev)
        self.timing = timing
        self._geo_key = None

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
        self.scale_d, self.cos_d, self.sin_d = rep(scale), rep(cos_t), rep(sin_t)
        self.gain_d = torch.tensor(self.gains * (n_files // len(self.gains)), dtype=torch.int32,
                                   device=self.dev)
        self._geo_key = n_files

    def run(self, echo: torch.Tensor, keep_points: bool = False) -> StackResult:
        p, lib, ws = self.p, self.lib, self.ws
        G = len(self.gains)
        F = echo.shape[0]
        n_files = F * G
        if echo.shape[1:] != (G, self.rows, self.bins):
            raise ValueError(f"echo must be [frames][{G}][{self.rows}][{self.bins}]")
        if self._geo_key != n_files:
            raise ValueError("call set_geometry(...) for this number of files first")
        dt = {torch.uint8: _abi.ECHO_U8, torch.float32: _abi.ECHO_F32}.get(echo.dtype)
        if dt is None:
            raise TypeError("echo must be uint8 or float32")
        echo = echo.contiguous()
        st = stream_handle(self.dev)
        ev = []

        def mark(name):
            if self.timing:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                ev.append((name, e))
        mark("start")
        # ---- K1: count
        n_rows = n_files * self.rows
        row_prefix = ws.get("row_prefix", n_rows + 1, torch.int64)
        file_off = ws.get("file_off", n_files + 1, torch.int64)
        total = _abi.C.c_int64(0)
        _abi.check(lib.rpt_polar_count(echo.data_ptr(), dt, n_files, self.rows, self.bins,
                                       float(np.float32(p.threshold)), p.stride,
                                       row_prefix.data_ptr(), file_off.data_ptr(),
                                       _abi.C.byref(total), st), "rpt_polar_count")
        N = int(total.value)
        foff = file_off.cpu().numpy()
        frame_off = foff[::G].copy()                     # [F+1]
        counts = np.diff(frame_off)
        built = np.nonzero(counts > 0)[0]                # build_frame returns None for empty
        # ---- K1: write
        x = ws.get("x", N, torch.float32)
        y = ws.get("y", N, torch.float32)
        v = ws.get("v", N, torch.float32)
        g = ws.get("g", N, torch.int32)
        pf = ws.get("pf", N, torch.int32)
        _abi.check(lib.rpt_polar_write(echo.data_ptr(), dt, n_files, self.rows, self.bins,
                                       self.scale_d.data_ptr(), self.cos_d.data_ptr(),
                                       self.sin_d.data_ptr(), self.gain_d.data_ptr(),
                                       float(np.float32(p.threshold)), p.stride,
                                       row_prefix.data_ptr(), file_off.data_ptr(), G,
                                       x.data_ptr(), y.data_ptr(), v.data_ptr(), g.data_ptr(),
                                       pf.data_ptr(), st), "rpt_polar_write")
        mark("polar")
        n_land = 0
        xs, ys, vs, gs, pfs = x, y, v, g, pf
        n_in = N
        if p.land_filter and len(built) > 10 and N > 0:
            b4 = (_abi.C.c_float * 4)()
            _abi.check(lib.rpt_bounds_xy(x.data_ptr(), y.data_ptr(), N, b4, st), "rpt_bounds_xy")
            x0, x1, y0, y1 = (np.float32(b4[k]) for k in range(4))
            xe = np.arange(x0, x1 + LAND_GRID_RESOLUTION, LAND_GRID_RESOLUTION)
            ye = np.arange(y0, y1 + LAND_GRID_RESOLUTION, LAND_GRID_RESOLUTION)
            xe_d = torch.from_numpy(np.ascontiguousarray(xe, np.float64)).to(self.dev)
            ye_d = torch.from_numpy(np.ascontiguousarray(ye, np.float64)).to(self.dev)
            cells = (len(xe) - 1) * (len(ye) - 1)
            cnt = ws.get("land_cnt", cells, torch.int32)
            tot = ws.get("land_tot", cells, torch.float64)
            mask = ws.get("land_mask", cells, torch.uint8)
            _abi.check(lib.rpt_land_grid(x.data_ptr(), y.data_ptr(), v.data_ptr(), N,
                                         xe_d.data_ptr(), len(xe), ye_d.data_ptr(), len(ye),
                                         cnt.data_ptr(), tot.data_ptr(), st), "rpt_land_grid")
            nl = _abi.C.c_int64(0)
            _abi.check(lib.rpt_land_mask(cnt.data_ptr(), tot.data_ptr(), cells, len(built),
                                         LAND_PERSISTENCE_THRESHOLD, float(LAND_MIN_INTENSITY),
                                         mask.data_ptr(), _abi.C.byref(nl), st), "rpt_land_mask")
            n_land = int(nl.value)
            xs = ws.get("x2", N, torch.float32)
            ys = ws.get("y2", N, torch.float32)
            vs = ws.get("v2", N, torch.float32)
            gs = ws.get("g2", N, torch.int32)
            pfs = ws.get("pf2", N, torch.int32)
            fo_d = torch.from_numpy(frame_off.astype(np.int64)).to(self.dev)
            nfo = ws.get("new_frame_off", F + 1, torch.int64)
            kept = _abi.C.c_int64(0)
            _abi.check(lib.rpt_land_filter(x.data_ptr(), y.data_ptr(), v.data_ptr(), g.data_ptr(),
                                           pf.data_ptr(), N, fo_d.data_ptr(), F, xe_d.data_ptr(),
                                           len(xe), ye_d.data_ptr(), len(ye), mask.data_ptr(),
                                           xs.data_ptr(), ys.data_ptr(), vs.data_ptr(),
                                           gs.data_ptr(), pfs.data_ptr(), nfo.data_ptr(),
                                           _abi.C.byref(kept), st), "rpt_land_filter")
            n_in = int(kept.value)
            xs, ys, vs, gs, pfs = xs[:n_in], ys[:n_in], vs[:n_in], gs[:n_in], pfs[:n_in]
        mark("land")
        if n_in == 0:
            raise ValueError("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 "
                             "is required.")
        # ---- K4-K8: ST-DBSCAN over the stack (times = float32 frame id = frame slot)
        t = ws.get("t", n_in, torch.float32)
        _abi.check(lib.rpt_frame_times(pfs.data_ptr(), n_in, None, t.data_ptr(), st),
                   "rpt_frame_times")
        labels = ws.get("labels", n_in, torch.int32)
        sts = _abi.StdbscanStats()
        sts.timing = 1 if self.timing else 0
        _abi.check(lib.rpt_stdbscan(xs.data_ptr(), ys.data_ptr(), None, 1, t.data_ptr(), n_in,
                                    float(p.eps_space), float(p.eps_time), int(p.min_samples),
                                    labels.data_ptr(), _abi.C.byref(sts), st), "rpt_stdbscan")
        n_clusters = int(sts.n_clusters)
        mark("stdbscan")
        # ---- K9: summaries
        so = {k: ws.get("seg_" + k, n_in, dtp) for k, dtp in
              (("frame", torch.int32), ("label", torch.int32), ("count", torch.int64),
               ("first", torch.int64), ("cx", torch.float32), ("cy", torch.float32),
               ("mi", torch.float32))}
        ffn = ws.get("first_noise", F, torch.int64)
        nseg = _abi.C.c_int64(0)
        _abi.check(lib.rpt_cluster_summaries(
            labels.data_ptr(), xs.data_ptr(), ys.data_ptr(), vs.data_ptr(), pfs.data_ptr(), n_in,
            F, n_clusters, so["frame"].data_ptr(), so["label"].data_ptr(),
            so["count"].data_ptr(), so["first"].data_ptr(), so["cx"].data_ptr(),
            so["cy"].data_ptr(), so["mi"].data_ptr(), ffn.data_ptr(), _abi.C.byref(nseg), st),
            "rpt_cluster_summaries")
        S = int(nseg.value)
        seg = {k: t_[:S].cpu().numpy() for k, t_ in so.items()}
        first_noise = ffn.cpu().numpy()
        mark("summaries")
        # ---- host: per-frame order + tracker over the built frames
        t0 = time.perf_counter()
        fo = np.empty(F + 1, np.int64)
        order = np.empty(max(S, 1), np.int64)
        _abi.check(lib.rpt_order_clusters(
            F, S, seg["frame"].ctypes.data_as(_abi.c_i32p),
            seg["label"].ctypes.data_as(_abi.c_i32p), seg["first"].ctypes.data_as(_abi.c_i64p),
            first_noise.ctypes.data_as(_abi.c_i64p), fo.ctypes.data_as(_abi.c_i64p),
            order.ctypes.data_as(_abi.c_i64p)), "rpt_order_clusters")
        order = order[:S]
        trk = NativeTracker(p.max_association_distance, p.max_missed_frames,
                            p.motion_history_frames, p.stationary_velocity_threshold)
        # clusters of built frames, in reference order, concatenated
        sel = np.concatenate([order[fo[f]:fo[f + 1]] for f in built]) if len(built) else \
            np.zeros(0, np.int64)
        offs = np.zeros(len(built) + 1, np.int64)
        offs[1:] = np.cumsum(fo[built + 1] - fo[built])
        trk.run(built.astype(np.int64), offs, seg["cx"][sel], seg["cy"][sel])
        host_ms = (time.perf_counter() - t0) * 1e3
        stage_ms = {}
        if self.timing:
            torch.cuda.synchronize(self.dev)
            for (a, ea), (b, eb) in zip(ev[:-1], ev[1:]):
                stage_ms[b] = ea.elapsed_time(eb)
            stage_ms["tracker_host"] = host_ms
            stage_ms.update({"dbscan_grid": sts.ms_grid, "dbscan_core": sts.ms_core,
                             "dbscan_union": sts.ms_union, "dbscan_label": sts.ms_label})
        self.last_stats = sts
        res = StackResult(n_points=N, n_clustered_input=n_in, frame_ids=built,
                          n_land_cells=n_land, n_clusters=n_clusters, n_segments=S, seg=seg,
                          frame_order_offsets=fo, frame_order=order, tracker=trk,
                          stage_ms=stage_ms)
        if keep_points:
            res.labels = labels
            res.points = {"x": xs, "y": ys, "v": vs, "gain": gs, "frame": pfs}
        return res
