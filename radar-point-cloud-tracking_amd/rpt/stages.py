"""Per-device stages of the path as one object (``HipOps``), shared by the single-GPU pipeline
(rpt/pipeline.py) and the frame-sharded multi-GPU pipeline (rpt/dist.py).  Every method runs
librpt kernels on the current stream; tensors stay on the device.

The multi-GPU protocol only talks to these methods, which is what lets tests/test_dist_cpu.py run
the protocol with world_size 2 over gloo on CPU with a test-only implementation of the same
interface (tests/_cpu_ops.py).  The product has no CPU implementation.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from . import _abi
from ._device import stream_handle

LAND_GRID_RESOLUTION = 5.0        # 4_temporal_object_tracker.py:81
LAND_PERSISTENCE_THRESHOLD = 0.8  # :80
LAND_MIN_INTENSITY = 100          # :82


@dataclass
class Points:
    """SoA point set of a frame stack (device tensors) + per-frame offsets (host)."""

    x: torch.Tensor
    y: torch.Tensor
    v: torch.Tensor
    g: torch.Tensor
    pf: torch.Tensor               # frame slot (local frame index) per point
    frame_off: np.ndarray          # int64 [n_frames + 1]

    @property
    def n(self) -> int:
        return int(self.x.numel())

    def slice(self, a: int, b: int) -> "Points":
        off = np.clip(self.frame_off - a, 0, b - a)
        return Points(self.x[a:b], self.y[a:b], self.v[a:b], self.g[a:b], self.pf[a:b], off)


class _Ws:
    """Grow-only device buffers keyed by name (reused across runs)."""

    def __init__(self, dev):
        self.dev = dev
        self.bufs: Dict[str, torch.Tensor] = {}

    def get(self, name, n, dtype):
        b = self.bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = torch.empty(max(int(n * 1.1) + 64, 64), dtype=dtype, device=self.dev)
            self.bufs[name] = b
        return b[:n]


_NP_DT = {torch.int32: np.int32, torch.int64: np.int64, torch.float32: np.float32}


class HipOps:
    """librpt-backed stages for one device."""

    def __init__(self, dev: torch.device, timing: bool = False):
        self.dev = dev
        self.lib = _abi.load()
        self.ws = _Ws(dev)
        self._dbscan = None
        self.timing = timing          # hipEvents around rpt_dbscan_core (bench roofline)
        self._core_ev = None
        self.core_points = 0

    def st(self):
        return stream_handle(self.dev)

    # ---- K1
    def polar(self, echo, dt, rows, bins, geo, gain_d, threshold, stride, files_per_frame,
              prefix="") -> Points:
        lib, ws = self.lib, self.ws
        n_files = echo.shape[0] * echo.shape[1]
        n_rows = n_files * rows
        row_prefix = ws.get(prefix + "row_prefix", n_rows + 1, torch.int64)
        file_off = ws.get(prefix + "file_off", n_files + 1, torch.int64)
        thr = float(np.float32(threshold))
        _abi.check(lib.rpt_polar_count(echo.data_ptr(), dt, n_files, rows, bins, thr, stride,
                                       row_prefix.data_ptr(), file_off.data_ptr(), None,
                                       self.st()), "rpt_polar_count")
        foff = file_off.cpu().numpy()   # one readback: the offsets end with the total
        N = int(foff[-1])
        x = ws.get(prefix + "x", N, torch.float32)
        y = ws.get(prefix + "y", N, torch.float32)
        v = ws.get(prefix + "v", N, torch.float32)
        g = ws.get(prefix + "g", N, torch.int32)
        pf = ws.get(prefix + "pf", N, torch.int32)
        scale_d, cos_d, sin_d = geo
        _abi.check(lib.rpt_polar_write(echo.data_ptr(), dt, n_files, rows, bins,
                                       scale_d.data_ptr(), cos_d.data_ptr(), sin_d.data_ptr(),
                                       gain_d.data_ptr(), thr, stride, row_prefix.data_ptr(),
                                       file_off.data_ptr(), files_per_frame, x.data_ptr(),
                                       y.data_ptr(), v.data_ptr(), g.data_ptr(), pf.data_ptr(),
                                       self.st()), "rpt_polar_write")
        return Points(x, y, v, g, pf, foff[::files_per_frame].copy())

    # ---- K2/K3
    def bounds(self, pts: Points):
        b4 = (_abi.C.c_float * 4)()
        _abi.check(self.lib.rpt_bounds_xy(pts.x.data_ptr(), pts.y.data_ptr(), pts.n, b4,
                                          self.st()), "rpt_bounds_xy")
        return np.array([b4[0], b4[1], b4[2], b4[3]], np.float32)

    def land_grid(self, pts: Points, xe: np.ndarray, ye: np.ndarray):
        self._xe = torch.from_numpy(np.ascontiguousarray(xe, np.float64)).to(self.dev)
        self._ye = torch.from_numpy(np.ascontiguousarray(ye, np.float64)).to(self.dev)
        cells = (len(xe) - 1) * (len(ye) - 1)
        cnt = self.ws.get("land_cnt", cells, torch.int32)
        tot = self.ws.get("land_tot", cells, torch.float64)
        _abi.check(self.lib.rpt_land_grid(pts.x.data_ptr(), pts.y.data_ptr(), pts.v.data_ptr(),
                                          pts.n, self._xe.data_ptr(), len(xe),
                                          self._ye.data_ptr(), len(ye), cnt.data_ptr(),
                                          tot.data_ptr(), self.st()), "rpt_land_grid")
        return cnt, tot

    def land_apply(self, pts: Points, cnt, tot, num_frames: int, xe, ye,
                   want_land_cells: bool = False):
        """Land mask + compaction; the land-cell count (a readback) only when asked for."""
        cells = cnt.numel()
        mask = self.ws.get("land_mask", cells, torch.uint8)
        nl = _abi.C.c_int64(0)
        _abi.check(self.lib.rpt_land_mask(cnt.data_ptr(), tot.data_ptr(), cells, num_frames,
                                          LAND_PERSISTENCE_THRESHOLD, float(LAND_MIN_INTENSITY),
                                          mask.data_ptr(),
                                          _abi.C.byref(nl) if want_land_cells else None,
                                          self.st()), "rpt_land_mask")
        N, F = pts.n, len(pts.frame_off) - 1
        ws = self.ws
        out = [ws.get("x2", N, torch.float32), ws.get("y2", N, torch.float32),
               ws.get("v2", N, torch.float32), ws.get("g2", N, torch.int32),
               ws.get("pf2", N, torch.int32)]
        fo_d = torch.from_numpy(pts.frame_off.astype(np.int64)).to(self.dev)
        nfo = ws.get("new_frame_off", F + 1, torch.int64)
        _abi.check(self.lib.rpt_land_filter(
            pts.x.data_ptr(), pts.y.data_ptr(), pts.v.data_ptr(), pts.g.data_ptr(),
            pts.pf.data_ptr(), N, fo_d.data_ptr(), F, self._xe.data_ptr(), len(xe),
            self._ye.data_ptr(), len(ye), mask.data_ptr(), *[o.data_ptr() for o in out],
            nfo.data_ptr(), None, self.st()), "rpt_land_filter")
        nfo_h = nfo.cpu().numpy()        # one readback: the new offsets end with the kept count
        k = int(nfo_h[-1])
        return Points(*[o[:k] for o in out], nfo_h), int(nl.value)

    def frame_times(self, pts: Points, frame0: int, name="t") -> torch.Tensor:
        t = self.ws.get(name, pts.n, torch.float32)
        if frame0 == 0:
            _abi.check(self.lib.rpt_frame_times(pts.pf.data_ptr(), pts.n, None, t.data_ptr(),
                                                self.st()), "rpt_frame_times")
        else:
            F = len(pts.frame_off) - 1
            ids = torch.arange(frame0, frame0 + F, dtype=torch.int64, device=self.dev)
            _abi.check(self.lib.rpt_frame_times(pts.pf.data_ptr(), pts.n, ids.data_ptr(),
                                                t.data_ptr(), self.st()), "rpt_frame_times")
        return t

    # ---- K4-K8 fused (single device)
    def stdbscan(self, x, y, t, eps, eps_t, min_samples, timing=False):
        n = x.numel()
        labels = self.ws.get("labels", n, torch.int32)
        sts = _abi.StdbscanStats()
        sts.timing = 1 if timing else 0
        _abi.check(self.lib.rpt_stdbscan(x.data_ptr(), y.data_ptr(), None, 1, t.data_ptr(), n,
                                         float(eps), float(eps_t), int(min_samples),
                                         labels.data_ptr(), _abi.C.byref(sts), self.st()),
                   "rpt_stdbscan")
        return labels, sts

    # ---- K4-K8 phased (multi-GPU)
    def _state(self):
        if self._dbscan is None:
            self._dbscan = self.lib.rpt_dbscan_create()
        return self._dbscan

    def dbscan_core(self, x, y, t, eps, eps_t, min_samples) -> torch.Tensor:
        h = self._state()
        n = x.numel()
        _abi.check(self.lib.rpt_dbscan_build(h, x.data_ptr(), y.data_ptr(), None, 1,
                                             t.data_ptr(), n, float(eps), float(eps_t),
                                             int(min_samples), self.st()), "rpt_dbscan_build")
        core = self.ws.get("core", n, torch.uint8)
        if self.timing:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _abi.check(self.lib.rpt_dbscan_core(h, core.data_ptr(), self.st()), "rpt_dbscan_core")
        if self.timing:
            e1.record()
            self._core_ev = (e0, e1)
        self.core_points = n
        return core

    def last_core_ms(self) -> Optional[float]:
        """Duration of the last rpt_dbscan_core launch (timing=True; synchronises)."""
        if self._core_ev is None:
            return None
        self._core_ev[1].synchronize()
        return self._core_ev[0].elapsed_time(self._core_ev[1])

    def dbscan_components(self, core: torch.Tensor) -> torch.Tensor:
        h = self._state()
        _abi.check(self.lib.rpt_dbscan_set_core(h, core.data_ptr(), self.st()),
                   "rpt_dbscan_set_core")
        comp = self.ws.get("comp", core.numel(), torch.int32)
        _abi.check(self.lib.rpt_dbscan_components(h, comp.data_ptr(), self.st()),
                   "rpt_dbscan_components")
        return comp

    def remap(self, comp, base: int, keys: np.ndarray, vals: np.ndarray) -> torch.Tensor:
        n = comp.numel()
        rep = self.ws.get("rep", n, torch.int64)
        kd = torch.from_numpy(np.ascontiguousarray(keys, np.int64)).to(self.dev)
        vd = torch.from_numpy(np.ascontiguousarray(vals, np.int64)).to(self.dev)
        _abi.check(self.lib.rpt_remap_components(comp.data_ptr(), n, int(base), kd.data_ptr(),
                                                 vd.data_ptr(), len(keys), rep.data_ptr(),
                                                 self.st()), "rpt_remap_components")
        return rep

    def select_roots(self, rep, base: int, lo: int, hi: int) -> torch.Tensor:
        out = self.ws.get("roots", max(hi - lo, 1), torch.int64)
        cnt = _abi.C.c_int64(0)
        _abi.check(self.lib.rpt_select_roots(rep.data_ptr(), int(base), int(lo), int(hi),
                                             out.data_ptr(), _abi.C.byref(cnt), self.st()),
                   "rpt_select_roots")
        return out[:int(cnt.value)]

    def dbscan_labels_global(self, rep, reps_sorted: torch.Tensor) -> torch.Tensor:
        n = rep.numel()
        labels = self.ws.get("labels", n, torch.int32)
        reps = reps_sorted.to(self.dev).contiguous()
        _abi.check(self.lib.rpt_dbscan_labels_global(self._state(), rep.data_ptr(),
                                                     reps.data_ptr(), reps.numel(),
                                                     labels.data_ptr(), self.st()),
                   "rpt_dbscan_labels_global")
        return labels

    # ---- K9
    def summaries(self, pts: Points, labels, n_clusters: int):
        n, F = pts.n, len(pts.frame_off) - 1
        so = {k: self.ws.get("seg_" + k, max(n, 1), dt) for k, dt in
              (("frame", torch.int32), ("label", torch.int32), ("count", torch.int64),
               ("first", torch.int64), ("cx", torch.float32), ("cy", torch.float32),
               ("mi", torch.float32))}
        ffn = self.ws.get("first_noise", max(F, 1), torch.int64)
        nseg = _abi.C.c_int64(0)
        _abi.check(self.lib.rpt_cluster_summaries(
            labels.data_ptr(), pts.x.data_ptr(), pts.y.data_ptr(), pts.v.data_ptr(),
            pts.pf.data_ptr(), n, F, n_clusters, so["frame"].data_ptr(), so["label"].data_ptr(),
            so["count"].data_ptr(), so["first"].data_ptr(), so["cx"].data_ptr(),
            so["cy"].data_ptr(), so["mi"].data_ptr(), ffn.data_ptr(), _abi.C.byref(nseg),
            self.st()), "rpt_cluster_summaries")
        S = int(nseg.value)
        # one readback: the arrays packed on the device as float64 (exact for every field)
        keys = list(so)
        flat = torch.cat([so[k][:S].to(torch.float64) for k in keys] +
                         [ffn[:F].to(torch.float64)]).cpu().numpy()
        seg = {k: flat[i * S:(i + 1) * S].astype(_NP_DT[so[k].dtype])
               for i, k in enumerate(keys)}
        return seg, flat[len(keys) * S:].astype(np.int64)

    def close(self):
        if self._dbscan is not None:
            self.lib.rpt_dbscan_destroy(self._dbscan)
            self._dbscan = None


def order_frames(n_frames: int, seg: Dict[str, np.ndarray], first_noise: np.ndarray):
    """Host: per frame slot, its segments in the reference's cluster order (CPython set
    iteration of the frame's labels, 4_temporal_object_tracker.py:519-522) -> (offsets
    [n_frames + 1], order = indices into seg)."""
    lib = _abi.load()
    S = len(seg["frame"])
    fo = np.empty(n_frames + 1, np.int64)
    order = np.empty(max(S, 1), np.int64)
    _abi.check(lib.rpt_order_clusters(
        n_frames, S, np.ascontiguousarray(seg["frame"], np.int32).ctypes.data_as(_abi.c_i32p),
        np.ascontiguousarray(seg["label"], np.int32).ctypes.data_as(_abi.c_i32p),
        np.ascontiguousarray(seg["first"], np.int64).ctypes.data_as(_abi.c_i64p),
        np.ascontiguousarray(first_noise, np.int64).ctypes.data_as(_abi.c_i64p),
        fo.ctypes.data_as(_abi.c_i64p), order.ctypes.data_as(_abi.c_i64p)),
        "rpt_order_clusters")
    return fo, order[:S]


def track_ordered(slots: np.ndarray, fo: np.ndarray, order: np.ndarray,
                  seg: Dict[str, np.ndarray], params, frame_ids: Optional[np.ndarray] = None):
    """Host: the C++ tracker over the built frame slots (ascending), each frame's clusters in
    the order given by (fo, order); frame_ids[k] is the frame id of slots[k] (default: the
    slot)."""
    from .native_tracker import NativeTracker

    trk = NativeTracker(params.max_association_distance, params.max_missed_frames,
                        params.motion_history_frames, params.stationary_velocity_threshold)
    slots = np.asarray(slots, np.int64)
    if len(slots):
        cnts = fo[slots + 1] - fo[slots]
        starts = fo[slots]
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(cnts)[:-1]]), cnts) + \
            np.arange(int(cnts.sum()))
        sel = order[idx]
        offs = np.concatenate([[0], np.cumsum(cnts)]).astype(np.int64)
    else:
        sel = np.zeros(0, np.int64)
        offs = np.zeros(1, np.int64)
    ids = slots if frame_ids is None else np.asarray(frame_ids, np.int64)
    trk.run(ids, offs, seg["cx"][sel], seg["cy"][sel])
    return trk


def order_and_track(n_frames: int, built: np.ndarray, seg: Dict[str, np.ndarray],
                    first_noise: np.ndarray, params, frame_ids: Optional[np.ndarray] = None):
    """Host: per-frame reference cluster order (CPython set emulation) + the C++ tracker over the
    built frames, in one native call (rpt_order_and_track: frames ordered on a second thread
    ahead of the tracker).  frame_ids[f] is the frame id of slot f (default: the slot)."""
    from .native_tracker import NativeTracker

    lib = _abi.load()
    trk = NativeTracker(params.max_association_distance, params.max_missed_frames,
                        params.motion_history_frames, params.stationary_velocity_threshold)
    S = len(seg["frame"])
    fo = np.empty(n_frames + 1, np.int64)
    order = np.empty(max(S, 1), np.int64)
    built = np.ascontiguousarray(built, np.int64)
    ids = None if frame_ids is None else np.ascontiguousarray(frame_ids, np.int64)
    if ids is not None and len(ids) < n_frames:
        raise ValueError("frame_ids needs one id per frame slot")
    a32 = lambda k: np.ascontiguousarray(seg[k], np.int32).ctypes.data_as(_abi.c_i32p)  # noqa: E731
    af = lambda k: np.ascontiguousarray(seg[k], np.float32).ctypes.data_as(_abi.c_f32p)  # noqa: E731
    _abi.check(lib.rpt_order_and_track(
        n_frames, S, a32("frame"), a32("label"),
        np.ascontiguousarray(seg["first"], np.int64).ctypes.data_as(_abi.c_i64p),
        np.ascontiguousarray(first_noise, np.int64).ctypes.data_as(_abi.c_i64p),
        af("cx"), af("cy"), len(built), built.ctypes.data_as(_abi.c_i64p),
        ids.ctypes.data_as(_abi.c_i64p) if ids is not None else None, trk._h,
        fo.ctypes.data_as(_abi.c_i64p), order.ctypes.data_as(_abi.c_i64p)),
        "rpt_order_and_track")
    return fo, order[:S], trk
