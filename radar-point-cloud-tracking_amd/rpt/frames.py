"""Frame stacks from radar CSV files: the grouped files of run_pipeline
(PointCloudWork/4_temporal_object_tracker.py:929-947) as ONE device echo tensor
[frame][gain][row][bin] for rpt_stack_run.

* Gains are the sorted union over the stack (build_frame iterates sorted(frame_files), :324); a
  frame that lacks a gain gets an all-zero sweep there, which keeps no point — the same fusion
  as build_frame skipping it.
* Rows: the longest file; shorter files are zero past their end (no point), and their per-row
  geometry there is never read for a kept sample.
* Files parse natively (rpt.core.ingest, multithreaded, u8 when every sample is an integer in
  0..255); unreadable files and files without rows are empty sweeps, like load_radar_csv's
  except / df.empty branches (:193-201).
* cos/sin tables: numpy float32 cos/sin of each FILE's own Angle column, shaped [rows, 1] as the
  reference evaluates them (:203, :217-218) -- the device path takes them as inputs.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .core.ingest import GAIN_FIRST_NAN, STATUS_NON_NUMERIC, STATUS_OK, read_sweeps
from .core.transforms import trig_tables


@dataclass
class FrameStackInput:
    echo: torch.Tensor           # device [F][G][R][bins], uint8 or float32
    gains: List[int]             # ascending
    rows: int
    scale: np.ndarray            # float32 [F*G*R]
    cos_t: np.ndarray
    sin_t: np.ndarray
    file_status: Dict[Path, int]  # per parsed file: rpt.core.ingest STATUS_*


def load_frame_stack(frame_files: Sequence[Dict[int, Path]], device, bins: int = 1024,
                     threads: int = 0, on_error=None) -> FrameStackInput:
    """on_error(path, message): called, in frame order, for each file the reference's read_csv
    would reject, with the text of read_csv's exception (the reference prints
    f"Error loading {path}: {e}" and uses an empty sweep, :191-195).  A data file whose first
    Gain value is missing raises ValueError like the reference's int(df["Gain"].iloc[0]) (:200)."""
    gains = sorted({g for ff in frame_files for g in ff})
    F, G = len(frame_files), len(gains)
    slots, paths = [], []
    for f, ff in enumerate(frame_files):
        for k, g in enumerate(gains):
            if g in ff:
                slots.append(f * G + k)
                paths.append(Path(ff[g]))
    batch = read_sweeps(paths, bins=bins, threads=threads)
    for j, p in enumerate(paths):  # the first file (in the reference's load order) that raises
        st = int(batch.status[j])
        if st == STATUS_OK and batch.rows[j] > 0 and batch.gain_flags[j] & GAIN_FIRST_NAN:
            # int(df["Gain"].iloc[0]) of a NaN (uncaught, :200)
            raise ValueError(f"cannot convert float NaN to integer ({p})")
        if st == STATUS_NON_NUMERIC:
            # the reference's to_numpy(np.float32) raises on a non-numeric column (uncaught, :207)
            raise ValueError(f"could not convert string to float in {p}")
    R = max(int(batch.echo.shape[1]), 1)
    dt = torch.uint8 if batch.echo.dtype == np.uint8 else torch.float32
    echo = torch.zeros((F * G, R, bins), dtype=dt, device=device)
    scale = np.zeros((F * G, R), np.float32)
    cos_t = np.zeros((F * G, R), np.float32)
    sin_t = np.zeros((F * G, R), np.float32)
    if paths and batch.echo.shape[1] > 0:
        idx = torch.tensor(slots, dtype=torch.int64, device=device)
        echo.index_copy_(0, idx, torch.from_numpy(batch.echo).to(device))
    for j, (s, p) in enumerate(zip(slots, paths)):
        st = int(batch.status[j])
        if batch.errors[j] is not None and on_error is not None:
            on_error(p, batch.errors[j])
        n = int(batch.rows[j])
        if st != 0 or n <= 0:
            continue
        scale[s, :n] = batch.scale[j, :n]
        c, si = trig_tables(batch.angle[j, :n])
        cos_t[s, :n] = c
        sin_t[s, :n] = si
    return FrameStackInput(echo=echo.view(F, G, R, bins), gains=gains, rows=R,
                           scale=scale.reshape(-1), cos_t=cos_t.reshape(-1),
                           sin_t=sin_t.reshape(-1),
                           file_status={p: int(s) for p, s in zip(paths, batch.status)})


def frame_points(frame_files: Dict[int, Path], threshold: float, stride: int, device,
                 bins: int = 1024, threads: int = 0):
    """One frame's fused points on the device: load_radar_csv per gain in ascending gain order,
    concatenated (build_frame :312-352 / fuse_gains_absolute 5_gain_fusion_ply_builder.py:193-219)
    with a loader's own threshold and stride.  Returns (x, y, intensity, gain) device tensors."""
    from . import _abi
    from ._device import stream_handle

    stack = load_frame_stack([frame_files], device, bins=bins, threads=threads,
                             on_error=lambda p, e: print(f"Error loading {p}: {e}"))
    lib = _abi.load()
    G, R = len(stack.gains), stack.rows
    dt = _abi.ECHO_U8 if stack.echo.dtype == torch.uint8 else _abi.ECHO_F32
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    sc, ct, sn = T(stack.scale), T(stack.cos_t), T(stack.sin_t)
    gd = torch.tensor(stack.gains, dtype=torch.int32, device=device)
    rp = torch.empty(G * R + 1, dtype=torch.int64, device=device)
    fo = torch.empty(G + 1, dtype=torch.int64, device=device)
    tot = _abi.C.c_int64(0)
    thr = float(np.float32(threshold))
    with torch.cuda.device(device):
        st = stream_handle(device)
        _abi.check(lib.rpt_polar_count(stack.echo.data_ptr(), dt, G, R, bins, thr, stride,
                                       rp.data_ptr(), fo.data_ptr(), _abi.C.byref(tot), st),
                   "rpt_polar_count")
        n = tot.value
        x = torch.empty(max(n, 1), dtype=torch.float32, device=device)
        y, v = torch.empty_like(x), torch.empty_like(x)
        g = torch.empty(max(n, 1), dtype=torch.int32, device=device)
        _abi.check(lib.rpt_polar_write(stack.echo.data_ptr(), dt, G, R, bins, sc.data_ptr(),
                                       ct.data_ptr(), sn.data_ptr(), gd.data_ptr(), thr, stride,
                                       rp.data_ptr(), fo.data_ptr(), G, x.data_ptr(),
                                       y.data_ptr(), v.data_ptr(), g.data_ptr(), None, st),
                   "rpt_polar_write")
    return x[:n], y[:n], v[:n], g[:n]
