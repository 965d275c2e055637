"""Gain fusion of PointCloudWork/5_gain_fusion_ply_builder.py:
fuse_gains_absolute (:193-219, concatenation in ascending gain order) and fuse_gains_max
(:222-273, per-cell maximum intensity on a grid_resolution grid) over one frame's CSV files, with
that script's loader constants (INTENSITY_THRESHOLD 5.0, POINT_STRIDE 8, :57-58).  CSV parse in
librpt's native reader, polar scatter and max-pool on the device (K1 + rpt_fuse_gains_max)."""
from __future__ import annotations

from pathlib import Path
from typing import Dict, Tuple

import numpy as np
import torch

from .. import _abi
from .._device import require_gpu, stream_handle

INTENSITY_THRESHOLD = 5.0   # 5_gain_fusion_ply_builder.py:57
POINT_STRIDE = 8            # :58


def fuse_gains_absolute(frame_files: Dict[int, Path], device=None
                        ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """(x, y, intensity float32, gain int32), gains concatenated in ascending order."""
    from ..frames import frame_points

    dev = require_gpu(device)
    x, y, v, g = frame_points(frame_files, INTENSITY_THRESHOLD, POINT_STRIDE, dev)
    if x.numel() == 0:
        return np.array([]), np.array([]), np.array([]), np.array([])
    return x.cpu().numpy(), y.cpu().numpy(), v.cpu().numpy(), g.cpu().numpy()


def fuse_gains_max_points(x: torch.Tensor, y: torch.Tensor, v: torch.Tensor,
                          grid_resolution: float = 1.0):
    """Device form: max-pool float32 points (x, y, intensity > 0) -> (x f64, y f64, max f32)."""
    dev = x.device
    n = x.numel()
    ox = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    oy = torch.empty_like(ox)
    oi = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    cnt = _abi.C.c_int64(0)
    with torch.cuda.device(dev):
        _abi.check(_abi.load().rpt_fuse_gains_max(
            x.data_ptr(), y.data_ptr(), v.data_ptr(), n, float(grid_resolution), ox.data_ptr(),
            oy.data_ptr(), oi.data_ptr(), _abi.C.byref(cnt), stream_handle(dev)),
            "rpt_fuse_gains_max")
    k = cnt.value
    return ox[:k], oy[:k], oi[:k]


def fuse_gains_max(frame_files: Dict[int, Path], grid_resolution: float = 1.0, device=None
                   ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """:222-273 — (out_x float64, out_y float64, max intensity float32); empty arrays when no
    gain keeps a point."""
    from ..frames import frame_points

    dev = require_gpu(device)
    x, y, v, _ = frame_points(frame_files, INTENSITY_THRESHOLD, POINT_STRIDE, dev)
    if x.numel() == 0:
        return np.array([]), np.array([]), np.array([])
    ox, oy, oi = fuse_gains_max_points(x, y, v, grid_resolution)
    return ox.cpu().numpy(), oy.cpu().numpy(), oi.cpu().numpy()
