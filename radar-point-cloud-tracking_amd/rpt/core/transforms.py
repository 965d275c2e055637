"""Drop-in for ``radar_pipeline.core.transforms`` (radar-pipeline/src/radar_pipeline/core/
transforms.py) — the polar -> Cartesian members run on the device (K1 kernels of librpt).

``trig_tables`` is the host half of the boundary: the reference evaluates numpy float32
cos/sin per azimuth row (4_temporal_object_tracker.py:203, :217-218); numpy's SIMD float32
cos/sin are not correctly rounded, so the tables are computed here exactly that way (4096 values
per sweep geometry) and handed to the kernels as inputs.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from .. import _abi
from .._device import is_torch, require_gpu, stream_handle, to_device
from ..config import ProcessingConfig, RadarConfig
from .loaders import PointCloud, RadarSweep

ANGLE_SCALE = 360.0 / 8196.0


def trig_tables(angle_col, angle_scale: float = ANGLE_SCALE) -> Tuple[np.ndarray, np.ndarray]:
    """float32 cos/sin of deg2rad(float32(Angle) * angle_scale) as the reference evaluates them
    (np.cos(angles_rad[:, None]) over the column)."""
    a = np.deg2rad(np.asarray(angle_col).astype(np.float32) * angle_scale)
    return np.cos(a[:, None])[:, 0].copy(), np.sin(a[:, None])[:, 0].copy()


def polar_to_cartesian(angles_rad, ranges):
    """transforms.py:13-34: x = ranges * cos(angles)[:, None], y = ranges * sin(...)."""
    want_torch = is_torch(ranges)
    a = angles_rad.detach().cpu().numpy() if is_torch(angles_rad) else np.asarray(angles_rad)
    c = np.cos(a[:, None])
    s = np.sin(a[:, None])
    if (not want_torch and (np.asarray(ranges).dtype != np.float32 or c.dtype != np.float32)):
        raise NotImplementedError("rpt polar_to_cartesian: float32 angles and ranges required")
    c = c[:, 0].astype(np.float32)
    s = s[:, 0].astype(np.float32)
    dev = require_gpu(ranges.device if want_torch else None)
    rd = to_device(ranges, torch.float32, dev)
    rows, bins = rd.shape
    x = torch.empty_like(rd)
    y = torch.empty_like(rd)
    cd = to_device(c, torch.float32, dev)
    sd = to_device(s, torch.float32, dev)
    st = _abi.load().rpt_polar_to_cartesian(cd.data_ptr(), sd.data_ptr(), rd.data_ptr(), rows,
                                            bins, x.data_ptr(), y.data_ptr(), stream_handle(dev))
    _abi.check(st, "rpt_polar_to_cartesian")
    if want_torch:
        return x, y
    return x.cpu().numpy(), y.cpu().numpy()


def sweep_to_point_cloud(sweep: RadarSweep, config: Optional[ProcessingConfig] = None,
                         radar_config: Optional[RadarConfig] = None) -> PointCloud:
    """transforms.py:37-79: threshold (strict >) + row-major flatten + stride, on the device."""
    if config is None:
        config = ProcessingConfig()
    if radar_config is None:
        radar_config = RadarConfig()
    a = np.asarray(sweep.angles_rad)
    c = np.cos(a[:, None])[:, 0]
    s = np.sin(a[:, None])[:, 0]
    inten = np.asarray(sweep.intensities)
    ranges = np.asarray(sweep.ranges)
    if inten.dtype != np.float32 or ranges.dtype != np.float32 or c.dtype != np.float32:
        raise NotImplementedError("rpt sweep_to_point_cloud: float32 sweep arrays required")
    rows, bins = inten.shape
    dev = require_gpu()
    idev = to_device(inten, torch.float32, dev)
    rdev = to_device(np.broadcast_to(ranges, inten.shape), torch.float32, dev)
    cd = to_device(c.astype(np.float32), torch.float32, dev)
    sd = to_device(s.astype(np.float32), torch.float32, dev)
    stride = max(int(config.point_stride), 1)
    cap = rows * bins // stride + 1
    x = torch.empty(cap, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    z = torch.empty_like(x)
    nout = _abi.C.c_int64(0)
    st = _abi.load().rpt_sweep_to_points(idev.data_ptr(), rdev.data_ptr(), cd.data_ptr(),
                                         sd.data_ptr(), rows, bins,
                                         float(np.float32(config.intensity_threshold)), stride,
                                         x.data_ptr(), y.data_ptr(), z.data_ptr(), cap,
                                         _abi.C.byref(nout), stream_handle(dev))
    _abi.check(st, "rpt_sweep_to_points")
    k = int(nout.value)
    return PointCloud(x=x[:k].cpu().numpy(), y=y[:k].cpu().numpy(), z=z[:k].cpu().numpy())


def subsample_cloud(cloud: PointCloud, max_points: int) -> Tuple[PointCloud, int]:
    """transforms.py:135-167 (host; unseeded random choice only above max_points)."""
    n = cloud.size
    if n <= max_points:
        return cloud, 1
    idx = np.random.choice(n, max_points, replace=False)
    stride = int(np.ceil(n / max_points))
    new_colors = cloud.colors[idx] if cloud.colors is not None else None
    return PointCloud(x=cloud.x[idx], y=cloud.y[idx], z=cloud.z[idx], colors=new_colors), stride


def apply_stride(cloud: PointCloud, stride: int) -> PointCloud:
    """transforms.py:170-198"""
    if stride <= 1:
        return cloud
    new_colors = cloud.colors[::stride] if cloud.colors is not None else None
    return PointCloud(x=cloud.x[::stride], y=cloud.y[::stride], z=cloud.z[::stride],
                      colors=new_colors)
