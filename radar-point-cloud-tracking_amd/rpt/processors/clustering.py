"""Drop-in for ``radar_pipeline.processors.clustering`` (radar-pipeline/src/radar_pipeline/
processors/clustering.py) and the ``st_dbscan`` of ``PointCloudWork/3_stdbscan_point_clouds.py``.

Same names, argument meaning and error behaviour; the work runs in librpt's HIP kernels:
numpy inputs are copied to the current ROCm device and numpy labels come back, torch inputs
stay on their device and a torch int32 tensor comes back.
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .. import _abi
from .._device import is_torch, ptr, require_gpu, stream_handle, to_device
from ..config import ClusteringConfig, GainConfig


def _times_to_f32(times, eps_time: float):
    """Reduce the reference's time comparison to the float32 form the kernel implements.

    float32 times: exact (NEP 50 makes the reference compare in float32).  Integer times, or
    float64 times that are all integers below 2^24: |dt| is an exact integer in every precision,
    so ``|dt| <= eps`` equals ``|dt| <= floor(eps)``, which float32 represents exactly.
    """
    if is_torch(times):
        dt = times.dtype
        if dt == torch.float32:
            return times, eps_time
        tt = times.to(torch.float64)
        fin = torch.isfinite(tt)
        integral = bool(torch.all(~fin | ((tt == torch.floor(tt)) & (tt.abs() < 2**24))))
        if not integral:
            raise NotImplementedError(
                f"rpt st_dbscan: non-float32 times ({dt}) must be integral below 2^24")
        return tt.to(torch.float32), float(np.floor(eps_time)) if np.isfinite(eps_time) else eps_time
    a = np.asarray(times)
    if a.dtype == np.float32:
        return a, eps_time
    if a.dtype.kind in "iub" or a.dtype.kind == "f":
        af = a.astype(np.float64)
        fin = np.isfinite(af)
        if not np.all(~fin | ((af == np.floor(af)) & (np.abs(af) < 2**24))):
            raise NotImplementedError(
                f"rpt st_dbscan: non-float32 times ({a.dtype}) must be integral below 2^24")
        e = float(np.floor(eps_time)) if np.isfinite(eps_time) else eps_time
        return af.astype(np.float32), e
    raise TypeError(f"unsupported times dtype {a.dtype}")


def _coords_to_f32(coords):
    if is_torch(coords):
        if coords.dtype == torch.float32:
            return coords
        c32 = coords.to(torch.float32)
        if not torch.equal(c32.to(coords.dtype), coords):
            raise NotImplementedError("rpt st_dbscan: coordinates must be float32-representable")
        return c32
    a = np.asarray(coords)
    if a.dtype == np.float32:
        return a
    a32 = a.astype(np.float32)
    with np.errstate(invalid="ignore"):
        same = np.array_equal(a32.astype(a.dtype), a, equal_nan=True)
    if not same:
        raise NotImplementedError("rpt st_dbscan: coordinates must be float32-representable")
    return a32


def st_dbscan(coords, times, eps_space: float, eps_time: float, min_samples: int,
              stats: Optional[dict] = None):
    """Spatio-temporal DBSCAN (clustering.py:49-115; 3_stdbscan_point_clouds.py:101-136).

    coords: (N, 2|3) float32 array/tensor; times: (N,) float32 (integral int/f64 accepted).
    Returns int32 labels, -1 for noise, ids ascending with each cluster's first core point —
    bit-identical to the reference BFS.  Empty input raises ValueError like sklearn's BallTree.
    """
    want_torch = is_torch(coords)
    c = _coords_to_f32(coords)
    shape = tuple(c.shape)
    if len(shape) != 2:
        raise ValueError(f"Expected 2D array, got {len(shape)}D array instead")
    n, dim = shape
    if n == 0:
        raise ValueError(
            f"Found array with 0 sample(s) (shape=(0, {dim})) while a minimum of 1 is required.")
    if dim not in (2, 3):
        raise NotImplementedError(f"rpt st_dbscan supports 2 or 3 coordinates, got {dim}")
    t, eps_t = _times_to_f32(times, float(eps_time))
    if (t.shape[0] if is_torch(t) else len(t)) != n:
        raise ValueError("coords and times must have the same length")
    dev = require_gpu(c.device if is_torch(c) else None)
    cd = to_device(c, torch.float32, dev)
    td = to_device(t, torch.float32, dev)
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    lib = _abi.load()
    st = _abi.StdbscanStats()
    st.timing = 1 if stats is not None else 0
    base = cd.data_ptr()
    with torch.cuda.device(dev):
        status = lib.rpt_stdbscan(base, base + 4, (base + 8) if dim == 3 else None, dim,
                                  td.data_ptr(), n, float(eps_space), float(eps_t),
                                  int(min_samples), labels.data_ptr(), st,
                                  stream_handle(dev))
    _abi.check(status, "rpt_stdbscan")
    if stats is not None:
        stats.update(n_clusters=st.n_clusters, grid_dims=tuple(st.grid_dims),
                     grid_cells=st.grid_cells, ms_bounds=st.ms_bounds, ms_grid=st.ms_grid,
                     ms_core=st.ms_core, ms_union=st.ms_union, ms_label=st.ms_label)
    if want_torch:
        return labels
    return labels.cpu().numpy()


def st_dbscan_soa(x: torch.Tensor, y: torch.Tensor, times: torch.Tensor, eps_space: float,
                  eps_time: float, min_samples: int, z: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None, stats: Optional[dict] = None
                  ) -> torch.Tensor:
    """Device-resident form for structure-of-arrays float32 tensors (the tracker's frame stack)."""
    n = x.numel()
    if n == 0:
        raise ValueError("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 is "
                         "required.")
    dev = x.device
    labels = out if out is not None else torch.empty(n, dtype=torch.int32, device=dev)
    st = _abi.StdbscanStats()
    st.timing = 1 if stats is not None else 0
    with torch.cuda.device(dev):  # librpt allocates on the calling thread's current device
        status = _abi.load().rpt_stdbscan(ptr(x), ptr(y), ptr(z), 1, ptr(times), n,
                                          float(eps_space), float(eps_time), int(min_samples),
                                          labels.data_ptr(), st, stream_handle(dev))
    _abi.check(status, "rpt_stdbscan")
    if stats is not None:
        stats.update(n_clusters=st.n_clusters, grid_dims=tuple(st.grid_dims),
                     grid_cells=st.grid_cells, ms_bounds=st.ms_bounds, ms_grid=st.ms_grid,
                     ms_core=st.ms_core, ms_union=st.ms_union, ms_label=st.ms_label)
    return labels


def infer_time_from_colors(colors, gain_colors: Optional[Dict[int, Tuple[int, int, int]]] = None):
    """clustering.py:17-46: nearest gain tint (first minimum) -> 0, 1, 2, ... as float32."""
    if gain_colors is None:
        gain_colors = GainConfig().colors
    gains_sorted = sorted(gain_colors.keys())
    palette = np.array([gain_colors[g] for g in gains_sorted], dtype=np.float32).reshape(-1, 3)
    want_torch = is_torch(colors)
    n = int(colors.shape[0])
    if n == 0:
        return colors.new_empty((0,), dtype=torch.float32) if want_torch else \
            np.zeros(0, dtype=np.float32)
    if palette.shape[0] == 0:
        raise ValueError("attempt to get argmin of an empty sequence")
    dev = require_gpu(colors.device if want_torch else None)
    cd = to_device(colors, torch.uint8, dev)
    pd = to_device(palette, torch.float32, dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        status = _abi.load().rpt_infer_time_from_colors(cd.data_ptr(), n, pd.data_ptr(),
                                                        palette.shape[0], out.data_ptr(),
                                                        stream_handle(dev))
    _abi.check(status, "rpt_infer_time_from_colors")
    return out if want_torch else out.cpu().numpy()


def cluster_point_cloud(cloud, config: Optional[ClusteringConfig] = None,
                        gain_config: Optional[GainConfig] = None):
    """clustering.py:118-154"""
    if config is None:
        config = ClusteringConfig()
    if gain_config is None:
        gain_config = GainConfig()
    coords = cloud.to_coords()
    times = infer_time_from_colors(cloud.colors, gain_config.colors)
    return st_dbscan(coords, times, eps_space=config.eps_space, eps_time=config.eps_time,
                     min_samples=config.min_samples)


def process_ply_clustering(ply_path: Path, output_dir: Optional[Path] = None,
                           config: Optional[ClusteringConfig] = None,
                           gain_config: Optional[GainConfig] = None):
    """clustering.py:157-208 (PLY load -> subsample -> cluster -> labels CSV)."""
    from ..core.loaders import load_ply
    from ..core.transforms import subsample_cloud
    from ..core.writers import write_labels_csv

    if config is None:
        config = ClusteringConfig()
    if gain_config is None:
        gain_config = GainConfig()
    ply_path = Path(ply_path)
    if output_dir is None:
        output_dir = ply_path.parent
    cloud = load_ply(ply_path)
    cloud, stride = subsample_cloud(cloud, config.max_points)
    print(f"{ply_path.name}: using {cloud.size:,} points (approx stride={stride})")
    labels = cluster_point_cloud(cloud, config, gain_config)
    unique, counts = np.unique(labels, return_counts=True)
    summary = dict(zip(unique.tolist(), counts.tolist()))
    print(f"{ply_path.name}: labels summary {summary}")
    out_stem = f"{ply_path.stem}_dbscan"
    csv_path = Path(output_dir) / f"{out_stem}_labels.csv"
    write_labels_csv(csv_path, cloud.to_coords(), labels)
    print(f"Labels CSV -> {csv_path.name}")
    return csv_path, labels
