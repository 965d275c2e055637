"""Denoise mode: drop-in for PointCloudWorkF/stdbscan_denoising_pipeline.py.

The reference's variant ST-DBSCAN (st_dbscan :264-369) differs from the tracker's in two ways,
both computed on the device by ``rpt_stdbscan_denoise`` (csrc/stdbscan.hip):

* core points need >= min_samples space-time neighbours (itself included) that ALSO span
  >= min_frames distinct int32(time) frames (:308-315) -- single-frame blobs are noise;
* clusters grow through a FIFO queue that never re-queues a visited point (:340-367), so a
  border point takes the first cluster (in seed order) that reaches it while it is unvisited, or
  whose seed is its direct neighbour -- not simply the smallest adjacent cluster.

The pipeline around it (run_pipeline :862-1046) keeps the reference's file discovery and
2-second frame grouping (:155-216), loads every sweep through the native CSV parser and the K1
kernels (threshold 10, stride 4, gains concatenated in the frame's time order, :97-152 /
:219-231), stamps each point with its frame index (empty frames keep their index, :933-940), and
writes the same outputs: the binary PLYs (:767-855), denoising_stats.csv and clusters.csv (the
pandas group means of :997-1012, computed by ``rpt_label_means``).  The PNG / GIF visualisations
(:1015-1041) are not built: matplotlib rendering is outside this engine's scope.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _abi
from ._device import require_gpu, stream_handle, to_device

ANGLE_SCALE = 360.0 / 8196.0          # :64
NUM_ECHO_COLUMNS = 1024               # :65
INTENSITY_THRESHOLD = 10.0            # :68
POINT_STRIDE = 4                      # :69
MAX_TIME_DIFF_MS = 2000               # :70
MAX_WORKERS = min(4, os.cpu_count() or 1)   # :71 (only printed: the native parser is threaded)
DEFAULT_EPS_SPACE = 8.0               # :74-77
DEFAULT_EPS_TIME = 2.0
DEFAULT_MIN_SAMPLES = 15
DEFAULT_MIN_FRAMES = 2

_TS = re.compile(r"(\d{8})_(\d{6})_(\d{3})")
_GAIN_DIR = re.compile(r"gain[_-]?(\d+)", re.IGNORECASE)


def parse_timestamp(filename: str) -> datetime:
    """:87-94 -- 'YYYYMMDD_HHMMSS_mmm...' -> datetime with the milliseconds."""
    m = _TS.match(filename)
    if not m:
        raise ValueError(f"Cannot parse timestamp from: {filename}")
    day, hms, ms = m.groups()
    return datetime.strptime(f"{day}_{hms}", "%Y%m%d_%H%M%S").replace(microsecond=int(ms) * 1000)


def discover_files(data_dir: Path) -> Dict[int, List[Tuple[datetime, Path]]]:
    """:155-181 -- {gain: [(timestamp, path)] ascending} for every gain directory (any gain)."""
    out: Dict[int, List[Tuple[datetime, Path]]] = {}
    for gain_dir in Path(data_dir).iterdir():
        if not gain_dir.is_dir():
            continue
        m = _GAIN_DIR.match(gain_dir.name)
        if not m:
            continue
        files = []
        for p in sorted(gain_dir.glob("*.csv")):
            try:
                files.append((parse_timestamp(p.name), p))
            except ValueError:
                continue
        if files:
            out[int(m.group(1))] = sorted(files, key=lambda x: x[0])
    return out


def group_into_frames(gain_files: Dict[int, List[Tuple[datetime, Path]]]) -> List[Dict[int, Path]]:
    """:184-216 -- runs of files within MAX_TIME_DIFF_MS of the run's first file; the first file
    of each gain in a run wins; dict order = time order (the frame's concatenation order)."""
    all_files = sorted(((ts, gain, p) for gain, files in gain_files.items() for ts, p in files),
                       key=lambda x: x[0])
    frames: List[Dict[int, Path]] = []
    cur: Dict[int, Path] = {}
    t0 = None
    for ts, gain, p in all_files:
        if t0 is None:
            t0 = ts
            cur[gain] = p
        elif (ts - t0).total_seconds() * 1000 <= MAX_TIME_DIFF_MS:
            if gain not in cur:
                cur[gain] = p
        else:
            if cur:
                frames.append(cur)
            cur = {gain: p}
            t0 = ts
    if cur:
        frames.append(cur)
    return frames


@dataclass
class DenoiseFrames:
    x: torch.Tensor          # device float32 [n]: all points, frame-major
    y: torch.Tensor
    z: torch.Tensor          # intensity
    t: torch.Tensor          # device float32 [n]: frame index (empty frames keep theirs)
    frame_counts: np.ndarray  # int64 [n_frames]
    failed: List[tuple] = None  # [(frame index, exception text)] of frames whose load raised


class FrameLoadError(Exception):
    """A frame's load raised in the reference (sequential mode re-raises it as its own type)."""


def _raise_like_reference(detail_kind: int, msg: str):
    if detail_kind == 1:
        import errno as _errno
        code = int(msg.split("]")[0].split()[-1]) if msg.startswith("[Errno") else _errno.EIO
        raise OSError(code, msg)
    if detail_kind == 5:
        raise IndexError(msg)
    raise ValueError(msg)


def load_frames(frames: List[Dict[int, Path]], device=None, threads: int = 0,
                parallel: bool = False) -> DenoiseFrames:
    """load_frame / load_radar_csv (:97-152, :219-231) for every frame on the device: sweeps
    parsed natively with the reference loader's semantics (np.genfromtxt first, pd.read_csv when
    it raises: rpt.core.ingest MODE_GENFROMTXT), K1 (threshold > 10, every 4th kept sample of
    each file) with the frame's files in its dict order, times = frame index.  A file whose
    genfromtxt rows hold 5 + W fields with W != 1024 has W bins (num_bins = data[:, 5:].shape[1],
    range resolution Scale / W, :128-134): such files are parsed and scattered as batches of
    their own width and their points put back in file order.
    A file whose load raises fails its whole frame (load_frame stops at it): with parallel=True
    (load_frames_parallel, :234-257) the frame is empty and listed in `failed`; otherwise the
    exception propagates as in the sequential loop (:910-915)."""
    from .core.ingest import (MODE_GENFROMTXT, STATUS_NON_NUMERIC, STATUS_UNSUPPORTED,
                              read_sweeps)

    dev = require_gpu(device)
    paths, fidx = [], []
    for f, fr in enumerate(frames):
        for p in fr.values():
            paths.append(Path(p))
            fidx.append(f)
    n_files = len(paths)
    empty = torch.zeros(0, dtype=torch.float32, device=dev)
    if n_files == 0:
        return DenoiseFrames(empty, empty, empty, empty, np.zeros(len(frames), np.int64), [])
    batch = read_sweeps(paths, bins=NUM_ECHO_COLUMNS, threads=threads, mode=MODE_GENFROMTXT)
    # files of another bin count, re-parsed per width (their status and errors replace the first
    # parse's; genfromtxt itself raises nothing for them)
    groups = {NUM_ECHO_COLUMNS: ([j for j in range(n_files)
                                  if batch.status[j] != STATUS_UNSUPPORTED], batch, None)}
    status = list(batch.status)
    errors = list(batch.errors)
    kinds = list(batch.detail_kind)
    widths = sorted({int(w) - 5 for w, s_ in zip(batch.n_fields, batch.status)
                     if s_ == STATUS_UNSUPPORTED})
    for W in widths:
        js = [j for j in range(n_files) if batch.status[j] == STATUS_UNSUPPORTED and
              int(batch.n_fields[j]) - 5 == W]
        if W <= 0:   # Status..Angle only: no echo column, no point (:139-156 on an empty mask)
            for j in js:
                status[j] = -1
            continue
        sub = read_sweeps([paths[j] for j in js], bins=W, threads=threads, mode=MODE_GENFROMTXT)
        for k, j in enumerate(js):
            status[j], errors[j], kinds[j] = sub.status[k], sub.errors[k], sub.detail_kind[k]
        groups[W] = (js, sub, list(range(len(js))))
    failed, dead = [], set()
    for j, p in enumerate(paths):
        f = fidx[j]
        if f in dead:
            continue   # load_frame stopped at this frame's first failing file
        msg = errors[j]
        if msg is None and status[j] == STATUS_NON_NUMERIC:
            msg = f"could not convert string to float in {p}"
        if msg is None:
            continue
        if not parallel:
            _raise_like_reference(int(kinds[j]), msg)
        dead.add(f)
        failed.append((f, msg))
    counts = np.zeros(len(frames), np.int64)
    js0, b0, _ = groups[NUM_ECHO_COLUMNS]
    with torch.cuda.device(dev):
        if len(groups) == 1 and len(js0) == n_files:   # every file 1024 bins: one K1 batch
            x, y, z, pf, fo_h = _k1_files(b0, js0, [fidx[j] not in dead for j in js0],
                                          NUM_ECHO_COLUMNS, dev)
            n = int(fo_h[-1])
            t = torch.empty_like(x)
            if n:
                ids = torch.tensor(fidx, dtype=torch.int64, device=dev)
                _abi.check(_abi.load().rpt_frame_times(pf.data_ptr(), n, ids.data_ptr(),
                                                       t.data_ptr(), stream_handle(dev)),
                           "rpt_frame_times")
            np.add.at(counts, np.asarray(fidx, np.int64), np.diff(fo_h))
            return DenoiseFrames(x[:n], y[:n], z[:n], t[:n], counts, failed)
        # K1 per width group, then every file's points in the global file order
        per_file: List[Optional[Tuple[torch.Tensor, ...]]] = [None] * n_files
        for W, (js, b, idx) in groups.items():
            if not js:
                continue
            x, y, z, _, fo_h = _k1_files(b, js if idx is None else idx,
                                         [fidx[j] not in dead for j in js], W, dev)
            for k, j in enumerate(js):
                per_file[j] = (x[fo_h[k]:fo_h[k + 1]], y[fo_h[k]:fo_h[k + 1]],
                               z[fo_h[k]:fo_h[k + 1]])
        pieces = [(j, pc) for j, pc in enumerate(per_file) if pc is not None and pc[0].numel()]
        for j, pc in pieces:
            counts[fidx[j]] += pc[0].numel()
        if not pieces:
            return DenoiseFrames(empty, empty, empty, empty, counts, failed)
        x, y, z = (torch.cat([pc[k] for _, pc in pieces]) for k in range(3))
        t = torch.cat([torch.full((pc[0].numel(),), float(fidx[j]), dtype=torch.float32,
                                  device=dev) for j, pc in pieces])
    return DenoiseFrames(x, y, z, t, counts, failed)


def _k1_files(batch, idx: List[int], keep: List[bool], bins: int, dev):
    """K1 (threshold, stride 4 per file) over the files `idx` of a parsed batch of `bins` bins
    (files not kept scatter nothing) -> device x, y, intensity, file slot per point, and the
    host file offsets [len(idx) + 1]."""
    from .core.transforms import trig_tables

    lib = _abi.load()
    n_files = len(idx)
    R = max(int(batch.echo.shape[1]), 1)
    scale = np.zeros((n_files, R), np.float32)
    cos_t = np.zeros((n_files, R), np.float32)
    sin_t = np.zeros((n_files, R), np.float32)
    for k, j in enumerate(idx):
        n = int(batch.rows[j])
        if batch.status[j] != 0 or n <= 0 or not keep[k]:
            continue
        scale[k, :n] = batch.scale[j, :n]
        cos_t[k, :n], sin_t[k, :n] = trig_tables(batch.angle[j, :n], ANGLE_SCALE)
    if not batch.echo.shape[1]:
        echo = np.zeros((n_files, 1, bins), batch.echo.dtype)
    elif list(idx) == list(range(batch.echo.shape[0])):
        echo = np.ascontiguousarray(batch.echo)
    else:
        echo = np.ascontiguousarray(batch.echo[idx])
    drop = ~np.asarray(keep, bool)
    if drop.any():   # a failed frame is empty (load_frames_parallel's empty arrays)
        echo[drop] = 0
    dt = _abi.ECHO_U8 if echo.dtype == np.uint8 else _abi.ECHO_F32
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    st = stream_handle(dev)
    ed, sc, ct, sn = T(echo), T(scale), T(cos_t), T(sin_t)
    rp = torch.empty(n_files * R + 1, dtype=torch.int64, device=dev)
    fo = torch.empty(n_files + 1, dtype=torch.int64, device=dev)
    tot = _abi.C.c_int64(0)
    thr = float(np.float32(INTENSITY_THRESHOLD))
    _abi.check(lib.rpt_polar_count(ed.data_ptr(), dt, n_files, R, bins, thr, POINT_STRIDE,
                                   rp.data_ptr(), fo.data_ptr(), _abi.C.byref(tot), st),
               "rpt_polar_count")
    n = int(tot.value)
    x = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    y, z = torch.empty_like(x), torch.empty_like(x)
    pf = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    _abi.check(lib.rpt_polar_write(ed.data_ptr(), dt, n_files, R, bins, sc.data_ptr(),
                                   ct.data_ptr(), sn.data_ptr(), None, thr, POINT_STRIDE,
                                   rp.data_ptr(), fo.data_ptr(), 1, x.data_ptr(), y.data_ptr(),
                                   z.data_ptr(), None, pf.data_ptr(), st), "rpt_polar_write")
    return x, y, z, pf, fo.cpu().numpy()


def st_dbscan(coords, times, eps_space: float, eps_time: float, min_samples: int,
              min_frames: int = 2, device=None):
    """:264-369 on the device.  coords [n, 2] and times [n] (numpy or device tensors, float32);
    returns int32 labels (-1 noise) as numpy for numpy input, else a device tensor."""
    want_torch = isinstance(coords, torch.Tensor)
    dev = require_gpu(coords.device if want_torch else device)
    c = to_device(coords, torch.float32, dev)
    if c.ndim != 2 or c.shape[1] != 2:
        raise ValueError("coords must be [n, 2]")
    tt = to_device(times, torch.float32, dev).reshape(-1)
    n = int(c.shape[0])
    labels = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    if n:
        xs = c[:, 0].contiguous()
        ys = c[:, 1].contiguous()
        stats = _abi.StdbscanStats()
        with torch.cuda.device(dev):
            _abi.check(_abi.load().rpt_stdbscan_denoise(
                xs.data_ptr(), ys.data_ptr(), tt.data_ptr(), n, float(eps_space),
                float(eps_time), int(min_samples), int(min_frames), labels.data_ptr(),
                _abi.C.byref(stats), stream_handle(dev)), "rpt_stdbscan_denoise")
    labels = labels[:n]
    return labels if want_torch else labels.cpu().numpy()


def cluster_table(labels: torch.Tensor, x: torch.Tensor, y: torch.Tensor, z: torch.Tensor,
                  n_clusters: int):
    """:997-1012 -- pandas groupby('cluster_id').agg(count, mean, mean, mean) of the signal
    points, the means computed on the device (rpt_label_means: pandas' float32 Kahan group
    mean).  Returns the DataFrame the reference writes (same column dtypes)."""
    import pandas as pd

    dev = x.device
    k = max(int(n_clusters), 1)
    cnt = torch.zeros(k, dtype=torch.int64, device=dev)
    mx, my, mz = (torch.zeros(k, dtype=torch.float32, device=dev) for _ in range(3))
    n = int(labels.numel())
    with torch.cuda.device(dev):
        _abi.check(_abi.load().rpt_label_means(
            labels.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(), n, int(n_clusters),
            cnt.data_ptr(), mx.data_ptr(), my.data_ptr(), mz.data_ptr(), stream_handle(dev)),
            "rpt_label_means")
    cnt_h = cnt.cpu().numpy()[:n_clusters]
    keep = cnt_h > 0
    ids = np.nonzero(keep)[0].astype(np.int32)
    return pd.DataFrame({"cluster_id": ids, "num_points": cnt_h[keep].astype(np.int64),
                         "centroid_x": mx.cpu().numpy()[:n_clusters][keep],
                         "centroid_y": my.cpu().numpy()[:n_clusters][keep],
                         "mean_intensity": mz.cpu().numpy()[:n_clusters][keep]})


def write_ply(path: Path, x: np.ndarray, y: np.ndarray, z: np.ndarray,
              labels: Optional[np.ndarray] = None, use_binary: bool = True) -> None:
    """:767-855 -- file formatting on the host: tab20 colours by label % 20 (noise grey 128),
    or viridis of intensity / 255 without labels, exactly as the reference evaluates them."""
    import matplotlib

    num_points = len(x)
    if num_points == 0:
        print(f"Skipping empty point cloud: {Path(path).name}")
        return
    if labels is not None:
        colors = np.full((num_points, 3), 128, dtype=np.uint8)
        mask = labels >= 0
        if mask.any():
            cmap = matplotlib.colormaps["tab20"]
            lut = (np.array([cmap(i)[:3] for i in range(20)]) * 255).astype(np.uint8)
            colors[mask] = lut[labels[mask] % 20]
    else:
        z_norm = np.clip(z / 255.0, 0, 1)
        colors = (matplotlib.colormaps["viridis"](z_norm)[:, :3] * 255).astype(np.uint8)
    if use_binary:
        header = ("ply\nformat binary_little_endian 1.0\n"
                  f"element vertex {num_points}\n"
                  "property float x\nproperty float y\nproperty float z\n"
                  "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
        rec = np.empty(num_points, dtype=np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                                                   ("r", "u1"), ("g", "u1"), ("b", "u1")]))
        rec["x"], rec["y"], rec["z"] = (np.asarray(a).astype(np.float32) for a in (x, y, z))
        rec["r"], rec["g"], rec["b"] = colors[:, 0], colors[:, 1], colors[:, 2]
        with Path(path).open("wb") as fh:
            fh.write(header.encode("ascii"))
            rec.tofile(fh)
    else:
        header = ("ply\nformat ascii 1.0\n"
                  f"element vertex {num_points}\n"
                  "property float x\nproperty float y\nproperty float z\n"
                  "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
        data = np.column_stack([np.asarray(a).astype(np.float32) for a in (x, y, z)] + [colors])
        with Path(path).open("w", encoding="utf-8") as fh:
            fh.write(header)
            np.savetxt(fh, data, fmt="%.4f %.4f %.4f %d %d %d")
    print(f"Wrote {num_points:,} points to {Path(path).name}")


def run_pipeline(data_dir: Path, output_dir: Path, eps_space: float = DEFAULT_EPS_SPACE,
                 eps_time: float = DEFAULT_EPS_TIME, min_samples: int = DEFAULT_MIN_SAMPLES,
                 min_frames: int = DEFAULT_MIN_FRAMES, max_frames: int = 0, no_viz: bool = True,
                 skip_gif: bool = True, parallel: bool = True, low_memory: bool = False,
                 device=None) -> Optional[dict]:
    """:862-1046 with the compute on the device; the same stdout lines and output files.
    Returns the stats dict (None when no point was found)."""
    import pandas as pd

    print("=" * 60)
    print("ST-DBSCAN RADAR POINT CLOUD DENOISING PIPELINE")
    print("=" * 60)
    print("\n[1/5] Discovering data files...")
    gain_files = discover_files(Path(data_dir))
    if not gain_files:
        raise FileNotFoundError(f"No gain folders found in {data_dir}")
    for gain, files in sorted(gain_files.items()):
        print(f"  Gain {gain}: {len(files)} files")
    print("\n[2/5] Grouping files into temporal frames...")
    frames = group_into_frames(gain_files)
    print(f"  Found {len(frames)} frames")
    if max_frames > 0:
        frames = frames[:max_frames]
        print(f"  Processing first {len(frames)} frames")
    print("\n[3/5] Converting radar data to Cartesian point clouds...")
    par = parallel and len(frames) > 4
    if par:
        print(f"  Using parallel loading with {MAX_WORKERS} workers...")
    fr = load_frames(frames, device, parallel=par)
    if par:
        # load_frames_parallel (:234-257): a failed frame's warning, then every 20th completion
        # (printed here in frame order; the reference's as_completed order varies run to run)
        failed = dict(fr.failed)
        for k in range(1, len(frames) + 1):
            if k - 1 in failed:
                print(f"  Warning: Failed to load frame {k - 1}: {failed[k - 1]}")
            if k % 20 == 0:
                print(f"  Loaded {k}/{len(frames)} frames...")
    else:
        for k in range(10, len(frames) + 1, 10):
            print(f"  Processed {k}/{len(frames)} frames...")
    total = int(fr.frame_counts.sum())
    print(f"  Total points: {total:,}")
    if total == 0:
        print("  No points found! Check data directory.")
        return None
    print(f"  Total points: {total:,}")

    print("\n[4/5] Applying ST-DBSCAN clustering for denoising...")
    print(f"  Parameters: eps_space={eps_space}, eps_time={eps_time}, min_samples={min_samples}, "
          f"min_frames={min_frames}")
    coords = torch.stack([fr.x, fr.y], 1)
    labels_d = st_dbscan(coords, fr.t, eps_space, eps_time, min_samples, min_frames)
    labels = labels_d.cpu().numpy()
    noise_mask = labels == -1
    signal_mask = ~noise_mask
    num_clusters = len(np.unique(labels[signal_mask]))
    stats = {"total_points": total, "noise_points": noise_mask.sum(),
             "signal_points": signal_mask.sum(), "num_clusters": num_clusters,
             "noise_reduction_pct": 100.0 * noise_mask.sum() / total}
    print("\n  Results:")
    print(f"    Total points:      {stats['total_points']:,}")
    print(f"    Noise (removed):   {stats['noise_points']:,} "
          f"({stats['noise_reduction_pct']:.1f}%)")
    print(f"    Signal (kept):     {stats['signal_points']:,}")
    print(f"    Clusters found:    {stats['num_clusters']}")

    print("\n[5/5] Saving results...")
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    ax, ay, az = fr.x.cpu().numpy(), fr.y.cpu().numpy(), fr.z.cpu().numpy()
    write_ply(out / "denoised_point_cloud.ply", ax[signal_mask], ay[signal_mask],
              az[signal_mask], labels[signal_mask])
    write_ply(out / "raw_point_cloud.ply", ax, ay, az)
    pd.DataFrame([stats]).to_csv(out / "denoising_stats.csv", index=False)
    print("Saved: denoising_stats.csv")
    if num_clusters > 0:
        cluster_table(labels_d, fr.x, fr.y, fr.z, int(labels.max()) + 1).to_csv(
            out / "clusters.csv", index=False)
        print("Saved: clusters.csv")
    if not no_viz:
        import sys

        print("rpt: the PNG/GIF visualisations are not generated (plot rendering is outside "
              "this engine's scope)", file=sys.stderr)
    print("\n" + "=" * 60)
    print("PIPELINE COMPLETE")
    print(f"Results saved to: {out}")
    print("=" * 60)
    return stats
