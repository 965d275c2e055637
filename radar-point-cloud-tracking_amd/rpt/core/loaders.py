"""Drop-in for ``radar_pipeline.core.loaders`` containers and loaders
(radar-pipeline/src/radar_pipeline/core/loaders.py:15-101, :149-220).

The containers are the boundary types of the path.  The CSV/PLY parsers are host text I/O
("next"): they keep the reference's pandas / ASCII semantics here and
are not part of the timed device path.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np

from ..config import RadarConfig


@dataclass
class RadarSweep:
    """loaders.py:15-24"""

    angles_rad: np.ndarray
    ranges: np.ndarray
    intensities: np.ndarray
    scale: np.ndarray
    gain: Optional[int] = None
    source_path: Optional[Path] = None


@dataclass
class PointCloud:
    """loaders.py:27-43"""

    x: np.ndarray
    y: np.ndarray
    z: np.ndarray
    colors: Optional[np.ndarray] = None

    @property
    def size(self) -> int:
        return self.x.size

    def to_coords(self) -> np.ndarray:
        return np.column_stack((self.x, self.y, self.z))


def load_radar_csv(path: Path, config: Optional[RadarConfig] = None) -> RadarSweep:
    """loaders.py:46-101 (pandas C parser, like the reference)."""
    import pandas as pd

    if config is None:
        config = RadarConfig()
    cols = ["Status", "Scale", "Range", "Gain", "Angle"] + [
        f"Echo_{i}" for i in range(config.num_echo_columns)]
    df = pd.read_csv(path, header=None, names=cols, skiprows=1, engine="c")
    if df.empty:
        raise ValueError(f"CSV is empty: {path}")
    angles_rad = np.deg2rad(df["Angle"].to_numpy(np.float32) * config.angle_scale)
    echo = df.iloc[:, 5:].fillna(0).to_numpy(np.float32)
    scale = df["Scale"].to_numpy(np.float32)
    ranges = (scale[:, None] / echo.shape[1]) * np.arange(echo.shape[1], dtype=np.float32)
    gain = None
    gains = df["Gain"].unique()
    if len(gains) == 1:
        gain = int(gains[0])
    return RadarSweep(angles_rad=angles_rad, ranges=ranges, intensities=echo, scale=scale,
                      gain=gain, source_path=Path(path))


def load_ply(path: Path) -> PointCloud:
    """ASCII PLY reader with x/y/z and optional uchar RGB (loaders.py:149-220 /
    3_stdbscan_point_clouds.py:38-79)."""
    path = Path(path)
    with path.open("r", encoding="utf-8") as fh:
        lines = fh.readlines()
    if not lines or not lines[0].strip().startswith("ply"):
        raise ValueError(f"{path} is not a PLY file")
    n = None
    end = None
    props = []
    for i, line in enumerate(lines):
        s = line.strip()
        if s.startswith("element vertex"):
            n = int(s.split()[-1])
        elif s.startswith("property"):
            props.append(s.split()[-1])
        elif s == "end_header":
            end = i + 1
            break
    if n is None or end is None:
        raise ValueError(f"Could not parse header for {path}")
    rows = lines[end:end + n]
    data = np.fromiter((float(v) for ln in rows for v in ln.split()), dtype=np.float32,
                       count=len(rows[0].split()) * n if n else 0).reshape(n, -1)
    ix = {p: k for k, p in enumerate(props)}
    colors = None
    if {"red", "green", "blue"} <= ix.keys():
        colors = data[:, [ix["red"], ix["green"], ix["blue"]]].astype(np.uint8)
    return PointCloud(x=data[:, ix["x"]], y=data[:, ix["y"]], z=data[:, ix["z"]], colors=colors)
