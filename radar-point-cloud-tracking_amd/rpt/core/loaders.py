"""Drop-in for ``radar_pipeline.core.loaders`` containers and loaders
(radar-pipeline/src/radar_pipeline/core/loaders.py:15-101, :149-220).

The containers are the boundary types of the path.  load_radar_csv parses with librpt's native
CSV reader (csrc/csv.cpp; pandas read_csv semantics, checked against pandas
in tests/test_csv_ingest.py); the PLY reader keeps the reference's ASCII semantics.
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
    """loaders.py:46-101: pd.read_csv(names=Status..Echo_n, skiprows=1) semantics through the
    native parser; an empty CSV raises ValueError, a malformed one raises like read_csv."""
    from .ingest import (GAIN_DISAGREE, GAIN_FIRST_NAN, STATUS_EMPTY, STATUS_NON_NUMERIC,
                         STATUS_OK, read_sweeps)

    if config is None:
        config = RadarConfig()
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(f"[Errno 2] No such file or directory: '{path}'")
    b = read_sweeps([path], bins=config.num_echo_columns)
    st = int(b.status[0])
    if st == STATUS_EMPTY:
        raise ValueError(f"CSV is empty: {path}")
    if st == STATUS_NON_NUMERIC:
        raise ValueError(f"could not convert string to float in {path}")
    if st != STATUS_OK:  # read_csv's own exception text (ParserError is a ValueError)
        raise ValueError(b.errors[0] or f"Error tokenizing data in {path}")
    n = int(b.rows[0])
    angles_rad = np.deg2rad(b.angle[0, :n] * config.angle_scale)
    echo = b.echo[0, :n].astype(np.float32)
    scale = b.scale[0, :n].copy()
    ranges = (scale[:, None] / echo.shape[1]) * np.arange(echo.shape[1], dtype=np.float32)
    # gains = df["Gain"].unique(); one value -> int(it) (int(nan) raises), several -> None (:88-92)
    flags = int(b.gain_flags[0])
    gain = None
    if not flags & GAIN_DISAGREE:
        if flags & GAIN_FIRST_NAN:
            raise ValueError("cannot convert float NaN to integer")
        gain = int(float(b.gain[0]))
    return RadarSweep(angles_rad=angles_rad, ranges=ranges, intensities=echo, scale=scale,
                      gain=gain, source_path=path)


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
