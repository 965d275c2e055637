"""Data-directory discovery and frame grouping of the tracker CLI:
parse_timestamp (PointCloudWork/4_temporal_object_tracker.py:165-181), discover_files
(:235-267) and group_files_by_frame (:270-309).  Host code: names, order and grouping rule are
the reference's, so the frames (and therefore frame ids, :941-944) are the same."""
from __future__ import annotations

import re
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Tuple

SUPPORTED_GAINS = {40, 50, 70, 75}   # :55
MAX_TIME_DIFF_MS = 2000              # :72

_TS = re.compile(r"(\d{8})_(\d{6})_(\d{3})\.csv")
_GAIN_DIR = re.compile(r"gain[_-]?(\d+)", re.IGNORECASE)


def parse_timestamp(filename: str) -> Tuple[datetime, int]:
    """'YYYYMMDD_HHMMSS_mmm.csv' -> (naive local datetime, epoch milliseconds + mmm) (:165-181;
    the epoch conversion uses the local time zone, as datetime.timestamp() does)."""
    m = _TS.match(filename)
    if m is None:
        raise ValueError(f"Cannot parse timestamp from {filename}")
    day, hms, ms = m.groups()
    dt = datetime.strptime(f"{day}_{hms}", "%Y%m%d_%H%M%S")
    return dt, int(dt.timestamp() * 1000) + int(ms)


def discover_files(data_dir: Path) -> Dict[int, List[Path]]:
    """{gain: csv paths sorted by timestamp} for every sub-directory named like gain_40 / gain-50
    / Gain75 whose gain is supported (:235-267).  Dict order = directory iteration order, like
    the reference (it prints the gains in that order)."""
    found: Dict[int, List[Tuple[int, Path]]] = {}
    for sub in Path(data_dir).iterdir():
        if not sub.is_dir():
            continue
        m = _GAIN_DIR.search(sub.name)
        if m is None:
            continue
        gain = int(m.group(1))
        if gain not in SUPPORTED_GAINS:
            continue
        for p in sub.glob("*.csv"):
            try:
                ts = parse_timestamp(p.name)[1]
            except ValueError:
                continue
            found.setdefault(gain, []).append((ts, p))  # the gain appears once a file parses
    out: Dict[int, List[Path]] = {}
    for gain, items in found.items():
        items.sort(key=lambda t: t[0])   # stable: equal timestamps keep glob order
        out[gain] = [p for _, p in items]
    return out


def group_files_by_frame(files_by_gain: Dict[int, List[Path]]) -> List[Dict[int, Path]]:
    """Frames = runs of files (all gains, ascending timestamp) within MAX_TIME_DIFF_MS of the
    run's first file; the first file of each gain in a run wins (:270-309)."""
    stamped = [(parse_timestamp(p.name)[1], gain, p)
               for gain, paths in files_by_gain.items() for p in paths]
    stamped.sort(key=lambda t: t[0])
    frames: List[Dict[int, Path]] = []
    cur: Dict[int, Path] = {}
    start = None
    for ts, gain, p in stamped:
        if start is not None and ts - start <= MAX_TIME_DIFF_MS:
            cur.setdefault(gain, p)
            continue
        if cur:
            frames.append(cur)
        start, cur = ts, {gain: p}
    if cur:
        frames.append(cur)
    return frames
