"""Drop-in for ``radar_pipeline.core.writers.write_labels_csv`` (core/writers.py:65-81)."""
from __future__ import annotations

from pathlib import Path

import numpy as np


def write_labels_csv(path: Path, coords: np.ndarray, labels: np.ndarray) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    arr = np.column_stack((coords, labels))
    np.savetxt(path, arr, fmt="%.6f,%.6f,%.6f,%d", header="x,y,z,label", comments="")
