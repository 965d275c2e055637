"""Drop-in for ``radar_pipeline.core.writers.write_labels_csv`` (core/writers.py:65-81)."""
from __future__ import annotations

from pathlib import Path

import numpy as np


def write_labels_csv(path: Path, coords: np.ndarray, labels: np.ndarray) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    arr = np.column_stack((coords, labels))
    np.savetxt(path, arr, fmt="%.6f,%.6f,%.6f,%d", header="x,y,z,label", comments="")


def save_tracking_results(objects, cluster_rows, output_dir: Path) -> None:
    """PointCloudWork/4_temporal_object_tracker.py:832-886: tracked_objects.csv, trajectories.csv
    and clusters.csv written by pandas from the same Python scalars the reference puts in its
    rows (np.float32 centroids, the exact type of average_velocity, Python float mean
    intensities), so pandas infers the same column dtypes and the files are byte-identical.

    objects: TrackedObject snapshots in tracker dict order (rpt.native_tracker);
    cluster_rows: (frame_id, cluster_id, num_points, cx np.float32, cy np.float32, mean_i float)
    in clusters_by_frame order (frames with clusters, each frame's clusters in reference order).
    """
    import pandas as pd

    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    summary = []
    for o in objects:
        seen = o.frames_seen
        summary.append({"object_id": o.object_id, "object_type": o.object_type,
                        "num_frames_seen": len(seen),
                        "first_frame": min(seen) if seen else -1,
                        "last_frame": max(seen) if seen else -1,
                        "avg_velocity": o.average_velocity,
                        "final_x": o.centroid[0], "final_y": o.centroid[1]})
    path = output_dir / "tracked_objects.csv"
    pd.DataFrame(summary).to_csv(path, index=False)
    print(f"Saved object summary to {path}")

    traj = [{"object_id": o.object_id, "object_type": o.object_type, "frame_id": f,
             "x": pos[0], "y": pos[1]}
            for o in objects for pos, f in zip(o.positions, o.frames_seen)]
    path = output_dir / "trajectories.csv"
    pd.DataFrame(traj).to_csv(path, index=False)
    print(f"Saved trajectories to {path}")

    rows = [{"frame_id": fid, "cluster_id": cid, "num_points": n, "centroid_x": cx,
             "centroid_y": cy, "mean_intensity": mi}
            for fid, cid, n, cx, cy, mi in cluster_rows]
    path = output_dir / "clusters.csv"
    pd.DataFrame(rows).to_csv(path, index=False)
    print(f"Saved clusters to {path}")
