"""Drop-in for ``python PointCloudWork/3_stdbscan_point_clouds.py [--offset P] [--flat P]``
(main :196-215, process_one :174-193): ST-DBSCAN in 3-D (x, y, z) on stacked PLY clouds with the
time step inferred from each point's gain tint, on the MI355X (rpt_stdbscan D=3 + the colour
kernel).  Labels CSV byte-identical ("%.6f,%.6f,%.6f,%d", header x,y,z,label, :139-142).
The PNG preview (:145-171) is not rendered (outside this engine's scope)."""
from __future__ import annotations

import argparse
from pathlib import Path

import numpy as np

EPS_SPACE, EPS_TIME, MIN_SAMPLES, MAX_POINTS = 5.0, 1.0, 10, 10_000_000   # :17-20
GAIN_COLORS = {40: (0, 114, 255), 50: (0, 200, 83), 75: (255, 87, 34)}    # :23-27


def subsample(x, y, z, colors, max_points: int):
    """:82-88 — unseeded np.random.choice without replacement when n > max_points."""
    n = x.size
    if n <= max_points:
        return x, y, z, colors, 1
    idx = np.random.choice(n, max_points, replace=False)
    return x[idx], y[idx], z[idx], colors[idx], int(np.ceil(n / max_points))


def process_one(ply_path: Path, out_stem: str, eps: float = EPS_SPACE,
                min_samples: int = MIN_SAMPLES, max_points: int = MAX_POINTS) -> np.ndarray:
    from ..core.loaders import load_ply
    from ..core.writers import write_labels_csv
    from ..processors.clustering import infer_time_from_colors, st_dbscan

    cloud = load_ply(ply_path)
    colors = cloud.colors if cloud.colors is not None else \
        np.full((cloud.size, 3), 180, dtype=np.uint8)            # :75-78 default grey
    x, y, z, colors, stride = subsample(cloud.x, cloud.y, cloud.z, colors, max_points)
    coords = np.column_stack((x, y, z))
    times = infer_time_from_colors(colors, GAIN_COLORS)
    print(f"{ply_path.name}: using {coords.shape[0]:,} points (approx stride={stride})")
    labels = st_dbscan(coords, times, eps_space=eps, eps_time=EPS_TIME, min_samples=min_samples)
    unique, counts = np.unique(labels, return_counts=True)
    print(f"{ply_path.name}: labels summary {dict(zip(unique.tolist(), counts.tolist()))}")
    csv_out = ply_path.with_name(f"{out_stem}_labels.csv")
    write_labels_csv(csv_out, coords, labels)
    print(f"labels CSV -> {csv_out.name}")
    print(f"plot -> {ply_path.with_name(f'{out_stem}_labels.png').name} (not rendered by rpt)")
    return labels


def main(argv=None) -> None:
    here = Path.cwd() / "1.5_Folder"
    p = argparse.ArgumentParser(
        description="Run ST-DBSCAN on stacked PLY point clouds (using gain colors as time steps).")
    p.add_argument("--offset", type=Path, default=here / "frame_stack_v3.ply",
                   help="Path to offset stack PLY.")
    p.add_argument("--flat", type=Path, default=here / "frame_stack_flat_v3.ply",
                   help="Path to flat stack PLY.")
    args = p.parse_args(argv)
    for ply_path, stem in ((args.offset, "frame_stack_v3_dbscan"),
                           (args.flat, "frame_stack_flat_v3_dbscan")):
        if not ply_path.exists():
            print(f"skip: {ply_path} not found")
            continue
        process_one(ply_path, stem)


if __name__ == "__main__":
    main()
