"""Drop-in for ``python PointCloudWork/4_temporal_object_tracker.py`` (main :1041-1101,
run_pipeline :893-1038): the same flags, the same stdout lines and the same three output CSVs,
with the compute stages on the MI355X (rpt_stack_run: K1 polar scatter + fusion, land filter,
ST-DBSCAN, per-(frame, label) summaries) and the cluster order + tracker in librpt's host C++.

    python -m rpt.cli.tracker --data-dir D --output-dir O [--max-frames M] [--no-land-filter]
                              [--no-viz] [--eps-space 8] [--eps-time 2] [--min-samples 15]
                              [--intensity-threshold 10]

Kept quirks of the reference: --intensity-threshold is accepted and ignored (the loader uses the
INTENSITY_THRESHOLD constant, :896 vs :221); the land gate counts built frames (:954); object
counts print for frame ids divisible by 50 (:990-991).  The PNG visualisations (:1012-1035) are
not built (matplotlib rendering is outside this engine's scope): without --no-viz a note goes
to stderr and stdout is that of a --no-viz run.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path
from typing import List, Optional

import numpy as np

EPS_SPACE, EPS_TIME, MIN_SAMPLES, INTENSITY_THRESHOLD = 8.0, 2.0, 15, 10.0   # :75-77, :70
LAND_FILTER_MIN_FRAMES = 10                                                  # :954


def run_pipeline(data_dir: Path, output_dir: Path, max_frames: int = 0,
                 skip_land_filter: bool = False, visualize: bool = True,
                 eps_space: float = EPS_SPACE, eps_time: float = EPS_TIME,
                 min_samples: int = MIN_SAMPLES, intensity_threshold: float = INTENSITY_THRESHOLD,
                 device=None, csv_threads: int = 0) -> Optional[dict]:
    """run_pipeline (:893-1038).  Returns a summary dict (None when no data file is found)."""
    from ..core.discovery import discover_files, group_files_by_frame
    from ..core.writers import save_tracking_results
    from ..frames import load_frame_stack
    from ..native_tracker import NativeTracker
    from ..pipeline import FrameStackPipeline, PathParams
    from ..stages import order_frames

    del intensity_threshold  # accepted, unused: the reference thresholds at the constant (:221)
    data_dir, output_dir = Path(data_dir), Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    print("=" * 60)
    print("TEMPORAL OBJECT TRACKING PIPELINE")
    print("=" * 60)

    print("\n[1/6] Discovering data files...")
    files_by_gain = discover_files(data_dir)
    if not files_by_gain:
        print("ERROR: No valid data files found!")
        return None
    for gain, files in files_by_gain.items():
        print(f"  Gain {gain}: {len(files)} files")

    print("\n[2/6] Grouping files into temporal frames...")
    frame_files = group_files_by_frame(files_by_gain)
    print(f"  Found {len(frame_files)} frames")
    if max_frames > 0:
        frame_files = frame_files[:max_frames]
        print(f"  Processing first {len(frame_files)} frames")

    print("\n[3/6] Building point cloud frames...")
    import torch

    dev = torch.device("cuda", 0) if device is None else torch.device(device)
    errors: List[tuple] = []
    stack = load_frame_stack(frame_files, dev, threads=csv_threads,
                             on_error=lambda p, e: errors.append((p, e)))
    # build_frame's per-file "Error loading" lines (:194) interleave with the progress lines
    frame_of = {Path(p): i for i, ff in enumerate(frame_files) for p in ff.values()}
    by_frame = {}
    for p, e in errors:
        by_frame.setdefault(frame_of[Path(p)], []).append((p, e))
    F = len(frame_files)
    for i in range(F):
        for p, e in by_frame.get(i, []):
            print(f"Error loading {p}: {e}")
        if (i + 1) % 50 == 0:
            print(f"  Processed {i + 1}/{F} frames...")
    params = PathParams(eps_space=float(eps_space), eps_time=float(eps_time),
                        min_samples=int(min_samples), land_filter=not skip_land_filter)
    pipe = FrameStackPipeline(stack.gains, stack.rows, 1024, params, dev)
    pipe.set_geometry(stack.scale, stack.cos_t, stack.sin_t, F * len(stack.gains))
    res = pipe.run(stack.echo)          # K1 .. K9 on the device (ValueError like BallTree's)
    built = [int(f) for f in res.frame_ids]
    total_points = res.n_points
    print(f"  Built {len(built)} frames")
    print(f"  Total points: {total_points:,}")

    if not skip_land_filter and len(built) > LAND_FILTER_MIN_FRAMES:
        print("\n[4/6] Building land filter...")
        print(f"  Identified {res.n_land_cells} land cells")
        print("  Filtering land from frames...")
        removed = total_points - res.n_clustered_input
        print(f"  Removed {removed:,} land points ({100 * removed / total_points:.1f}%)")
    else:
        print("\n[4/6] Skipping land filter")

    print("\n[5/6] Running ST-DBSCAN clustering...")
    seg = res.seg
    fo, order = order_frames(F, seg, res.first_noise)
    with_clusters = [f for f in built if fo[f + 1] > fo[f]]
    print(f"  Found {res.n_segments} clusters across {len(with_clusters)} frames")

    print("\n[6/6] Tracking objects...")
    trk = NativeTracker(params.max_association_distance, params.max_missed_frames,
                        params.motion_history_frames, params.stationary_velocity_threshold)
    for f in built:
        sel = order[fo[f]:fo[f + 1]]
        n_obj = trk.update_arrays(f, seg["cx"][sel], seg["cy"][sel])
        if f % 50 == 0:
            print(f"  Frame {f}: {n_obj} active objects")

    print("\n" + "=" * 60)
    print("TRACKING RESULTS")
    print("=" * 60)
    objects = trk.objects()
    kinds = [o.object_type for o in objects]
    print(f"  Total objects tracked: {len(objects)}")
    print(f"  Buoys (stationary): {kinds.count('buoy')}")
    print(f"  Boats (moving): {kinds.count('boat')}")
    print(f"  Unknown: {kinds.count('unknown')}")

    print("\nSaving results...")
    rows = [(f, int(seg["label"][s]), int(seg["count"][s]), seg["cx"][s], seg["cy"][s],
             float(seg["mi"][s])) for f in with_clusters for s in order[fo[f]:fo[f + 1]]]
    save_tracking_results(objects, rows, output_dir)

    if visualize:
        print("note: visualisations (frame PNGs, tracking summary) are not produced by rpt; "
              "results match a --no-viz run", file=sys.stderr)
    print("\nPipeline complete!")
    print(f"Results saved to: {output_dir}")
    return {"frames": F, "built": len(built), "points": total_points,
            "clusters": res.n_segments, "objects": len(objects)}


def build_parser() -> argparse.ArgumentParser:
    """The reference's flags (:1057-1088), same names, defaults and types."""
    here = Path(__file__).resolve().parent
    ap = argparse.ArgumentParser(
        description="Track objects in radar point cloud time series",
        formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data-dir", type=Path, default=here / "data",
                    help="Directory containing gain subdirectories")
    ap.add_argument("--output-dir", type=Path, default=Path.cwd() / "tracking_results",
                    help="Output directory for results")
    ap.add_argument("--max-frames", type=int, default=0,
                    help="Maximum frames to process (0 = all)")
    ap.add_argument("--no-land-filter", action="store_true", help="Skip land filtering step")
    ap.add_argument("--no-viz", action="store_true", help="Skip visualization generation")
    ap.add_argument("--eps-space", type=float, default=EPS_SPACE,
                    help=f"Spatial clustering radius (default: {EPS_SPACE})")
    ap.add_argument("--eps-time", type=float, default=EPS_TIME,
                    help=f"Temporal clustering window (default: {EPS_TIME})")
    ap.add_argument("--min-samples", type=int, default=MIN_SAMPLES,
                    help=f"Min points per cluster (default: {MIN_SAMPLES})")
    ap.add_argument("--intensity-threshold", type=float, default=INTENSITY_THRESHOLD,
                    help=f"Minimum intensity threshold (default: {INTENSITY_THRESHOLD})")
    ap.add_argument("--device", default=None, help="rpt: torch device (default cuda:0)")
    return ap


def main(argv=None) -> None:
    a = build_parser().parse_args(argv)
    run_pipeline(data_dir=a.data_dir, output_dir=a.output_dir, max_frames=a.max_frames,
                 skip_land_filter=a.no_land_filter, visualize=not a.no_viz,
                 eps_space=a.eps_space, eps_time=a.eps_time, min_samples=a.min_samples,
                 intensity_threshold=a.intensity_threshold, device=a.device)


if __name__ == "__main__":
    main()
