"""Drop-in for ``python PointCloudWorkF/stdbscan_denoising_pipeline.py`` (main :1111-1173):
the same flags and defaults, the same stdout, the same output files (rpt.denoise.run_pipeline).

    python -m rpt.cli.denoise --data-dir D --output-dir O [--max-frames 5] [--eps-space 8]
                              [--eps-time 2] [--min-samples 15] [--min-frames 2] [--no-viz]
                              [--skip-gif] [--no-parallel] [--low-memory]

Without arguments the reference runs its quick mode (:1049-1108: 5 frames from a data
directory next to the script); here that is the default data directory below the working
directory with the same 5-frame default.  The PNG / GIF visualisations are not generated (a note
goes to stderr).
"""
from __future__ import annotations

import argparse
from pathlib import Path

from ..denoise import (DEFAULT_EPS_SPACE, DEFAULT_EPS_TIME, DEFAULT_MIN_FRAMES,
                       DEFAULT_MIN_SAMPLES, run_pipeline)


def build_parser() -> argparse.ArgumentParser:
    cwd = Path.cwd()
    p = argparse.ArgumentParser(description="ST-DBSCAN Radar Point Cloud Denoising Pipeline")
    p.add_argument("--data-dir", type=Path, default=cwd / "(.125NM)data_pattern3(.125NM)",
                   help="Directory containing gain_XX folders")
    p.add_argument("--output-dir", type=Path, default=cwd / "denoising_results",
                   help="Output directory for results")
    p.add_argument("--eps-space", type=float, default=DEFAULT_EPS_SPACE,
                   help=f"Spatial clustering radius in meters (default: {DEFAULT_EPS_SPACE})")
    p.add_argument("--eps-time", type=float, default=DEFAULT_EPS_TIME,
                   help=f"Temporal clustering window in frames (default: {DEFAULT_EPS_TIME})")
    p.add_argument("--min-samples", type=int, default=DEFAULT_MIN_SAMPLES,
                   help=f"Minimum points to form a cluster (default: {DEFAULT_MIN_SAMPLES})")
    p.add_argument("--min-frames", type=int, default=DEFAULT_MIN_FRAMES,
                   help=f"Minimum frames a cluster must span to be valid "
                        f"(default: {DEFAULT_MIN_FRAMES})")
    p.add_argument("--max-frames", type=int, default=5,
                   help="Maximum frames to process (default: 5, 0 = all)")
    p.add_argument("--no-viz", action="store_true", help="Skip visualization generation")
    p.add_argument("--skip-gif", action="store_true", help="Skip GIF generation")
    p.add_argument("--no-parallel", action="store_true", help="Disable parallel CSV loading")
    p.add_argument("--low-memory", action="store_true", help="Memory-efficient mode")
    return p


def main(argv=None) -> None:
    args = build_parser().parse_args(argv)
    run_pipeline(data_dir=args.data_dir, output_dir=args.output_dir, eps_space=args.eps_space,
                 eps_time=args.eps_time, min_samples=args.min_samples,
                 min_frames=args.min_frames, max_frames=args.max_frames, no_viz=args.no_viz,
                 skip_gif=args.skip_gif, parallel=not args.no_parallel,
                 low_memory=args.low_memory)


if __name__ == "__main__":
    main()
