"""Drop-in for the ``radar-pipeline`` click group's ``cluster`` command
(radar-pipeline/src/radar_pipeline/cli/main.py:17-35, 188-253): the same group options
(-c/--config YAML, -v, --version) and the same cluster arguments, with ST-DBSCAN on the MI355X.
The file-management commands of the group (sort-by-gain, filter-range, convert, build,
visualize) and the --plot PNG are outside this engine's scope."""
from __future__ import annotations

import sys
from pathlib import Path
from typing import Optional

import click

from .. import __version__
from ..config import PipelineConfig


@click.group()
@click.option("-c", "--config", type=click.Path(exists=True, path_type=Path),
              help="Path to YAML config file.")
@click.option("-v", "--verbose", count=True, help="Increase verbosity.")
@click.version_option(version=__version__)
@click.pass_context
def cli(ctx: click.Context, config: Optional[Path], verbose: int) -> None:
    """Radar point cloud processing pipeline."""
    ctx.ensure_object(dict)
    ctx.obj["config"] = PipelineConfig.from_yaml(config) if config else PipelineConfig()
    ctx.obj["verbose"] = verbose


@cli.command("cluster")
@click.argument("ply_file", type=click.Path(exists=True, path_type=Path))
@click.option("--output-dir", "-o", type=click.Path(path_type=Path), help="Output directory.")
@click.option("--eps-space", type=float, help="Spatial epsilon.")
@click.option("--eps-time", type=float, help="Temporal epsilon.")
@click.option("--min-samples", type=int, help="Minimum samples per cluster.")
@click.option("--max-points", type=int, help="Maximum points to process.")
@click.option("--plot/--no-plot", default=True, help="Generate PNG visualization.")
@click.pass_context
def cluster(ctx: click.Context, ply_file: Path, output_dir: Optional[Path],
            eps_space: Optional[float], eps_time: Optional[float], min_samples: Optional[int],
            max_points: Optional[int], plot: bool) -> None:
    """Run ST-DBSCAN clustering on point cloud."""
    from ..processors.clustering import process_ply_clustering

    config: PipelineConfig = ctx.obj["config"]
    cc = config.clustering.model_copy()
    for name, val in (("eps_space", eps_space), ("eps_time", eps_time),
                      ("min_samples", min_samples), ("max_points", max_points)):
        if val is not None:
            setattr(cc, name, val)
    if output_dir is None:
        output_dir = ply_file.parent
    csv_path, _ = process_ply_clustering(ply_file, output_dir, cc, config.gains)
    if plot:
        click.echo("note: the --plot PNG is not rendered by rpt", err=True)
    click.echo(f"Clustering complete. Labels saved to {csv_path}")


if __name__ == "__main__":
    cli(sys.argv[1:])
