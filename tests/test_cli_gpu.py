"""The tracker CLI drop-in end to end against the reference's own run_pipeline outputs
(tests/golden/g6_pipeline.npz: stdout + tracked_objects.csv + trajectories.csv + clusters.csv
of PointCloudWork/4_temporal_object_tracker.py run_pipeline on a 12-frame synthetic CSV stack,
regenerated here from the same seed): native CSV ingest -> device path -> host tracker ->
pandas writers, byte-identical."""
from __future__ import annotations

import contextlib
import io
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"


def _norm(text: str, out_dir: str) -> list:
    """The reference printed its own temp output dir, and discover_files lists gains in directory
    iteration order (file-system dependent): replace the one, sort the gain lines."""
    lines = text.replace(out_dir, "<OUT>").splitlines()
    gain = sorted(l for l in lines if l.startswith("  Gain "))
    it = iter(gain)
    return [next(it) if l.startswith("  Gain ") else l for l in lines]


def test_tracker_cli_matches_reference_run_pipeline(tmp_path, golden):
    sys.path.insert(0, str(GOLDEN))
    from make_golden import synth_csv_stack

    from rpt.cli.tracker import run_pipeline

    g = golden("g6_pipeline.npz")
    data = synth_csv_stack(tmp_path / "stack")
    out = tmp_path / "out"
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        run_pipeline(data, out, visualize=False)
    ref_out = str(g["stdout"])
    ref_dir = [l for l in ref_out.splitlines() if l.startswith("Results saved to: ")][0]
    ref_dir = ref_dir[len("Results saved to: "):]
    assert _norm(buf.getvalue(), str(out)) == _norm(ref_out, ref_dir)
    for name in ("tracked_objects", "trajectories", "clusters"):
        assert (out / f"{name}.csv").read_text() == str(g[name]), name


def _ref_root(text: str, marker: str) -> str:
    """The reference's temp data root, from its first line naming a file under it."""
    for l in text.splitlines():
        if marker in l and "/gain_" in l:
            return l[l.index("/"):l.index("/gain_")]
    return "\0"


def test_tracker_cli_malformed_files_match_reference(tmp_path, golden):
    """g11: a file with a too-long row (read_csv's tokenizing error: "Error loading {path}: {e}"
    with pandas' text, printed while frames build, :193-194), a one-row file, a comment line and
    empty echo fields (pandas reads the comment as a short row and NaN, fillna(0))."""
    sys.path.insert(0, str(GOLDEN))
    from make_golden import corrupt_csv_stack

    from rpt.cli.tracker import run_pipeline

    g = golden("g11_corrupt.npz")
    data = corrupt_csv_stack(tmp_path / "stack")
    out = tmp_path / "out"
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        run_pipeline(data, out, visualize=False)
    ref_out = str(g["tracker_stdout"])
    ref_dir = [l for l in ref_out.splitlines() if l.startswith("Results saved to: ")][0]
    ref_dir = ref_dir[len("Results saved to: "):]
    ref_out = ref_out.replace(_ref_root(ref_out, "Error loading"), "<DATA>")
    got = buf.getvalue().replace(str(data), "<DATA>")
    assert "Error loading <DATA>/gain_50/" in got
    assert _norm(got, str(out)) == _norm(ref_out, ref_dir)
    for name in ("tracked_objects", "trajectories", "clusters"):
        assert (out / f"{name}.csv").read_text() == str(g["tracker_" + name]), name


def test_tracker_cli_flags_and_max_frames(tmp_path):
    """argparse surface (:1057-1088): --max-frames truncates the grouped frames (:933-935),
    --no-land-filter skips the filter, --intensity-threshold is accepted and ignored."""
    sys.path.insert(0, str(GOLDEN))
    from make_golden import synth_csv_stack

    from rpt.cli.tracker import main

    data = synth_csv_stack(tmp_path / "stack")
    outs = {}
    for tag, extra in (("a", []), ("b", ["--intensity-threshold", "99"]),
                       ("c", ["--max-frames", "5"]), ("d", ["--no-land-filter"])):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            main(["--data-dir", str(data), "--output-dir", str(tmp_path / tag), "--no-viz",
                  *extra])
        outs[tag] = buf.getvalue()
    for name in ("tracked_objects", "trajectories", "clusters"):
        assert (tmp_path / "a" / f"{name}.csv").read_text() == \
            (tmp_path / "b" / f"{name}.csv").read_text()
    assert "Processing first 5 frames" in outs["c"] and "Built 5 frames" in outs["c"]
    assert "[4/6] Skipping land filter" in outs["c"] and "[4/6] Skipping land filter" in outs["d"]
    assert "Identified" in outs["a"]
