"""§8(f) rank 3 on the GPU: the PLY ST-DBSCAN drop-ins (3_stdbscan_point_clouds.py process_one and
radar_pipeline process_ply_clustering -> labels CSV + stdout) and fuse_gains_max, against the
reference's own outputs (tests/golden/g7_ply.npz, g8_fuse_max.npz; inputs regenerated from the
same seeds by tests/golden/make_golden.py's generators)."""
from __future__ import annotations

import contextlib
import io
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLDEN))


def _lines(text):
    # the reference's matplotlib PNG line is the one rpt does not render
    return [l for l in text.splitlines() if not l.startswith("plot -> ")]


def test_3_stdbscan_process_one_matches_reference(tmp_path, golden):
    from make_golden import synth_ply

    from rpt.cli.stdbscan_ply import process_one

    g = golden("g7_ply.npz")
    for k, (seed, col) in enumerate(((707, True), (708, True), (709, False))):
        d = tmp_path / f"c{k}"
        d.mkdir()
        ply = synth_ply(d / "stack.ply", seed, with_color=col)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            process_one(ply, "stack_dbscan")
        assert _lines(buf.getvalue()) == _lines(str(g[f"c{k}_script_stdout"]))
        assert (d / "stack_dbscan_labels.csv").read_text() == str(g[f"c{k}_script_csv"])


def test_radar_pipeline_cluster_cli_matches_reference(tmp_path, golden):
    from click.testing import CliRunner
    from make_golden import synth_ply

    from rpt.cli.main import cli

    g = golden("g7_ply.npz")
    for k, seed in enumerate((707, 708)):
        d = tmp_path / f"c{k}"
        d.mkdir()
        ply = synth_ply(d / "stack.ply", seed)
        out = d / "pkg"
        out.mkdir()
        r = CliRunner().invoke(cli, ["cluster", str(ply), "-o", str(out), "--no-plot"])
        assert r.exit_code == 0, r.output
        assert (out / "stack_dbscan_labels.csv").read_text() == str(g[f"c{k}_pkg_csv"])
        exp = str(g[f"c{k}_pkg_stdout"]).splitlines()
        assert r.output.splitlines()[:len(exp)] == exp
        assert r.output.splitlines()[-1].startswith("Clustering complete. Labels saved to ")


def test_fuse_gains_max_matches_reference(tmp_path, golden):
    from make_golden import synth_fuse_frames

    from rpt.processors.fusion import fuse_gains_max

    g = golden("g8_fuse_max.npz")
    frames = synth_fuse_frames(tmp_path / "fuse")
    for f, ff in enumerate(frames):
        for res in (1.0, 2.5):
            key = f"f{f}_r{str(res).replace('.', '_')}"
            x, y, i = fuse_gains_max(ff, grid_resolution=res)
            np.testing.assert_array_equal(x, g[key + "_x"])
            np.testing.assert_array_equal(y, g[key + "_y"])
            np.testing.assert_array_equal(i, g[key + "_i"])
            assert x.dtype == np.float64 and i.dtype == np.float32
