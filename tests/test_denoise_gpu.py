"""Denoise mode (PointCloudWorkF/stdbscan_denoising_pipeline.py) on the
GPU: rpt_stdbscan_denoise against the reference's own labels (g9) and against the C oracle on
synthetic radar stacks; rpt_label_means against pandas' group mean; the pipeline drop-in against
the reference's run_pipeline outputs (g10: stdout, both binary PLYs, both CSVs), byte-identical."""
from __future__ import annotations

import contextlib
import io
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_denoise_labels_match_reference(gpu, golden):
    from rpt.denoise import st_dbscan

    g = golden("g9_denoise.npz")
    for name in g["names"]:
        eps, et, ms, mf = g[f"{name}_params"]
        lab = st_dbscan(g[f"{name}_xy"], g[f"{name}_t"], eps, et, int(ms), int(mf), device=gpu)
        np.testing.assert_array_equal(lab, g[f"{name}_labels"], err_msg=str(name))


@pytest.mark.parametrize("min_frames,eps_time", [(2, 2.0), (3, 2.0), (1, 1.0), (2, 1.0)])
def test_denoise_matches_oracle_on_radar_stack(gpu, min_frames, eps_time):
    """Points of a synthetic radar stack (K1, no land filter) clustered by the device denoise
    path and by the oracle's FIFO restatement; frames as times, one missing frame id."""
    from rpt.denoise import st_dbscan
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    cfg = SynthConfig(n_frames=6, rows=1024, n_targets=20, clutter_density=0.01)
    ds = DeviceSynth(cfg, gpu)
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(land_filter=False), gpu)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      cfg.n_frames * len(cfg.gains))
    res = pipe.run(ds.echo(), keep_points=True)
    xy = torch.stack([res.points["x"], res.points["y"]], 1)
    t = res.points["frame"].to(torch.float32)
    t = torch.where(t >= 3, t + 1, t)  # a gap in the frame ids
    lab = st_dbscan(xy, t, 8.0, eps_time, 15, min_frames).cpu().numpy()
    ref = oracle.stdbscan_denoise(xy.cpu().numpy(), t.cpu().numpy(), 8.0, eps_time, 15,
                                  min_frames)
    assert (ref >= 0).sum() > 1000
    np.testing.assert_array_equal(lab, ref)


def test_denoise_float_times_and_edges(gpu):
    from rpt.denoise import st_dbscan

    rng = np.random.default_rng(3)
    xy = (rng.random((3000, 2)) * 60).astype(np.float32)
    t = (rng.integers(0, 6, 3000) + rng.random(3000) * 0.8).astype(np.float32)
    for et, ms, mf in ((1.5, 6, 2), (0.5, 4, 2), (2.0, 10, 3), (2.0, 0, 0)):
        np.testing.assert_array_equal(st_dbscan(xy, t, 5.0, et, ms, mf, device=gpu),
                                      oracle.stdbscan_denoise(xy, t, 5.0, et, ms, mf))
    # empty input: no labels, no error (:286-287)
    assert st_dbscan(np.zeros((0, 2), np.float32), np.zeros(0, np.float32), 8.0, 2.0, 15,
                     2, device=gpu).shape == (0,)
    # no pair passes: all noise, or singletons when nothing is required
    assert (st_dbscan(xy, t, -1.0, 2.0, 3, 2, device=gpu) == -1).all()
    np.testing.assert_array_equal(st_dbscan(xy, t, -1.0, 2.0, 0, 0, device=gpu),
                                  np.arange(3000, dtype=np.int32))
    # the distinct-frame list holds 256 frames: more min_frames with eps_time > 30 is refused
    with pytest.raises(NotImplementedError):
        st_dbscan(xy, t, 5.0, 40.0, 5, 257, device=gpu)


@pytest.mark.parametrize("eps_time,min_frames,float_t", [(40.0, 2, False), (45.5, 5, False),
                                                          (120.0, 30, False), (31.0, 3, True),
                                                          (64.0, 70, False)])
def test_denoise_wide_time_window(gpu, eps_time, min_frames, float_t):
    """eps_time > 30 (the distinct int32(t) frames as a wave-wide list instead of a 64-bit offset
    set, k_frames_points_list): buoys seen in a random subset of 200 frames, clutter, a NaN
    time; against the oracle's FIFO restatement (:264-369)."""
    from rpt.denoise import st_dbscan

    rng = np.random.default_rng(int(eps_time * 10) + min_frames)
    pts, ts = [], []
    for c in rng.random((25, 2)) * 300:
        fr = np.sort(rng.choice(200, rng.integers(20, 120), replace=False))
        k = rng.integers(1, 4, len(fr))
        pts.append(np.repeat(c[None], k.sum(), 0) + rng.normal(0, 1.5, (k.sum(), 2)))
        ts.append(np.repeat(fr, k))
    pts.append(rng.random((3000, 2)) * 300)
    ts.append(rng.integers(0, 200, 3000))
    xy = np.vstack(pts).astype(np.float32)
    t = np.concatenate(ts).astype(np.float32)
    if float_t:
        t = (t + rng.random(len(t)).astype(np.float32) * 0.9).astype(np.float32)
    t[::997] = np.nan
    perm = rng.permutation(len(t))
    xy, t = xy[perm], t[perm]
    lab = st_dbscan(xy, t, 5.0, eps_time, 12, min_frames, device=gpu)
    ref = oracle.stdbscan_denoise(xy, t, 5.0, eps_time, 12, min_frames)
    assert (ref >= 0).sum() > 500
    np.testing.assert_array_equal(lab, ref)


@pytest.mark.parametrize("eps_time,min_frames", [(40.0, 6), (2.0, 4)])
def test_denoise_wide_slabs(gpu, eps_time, min_frames):
    """Long runs of frames over a small region: the grid's cell cap (max(2^22, 4n) cells) widens
    the slabs to two frames each (ct = 2), so a cell wholly inside eps can hold points of two
    frames and must not be counted as one (k_frames_points / k_frames_points_list)."""
    from rpt.denoise import st_dbscan

    rng = np.random.default_rng(7)
    n_frames = 200_000
    pts, ts = [], []
    for c in rng.random((400, 2)) * 30:
        f0 = int(rng.integers(0, n_frames - 12))
        fr = np.repeat(np.arange(f0, f0 + 10), 2)   # two returns per frame, 10 frames
        pts.append(c + rng.normal(0, 0.5, (len(fr), 2)))
        ts.append(fr)
    pts.append(rng.random((20_000, 2)) * 30)
    ts.append(rng.integers(0, n_frames, 20_000))
    xy = np.vstack(pts).astype(np.float32)
    t = np.concatenate(ts).astype(np.float32)
    perm = rng.permutation(len(t))
    xy, t = xy[perm], t[perm]
    lab = st_dbscan(xy, t, 8.0, eps_time, 4, min_frames, device=gpu)
    ref = oracle.stdbscan_denoise(xy, t, 8.0, eps_time, 4, min_frames)
    assert (ref >= 0).sum() > 2000
    np.testing.assert_array_equal(lab, ref)


def test_label_means_match_pandas_group_mean(gpu):
    """rpt_label_means = pandas groupby mean of float32 columns (Kahan-compensated float32)."""
    import pandas as pd

    from rpt.denoise import cluster_table

    rng = np.random.default_rng(8)
    n = 200_000
    lab = rng.integers(-1, 300, n).astype(np.int32)
    lab[rng.random(n) < 0.2] = 7  # one large group
    x = (rng.normal(0, 1, n) * 150 + 30).astype(np.float32)
    y = (rng.random(n) * 1e4).astype(np.float32)
    v = (rng.random(n) * 255).astype(np.float32)
    keep = lab >= 0
    ref = pd.DataFrame({"cluster_id": lab[keep], "x": x[keep], "y": y[keep],
                        "intensity": v[keep]}).groupby("cluster_id").agg(
        num_points=("x", "count"), centroid_x=("x", "mean"), centroid_y=("y", "mean"),
        mean_intensity=("intensity", "mean")).reset_index()
    T = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
    got = cluster_table(T(lab), T(x), T(y), T(v), int(lab.max()) + 1)
    assert ref.to_csv(index=False) == got.to_csv(index=False)


def test_denoise_pipeline_matches_reference_outputs(tmp_path, golden):
    sys.path.insert(0, str(GOLDEN))
    from make_golden import synth_csv_stack

    from rpt.denoise import run_pipeline

    g = golden("g10_denoise_pipeline.npz")
    data = synth_csv_stack(tmp_path / "stack")
    out = tmp_path / "out"
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        run_pipeline(data, out, eps_space=8.0, eps_time=2.0, min_samples=15, min_frames=2,
                     max_frames=0, no_viz=True, parallel=False)
    ref_out = str(g["stdout"])
    ref_dir = [l for l in ref_out.splitlines() if l.startswith("Results saved to: ")][0]
    ref_dir = ref_dir[len("Results saved to: "):]
    assert buf.getvalue().replace(str(out), "<OUT>") == ref_out.replace(ref_dir, "<OUT>")
    for name in ("denoised_point_cloud.ply", "raw_point_cloud.ply"):
        assert (out / name).read_bytes() == bytes(g[name.replace(".", "_")]), name
    for name in ("denoising_stats.csv", "clusters.csv"):
        assert (out / name).read_text() == str(g[name.replace(".", "_")]), name


def test_denoise_pipeline_malformed_files_parallel(tmp_path, golden):
    """g11 through the denoise drop-in with parallel loading (> 4 frames, :905-907): the
    genfromtxt-first loader (:104-119) -- a comment line skipped, empty fields and an empty
    Scale read as 0.0, a one-row file an empty sweep -- and a file whose load raises (a
    too-long row: genfromtxt raises, then read_csv's tokenizing error) failing its whole frame
    with load_frames_parallel's warning (:248-251); stdout, PLYs and CSVs byte-identical."""
    sys.path.insert(0, str(GOLDEN))
    from make_golden import corrupt_csv_stack

    from rpt.denoise import run_pipeline

    g = golden("g11_corrupt.npz")
    data = corrupt_csv_stack(tmp_path / "dstack", denoise=True)
    out = tmp_path / "dout"
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        run_pipeline(data, out, eps_space=8.0, eps_time=2.0, min_samples=15, min_frames=2,
                     max_frames=0, no_viz=True, parallel=True)
    ref_out = str(g["denoise_stdout"])
    ref_dir = [l for l in ref_out.splitlines() if l.startswith("Results saved to: ")][0]
    ref_dir = ref_dir[len("Results saved to: "):]
    assert "Warning: Failed to load frame 3" in buf.getvalue()
    assert buf.getvalue().replace(str(out), "<OUT>") == ref_out.replace(ref_dir, "<OUT>")
    for name in ("denoised_point_cloud.ply", "raw_point_cloud.ply"):
        assert (out / name).read_bytes() == bytes(g["denoise_" + name.replace(".", "_")]), name
    for name in ("denoising_stats.csv", "clusters.csv"):
        assert (out / name).read_text() == str(g["denoise_" + name.replace(".", "_")]), name


def test_denoise_loader_other_bin_counts(gpu, tmp_path):
    """The genfromtxt loader takes num_bins from the file (data[:, 5:], :128-134): a sweep of 512
    echo columns has range resolution Scale / 512; a file of only Status..Angle has no echo
    column and no point.  Points of every file in frame / file order against the reference's
    arithmetic on np.genfromtxt's array (oracle.path.polar_scatter)."""
    sys.path.insert(0, str(GOLDEN))
    from make_golden import echo_block, write_csv

    from oracle.path import polar_scatter, trig_tables
    from rpt.denoise import load_frames

    rng = np.random.default_rng(11)
    rows = 40
    frames, expect = [], []
    for f in range(3):
        fr = {}
        for k, (g, bins) in enumerate(((40, 1024), (50, 512 if f == 1 else 1024),
                                       (75, 0 if f == 2 else 1024))):
            p = tmp_path / f"f{f}_g{g}.csv"
            scale = rng.uniform(500, 2000, rows).astype(np.float32)
            angle = np.sort(rng.choice(8196, rows, replace=False))
            if bins:
                write_csv(p, 1, scale, 0, g, angle, echo_block(rng, rows, bins))
            else:   # Status..Angle only
                p.write_text("Status,Scale,Range,Gain,Angle\n" + "".join(
                    f"1,{scale[r]:g},0,{g},{angle[r]}\n" for r in range(rows)))
            fr[k] = p
            if bins:
                data = np.genfromtxt(p, delimiter=",", skip_header=1, dtype=np.float32,
                                     filling_values=0.0)
                c, s = trig_tables(data[:, 4])
                xs, ys, vs = polar_scatter(data[:, 5:], data[:, 1], c, s)
                expect.append((xs, ys, vs, np.full(len(xs), f, np.float32)))
        frames.append(fr)
    got = load_frames(frames, device=gpu)
    for k, name in enumerate(("x", "y", "z", "t")):
        np.testing.assert_array_equal(getattr(got, name).cpu().numpy(),
                                      np.concatenate([e[k] for e in expect]), err_msg=name)
    assert got.frame_counts.tolist() == [sum(len(e[0]) for e in expect if e[3][:1].tolist() == [f])
                                         for f in range(3)]
