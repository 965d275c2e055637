#!/usr/bin/env python3
"""Generate the golden parity fixtures by RUNNING THE REFERENCE in the build container.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Refuses to run unless /root/reference exists (the reference never travels to the GPU box; only
the .npz vectors written here do).  Inputs are generated from fixed seeds below, so the files
are reproducible.  Outputs (all in tests/golden/):

  g1_polar.npz      load_radar_csv (4_temporal_object_tracker.py:184-232) on small sweeps written
                    as CSV, build_frame (:312-352) fusion, radar_pipeline load_radar_csv +
                    sweep_to_point_cloud (core/loaders.py:46-101, core/transforms.py:37-79)
  g2_stdbscan.npz   st_dbscan labels (3_stdbscan_point_clouds.py:101-136) on random, lattice,
                    blob and float-time clouds, D=2 and D=3, plus the Rust KAT inputs
                    (radar-pipeline-rs/src/processors/clustering.rs:470-597)
  g3_land.npz       build_occupancy_grid / identify_land_cells / filter_land_from_frame on a
                    12-frame stack (:359-436)
  g4_clusters.npz   st_dbscan(frames) per-frame Cluster lists in reference order (:443-536)
  g5_tracker.npz    ObjectTracker.update sequences (:543-688)
  g6_pipeline.npz   run_pipeline (:893-1038) CSV outputs on a 12-frame synthetic CSV stack
  g7_ply.npz        3_stdbscan_point_clouds.process_one (:174-193) and radar_pipeline
                    process_ply_clustering (processors/clustering.py:157-208) on synthetic PLY
                    stacks (labels CSV text + stdout)
  g8_fuse_max.npz   5_gain_fusion_ply_builder.fuse_gains_max (:222-273) on small CSV frames
  g9_denoise.npz    PointCloudWorkF/stdbscan_denoising_pipeline.st_dbscan (:264-369: min_frames
                    core condition, FIFO expansion) on blob / lattice / float-time clouds
  g10_denoise_pipeline.npz
                    stdbscan_denoising_pipeline.run_pipeline (:862-1046, no_viz) on a synthetic
                    CSV stack: stdout, both binary PLYs, denoising_stats.csv, clusters.csv
  g11_corrupt.npz   the tracker's run_pipeline and the denoise run_pipeline (parallel loading)
                    on a CSV stack with malformed files (corrupt_csv_stack): a tokenizing error,
                    a one-row file, a comment line, empty fields, an empty Scale field
  meta.json         library versions / CPU of the generating run

    python tests/golden/make_golden.py [g7 g8 ...]   # only the named fixtures
"""
from __future__ import annotations

import importlib.util
import io
import json
import os
import platform
import sys
import tempfile
from contextlib import redirect_stdout
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.dont_write_bytecode = True


def _load(name: str, path: Path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod  # dataclasses + `from __future__ import annotations` need this
    spec.loader.exec_module(mod)
    return mod


def write_csv(path: Path, status, scale, rng_col, gain, angle, echo):
    hdr = "Status,Scale,Range,Gain,Angle," + ",".join(f"Echo_{i}" for i in range(echo.shape[1]))
    lines = [hdr]
    for r in range(echo.shape[0]):
        lines.append(f"{status},{scale[r]:g},{rng_col},{gain},{angle[r]}," +
                     ",".join(str(int(v)) for v in echo[r]))
    path.write_text("\n".join(lines) + "\n")


def echo_block(rng, rows, bins, p_keep=0.08):
    e = np.zeros((rows, bins), dtype=np.int64)
    m = rng.random((rows, bins)) < p_keep
    e[m] = rng.integers(0, 256, m.sum())
    # a few exact-threshold values (10 is dropped, 11 kept)
    e[rng.random((rows, bins)) < 0.01] = 10
    e[rng.random((rows, bins)) < 0.01] = 11
    return e


def g1_polar(trk, rp_loaders, rp_transforms, tmp: Path):
    rng = np.random.default_rng(101)
    rec = {}
    files = {}
    for k, (gain, rows) in enumerate([(40, 96), (50, 80), (75, 64)]):
        angle = np.sort(rng.choice(8196, rows, replace=False)).astype(np.int64)
        scale = rng.choice([231.5, 463.0, 115.75, 496.0], rows).astype(np.float64)
        echo = echo_block(rng, rows, 1024)
        d = tmp / f"gain_{gain}"
        d.mkdir(parents=True, exist_ok=True)
        p = d / f"20250813_142602_{100 + k:03d}.csv"
        write_csv(p, 1, scale, 0, gain, angle, echo)
        files[gain] = p
        x, y, inten, g = trk.load_radar_csv(p)
        rec[f"f{k}_echo"] = echo.astype(np.uint8)
        rec[f"f{k}_scale"] = scale.astype(np.float32)
        rec[f"f{k}_angle"] = angle.astype(np.float32)
        rec[f"f{k}_gain"] = np.int32(g)
        rec[f"f{k}_x"], rec[f"f{k}_y"], rec[f"f{k}_i"] = x, y, inten
        # package form: RadarSweep + sweep_to_point_cloud with default ProcessingConfig
        sw = rp_loaders.load_radar_csv(p)
        pc = rp_transforms.sweep_to_point_cloud(sw)
        rec[f"f{k}_pkg_x"], rec[f"f{k}_pkg_y"], rec[f"f{k}_pkg_z"] = pc.x, pc.y, pc.z
        rec[f"f{k}_pkg_ranges"] = sw.ranges
        rec[f"f{k}_pkg_angles"] = sw.angles_rad
    fr = trk.build_frame(files, 7)
    rec["frame_points"] = fr.points
    rec["frame_gains"] = fr.gains
    rec["frame_id"] = np.int64(fr.frame_id)
    np.savez_compressed(OUT / "g1_polar.npz", **rec)


def _cloud_cases():
    rng = np.random.default_rng(202)
    cases = []
    # random 2-D clouds over integer frames
    for k in range(10):
        n = int(rng.integers(200, 1500))
        F = int(rng.integers(1, 6))
        xy = (rng.random((n, 2)) * rng.choice([30, 60, 120])).astype(np.float32)
        t = rng.integers(0, F, n).astype(np.float32)
        eps = float(rng.choice([1.0, 2.0, 3.0, 5.0, 8.0]))
        et = float(rng.choice([0.0, 1.0, 2.0]))
        ms = int(rng.choice([1, 2, 3, 5, 10, 15]))
        cases.append(("rand2d", xy, t, eps, et, ms))
    # integer lattice: exact-boundary distances
    for k in range(5):
        s = int(rng.integers(8, 25))
        gx, gy = np.meshgrid(np.arange(s), np.arange(s))
        xy = np.column_stack([gx.ravel(), gy.ravel()]).astype(np.float32) * float(rng.choice([1, 2, 3]))
        keep = rng.random(len(xy)) < 0.7
        xy = xy[keep]
        t = rng.integers(0, 3, len(xy)).astype(np.float32)
        eps = float(rng.choice([1.0, 2.0, 3.0, 4.0, 5.0]))
        cases.append(("lattice", xy, t, eps, float(rng.choice([0.0, 1.0])), int(rng.choice([2, 3, 4, 5]))))
    # dense blobs + sparse noise over frames (tracker-like)
    for k in range(6):
        F = 6
        pts, ts = [], []
        centers = rng.random((5, 2)) * 200 - 100
        vel = rng.normal(0, 1.5, (5, 2))
        for f in range(F):
            for c, v in zip(centers, vel):
                m = int(rng.integers(20, 80))
                pts.append(c + v * f + rng.normal(0, 2.0, (m, 2)))
                ts.append(np.full(m, f))
            m = 60
            pts.append(rng.random((m, 2)) * 240 - 120)
            ts.append(np.full(m, f))
        xy = np.vstack(pts).astype(np.float32)
        t = np.concatenate(ts).astype(np.float32)
        cases.append(("blobs", xy, t, float(rng.choice([5.0, 8.0])), 2.0, int(rng.choice([8, 15]))))
    # float times, non-integral eps_time
    for k in range(4):
        n = 800
        xy = (rng.random((n, 2)) * 40).astype(np.float32)
        t = (rng.random(n) * 5).astype(np.float32)
        cases.append(("floattime", xy, t, 3.0, float(rng.choice([0.5, 1.25, 0.3])), 4))
    # D=3 PLY-like stacks, time from colour in {0,1,2}
    for k in range(5):
        n = int(rng.integers(300, 1200))
        xyz = np.column_stack([rng.random(n) * 50, rng.random(n) * 50,
                               rng.integers(11, 255, n).astype(np.float64) / 10]).astype(np.float32)
        t = rng.integers(0, 3, n).astype(np.float32)
        cases.append(("ply3d", xyz, t, float(rng.choice([3.0, 5.0])), 1.0, int(rng.choice([5, 10]))))
    # Rust KATs (clustering.rs:470-597) replayed
    sq = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0], [100, 100, 0], [101, 100, 0],
                   [100, 101, 0], [101, 101, 0]], np.float32)
    cases.append(("kat_squares", sq, np.zeros(8, np.float32), 5.0, 1.0, 2))
    cases.append(("kat_temporal", sq[:4], np.array([0, 0, 5, 5], np.float32), 5.0, 1.0, 2))
    cases.append(("kat_noise", np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [100, 100, 100]],
                                        np.float32), np.zeros(4, np.float32), 5.0, 1.0, 3))
    cases.append(("kat_single", np.zeros((1, 3), np.float32), np.zeros(1, np.float32), 5.0, 1.0, 2))
    # min_samples edge cases
    xy = (rng.random((300, 2)) * 20).astype(np.float32)
    t = rng.integers(0, 2, 300).astype(np.float32)
    cases.append(("ms0", xy, t, 2.0, 1.0, 0))
    cases.append(("ms1", xy, t, 2.0, 1.0, 1))
    return cases


def g2_stdbscan(ref3):
    rec = {}
    cases = _cloud_cases()
    for k, (kind, c, t, eps, et, ms) in enumerate(cases):
        lab = ref3.st_dbscan(c, t, eps_space=eps, eps_time=et, min_samples=ms)
        rec[f"c{k}_coords"] = c
        rec[f"c{k}_times"] = t
        rec[f"c{k}_params"] = np.array([eps, et, ms], dtype=np.float64)
        rec[f"c{k}_labels"] = lab
        rec[f"c{k}_kind"] = np.array(kind)
    rec["n_cases"] = np.int64(len(cases))
    np.savez_compressed(OUT / "g2_stdbscan.npz", **rec)
    return len(cases)


def _frames_stack(trk, rng, F=12, with_land=True, n_blobs=6, gap_at=None):
    frames = []
    centers = rng.random((n_blobs, 2)) * 300 - 150
    vel = rng.normal(0, 1.2, (n_blobs, 2))
    vel[: n_blobs // 2] *= 0.05  # half nearly stationary
    for f in range(F):
        if gap_at is not None and f == gap_at:
            continue
        xs, ys, ii, gg = [], [], [], []
        for gi, g in enumerate((40, 50, 75)):
            pts = []
            vals = []
            for c, v in zip(centers, vel):
                m = int(rng.integers(8, 30))
                pts.append(c + v * f + rng.normal(0, 1.8, (m, 2)))
                vals.append(rng.integers(40, 99, m))
            m = 25
            pts.append(rng.random((m, 2)) * 360 - 180)
            vals.append(rng.integers(11, 60, m))
            if with_land:
                m = 40
                pts.append(np.column_stack([rng.random(m) * 20 + 150, rng.random(m) * 60 - 30]))
                vals.append(rng.integers(150, 255, m))
            p = np.vstack(pts).astype(np.float32)
            v = np.concatenate(vals).astype(np.float32)
            xs.append(p[:, 0]); ys.append(p[:, 1]); ii.append(v)
            gg.append(np.full(len(v), g, np.int32))
        pts = np.column_stack([np.concatenate(xs), np.concatenate(ys), np.concatenate(ii)])
        frames.append(trk.RadarFrame(timestamp=None, timestamp_ms=f * 3000, frame_id=f,
                                     points=pts, gains=np.concatenate(gg)))
    return frames


def g3_land(trk):
    rng = np.random.default_rng(303)
    frames = _frames_stack(trk, rng, F=12)
    cnt, tot, edges = trk.build_occupancy_grid(frames, trk.LAND_GRID_RESOLUTION)
    land = trk.identify_land_cells(cnt, tot, len(frames))
    rec = {"n_frames": np.int64(len(frames)), "count": cnt, "intensity": tot, "land": land,
           "x_edges": edges[0], "y_edges": edges[1]}
    for k, fr in enumerate(frames):
        rec[f"in{k}_points"] = fr.points
        rec[f"in{k}_gains"] = fr.gains
        rec[f"in{k}_fid"] = np.int64(fr.frame_id)
        out = trk.filter_land_from_frame(fr, land, edges)
        rec[f"out{k}_points"] = out.points
        rec[f"out{k}_gains"] = out.gains
    np.savez_compressed(OUT / "g3_land.npz", **rec)


def g4_clusters(trk):
    rng = np.random.default_rng(404)
    rec = {}
    cases = [
        dict(F=8, n_blobs=14, eps=8.0, et=2.0, ms=15, gap=3),
        dict(F=5, n_blobs=20, eps=5.0, et=1.0, ms=6, gap=None),
        dict(F=4, n_blobs=9, eps=8.0, et=0.0, ms=10, gap=None),
    ]
    for k, cs in enumerate(cases):
        frames = _frames_stack(trk, rng, F=cs["F"], with_land=False, n_blobs=cs["n_blobs"],
                               gap_at=cs["gap"])
        res = trk.st_dbscan(frames, cs["eps"], cs["et"], cs["ms"])
        rows = []
        for fr in frames:
            for cl in res.get(fr.frame_id, []):
                rows.append((fr.frame_id, cl.cluster_id, cl.num_points, cl.centroid[0],
                             cl.centroid[1], cl.mean_intensity))
        for j, fr in enumerate(frames):
            rec[f"c{k}_f{j}_points"] = fr.points
            rec[f"c{k}_f{j}_fid"] = np.int64(fr.frame_id)
        rec[f"c{k}_nframes"] = np.int64(len(frames))
        rec[f"c{k}_params"] = np.array([cs["eps"], cs["et"], cs["ms"]], np.float64)
        rec[f"c{k}_frame"] = np.array([r[0] for r in rows], np.int64)
        rec[f"c{k}_label"] = np.array([r[1] for r in rows], np.int64)
        rec[f"c{k}_count"] = np.array([r[2] for r in rows], np.int64)
        rec[f"c{k}_cx"] = np.array([r[3] for r in rows], np.float32)
        rec[f"c{k}_cy"] = np.array([r[4] for r in rows], np.float32)
        rec[f"c{k}_mean_i"] = np.array([r[5] for r in rows], np.float64)
    rec["n_cases"] = np.int64(len(cases))
    np.savez_compressed(OUT / "g4_clusters.npz", **rec)


def _tracker_sequences(rng):
    seqs = []
    # 1) steady targets (buoys and boats) -> dtype switch after 5 velocities, classification
    F = 30
    pos = rng.random((8, 2)) * 300 - 150
    vel = np.vstack([rng.normal(0, 0.2, (4, 2)), rng.normal(0, 3.0, (4, 2))])
    seq = []
    for f in range(F):
        cl = []
        for k in range(8):
            if rng.random() < 0.85:
                cl.append(pos[k] + vel[k] * f + rng.normal(0, 0.3, 2))
        rng.shuffle(cl)
        seq.append((f, np.array(cl, np.float32).reshape(-1, 2)))
    seqs.append(seq)
    # 2) gating (> 50 m jumps), long misses (> 10 frames), empty frames, id gaps
    seq = []
    for f in list(range(0, 8)) + list(range(20, 34)):
        cl = [np.array([10.0, 10.0]) + f * 0.5]
        if f % 3 == 0:
            cl.append(np.array([-80.0, 40.0]) + rng.normal(0, 30, 2))
        if 24 <= f <= 26:
            cl = []
        seq.append((f, np.array(cl, np.float32).reshape(-1, 2)))
    seqs.append(seq)
    # 3) ties: integer-lattice centroids equidistant from predictions
    seq = []
    for f in range(12):
        cl = [[0, 0], [10, 0], [0, 10], [10, 10], [5, 5]]
        if f % 2:
            cl = cl[::-1]
        seq.append((f, np.array(cl, np.float32)))
    seqs.append(seq)
    # 4) many objects, births and deaths
    seq = []
    for f in range(40):
        m = int(rng.integers(0, 25))
        seq.append((f, (rng.random((m, 2)) * 400 - 200).astype(np.float32)))
    seqs.append(seq)
    return seqs


def g5_tracker(trk):
    rng = np.random.default_rng(505)
    rec = {}
    seqs = _tracker_sequences(rng)
    for s, seq in enumerate(seqs):
        tr = trk.ObjectTracker()
        alive = []
        for f, cents in seq:
            clusters = [trk.Cluster(cluster_id=i, frame_id=f, points=np.zeros((1, 2), np.float32),
                                    intensities=np.zeros(1, np.float32), centroid=c)
                        for i, c in enumerate(cents)]
            objs = tr.update(clusters, f)
            alive.append([o.object_id for o in objs])
        rec[f"s{s}_frames"] = np.array([f for f, _ in seq], np.int64)
        rec[f"s{s}_offsets"] = np.cumsum([0] + [len(c) for _, c in seq]).astype(np.int64)
        rec[f"s{s}_cents"] = (np.vstack([c for _, c in seq]) if seq else np.zeros((0, 2))).astype(np.float32)
        rec[f"s{s}_alive_off"] = np.cumsum([0] + [len(a) for a in alive]).astype(np.int64)
        rec[f"s{s}_alive"] = np.array([i for a in alive for i in a], np.int64)
        objs = list(tr.objects.values())
        rec[f"s{s}_obj_id"] = np.array([o.object_id for o in objs], np.int64)
        rec[f"s{s}_obj_type"] = np.array([o.object_type for o in objs])
        rec[f"s{s}_obj_npos"] = np.array([len(o.positions) for o in objs], np.int64)
        rec[f"s{s}_obj_pos"] = (np.vstack([np.vstack(o.positions) for o in objs]) if objs else np.zeros((0, 2))).astype(np.float32)
        rec[f"s{s}_obj_frames"] = np.array([f for o in objs for f in o.frames_seen], np.int64)
        rec[f"s{s}_obj_nvel"] = np.array([len(o.velocities) for o in objs], np.int64)
        rec[f"s{s}_obj_vel"] = np.vstack([np.vstack(o.velocities).astype(np.float64) for o in objs]) if objs else np.zeros((0, 2))
        rec[f"s{s}_obj_avgv"] = np.array([float(o.average_velocity) for o in objs], np.float64)
        rec[f"s{s}_obj_avgv_f32"] = np.array([isinstance(o.average_velocity, np.float32) for o in objs])
        rec[f"s{s}_obj_color"] = np.array([o.color for o in objs], np.int64).reshape(-1, 3)
    rec["n_seqs"] = np.int64(len(seqs))
    np.savez_compressed(OUT / "g5_tracker.npz", **rec)


def synth_csv_stack(root: Path, F=12, rows=48, seed=606):
    """Small deterministic CSV stack for run_pipeline (regenerated by the tests, never stored)."""
    rng = np.random.default_rng(seed)
    angles = np.sort(rng.choice(8196, rows, replace=False))
    targets = rng.random((6, 2)) * [rows, 1024]
    for f in range(F):
        for k, g in enumerate((40, 50, 75)):
            echo = np.zeros((rows, 1024), np.int64)
            m = rng.random((rows, 1024)) < 0.01
            echo[m] = rng.integers(11, 60, m.sum())
            for tr, tb in targets:
                r0 = int(tr) % rows
                b0 = int(tb + f * 3) % 1000
                echo[max(r0 - 2, 0): r0 + 3, b0: b0 + 20] = rng.integers(60, 99, (min(r0 + 3, rows) - max(r0 - 2, 0), 20))
            echo[rows - 6:, 900:1000] = rng.integers(150, 255, (6, 100))  # land
            d = root / f"gain_{g}"
            d.mkdir(parents=True, exist_ok=True)
            ts = f"20250813_1426{f * 3 // 60:02d}_{(f * 3 % 60) * 0 + 100 * k:03d}"
            sec = 2 + 3 * f
            name = f"20250813_14{26 + sec // 60:02d}{sec % 60:02d}_{100 * k:03d}.csv"
            write_csv(d / name, 1, np.full(rows, 231.5), 0, g, angles, echo)
    return root


def g6_pipeline(trk, tmp: Path):
    data = synth_csv_stack(tmp / "stack")
    out = tmp / "out"
    buf = io.StringIO()
    with redirect_stdout(buf):
        trk.run_pipeline(data, out, visualize=False)
    rec = {"stdout": np.array(buf.getvalue())}
    for name in ("tracked_objects.csv", "trajectories.csv", "clusters.csv"):
        rec[name.replace(".csv", "")] = np.array((out / name).read_text())
    np.savez_compressed(OUT / "g6_pipeline.npz", **rec)


def synth_ply(path: Path, seed: int, n_blobs: int = 8, with_color: bool = True):
    """ASCII PLY stack like 2_build_point_clouds.py writes (x y z [red green blue]); z is an
    intensity-like height, the colour is the gain tint (40/50/75) with a few off-palette ones."""
    rng = np.random.default_rng(seed)
    pal = np.array([(0, 114, 255), (0, 200, 83), (255, 87, 34)], np.int64)
    pts, cols = [], []
    for b in range(n_blobs):
        c = rng.random(3) * [200, 200, 40]
        m = int(rng.integers(30, 150))
        pts.append(c + rng.normal(0, [2.0, 2.0, 1.0], (m, 3)))
        cols.append(pal[rng.integers(0, 3, m)])
    m = 400
    pts.append(rng.random((m, 3)) * [220, 220, 40])
    cols.append(rng.integers(0, 256, (m, 3)))
    xyz = np.vstack(pts)
    rgb = np.vstack(cols)
    head = ["ply", "format ascii 1.0", f"element vertex {len(xyz)}", "property float x",
            "property float y", "property float z"]
    if with_color:
        head += ["property uchar red", "property uchar green", "property uchar blue"]
    head.append("end_header")
    lines = []
    for (x, y, z), (r, g, bl) in zip(xyz, rgb):
        lines.append(f"{x:.4f} {y:.4f} {z:.4f}" + (f" {r} {g} {bl}" if with_color else ""))
    path.write_text("\n".join(head + lines) + "\n")
    return path


def g7_ply(ref3, tmp: Path):
    from radar_pipeline.processors.clustering import process_ply_clustering

    rec = {}
    for k, (seed, col) in enumerate(((707, True), (708, True), (709, False))):
        d = tmp / f"c{k}"
        d.mkdir(parents=True)
        ply = synth_ply(d / "stack.ply", seed, with_color=col)
        buf = io.StringIO()
        with redirect_stdout(buf):
            ref3.process_one(ply, "stack_dbscan", eps=ref3.EPS_SPACE,
                             min_samples=ref3.MIN_SAMPLES, max_points=ref3.MAX_POINTS)
        rec[f"c{k}_script_stdout"] = np.array(buf.getvalue())
        rec[f"c{k}_script_csv"] = np.array((d / "stack_dbscan_labels.csv").read_text())
        if col:  # the package loader needs RGB for infer_time_from_colors
            out = d / "pkg"
            out.mkdir()
            buf = io.StringIO()
            with redirect_stdout(buf):
                csv_path, _ = process_ply_clustering(ply, out)
            rec[f"c{k}_pkg_stdout"] = np.array(buf.getvalue())
            rec[f"c{k}_pkg_csv"] = np.array(csv_path.read_text())
    rec["n_cases"] = np.int64(3)
    np.savez_compressed(OUT / "g7_ply.npz", **rec)


def synth_fuse_frames(root: Path, F: int = 2, rows: int = 256, seed: int = 808):
    """Small CSV frames (3 gains) for fuse_gains_max (regenerated by the tests)."""
    rng = np.random.default_rng(seed)
    angles = np.sort(rng.choice(8196, rows, replace=False))
    frames = []
    for f in range(F):
        ff = {}
        for k, g in enumerate((40, 50, 75)):
            echo = np.zeros((rows, 1024), np.int64)
            m = rng.random((rows, 1024)) < 0.05
            echo[m] = rng.integers(0, 256, m.sum())
            d = root / f"gain_{g}"
            d.mkdir(parents=True, exist_ok=True)
            p = d / f"20250813_1426{10 + 3 * f:02d}_{100 * k:03d}.csv"
            write_csv(p, 1, np.full(rows, [231.5, 115.75, 463.0][f % 3]), 0, g, angles, echo)
            ff[g] = p
        frames.append(ff)
    return frames


def g8_fuse_max(tmp: Path):
    fuse = _load("ref_fusion5", REF / "PointCloudWork" / "5_gain_fusion_ply_builder.py")
    frames = synth_fuse_frames(tmp / "fuse")
    rec = {}
    for f, ff in enumerate(frames):
        for res in (1.0, 2.5):
            x, y, i = fuse.fuse_gains_max(ff, grid_resolution=res)
            key = f"f{f}_r{str(res).replace('.', '_')}"
            rec[key + "_x"], rec[key + "_y"], rec[key + "_i"] = x, y, i
    rec["n_frames"] = np.int64(len(frames))
    np.savez_compressed(OUT / "g8_fuse_max.npz", **rec)


def _denoise_cases():
    """(name, coords f32 [n,2], times f32 [n], eps_space, eps_time, min_samples, min_frames)."""
    rng = np.random.default_rng(909)
    cases = []

    def blobs(n_frames, n_blobs, per, spread, drift, noise, skip=()):
        xs, ts = [], []
        centers = rng.random((n_blobs, 2)) * 120.0
        for f in range(n_frames):
            if f in skip:
                continue
            for b in range(n_blobs):
                if rng.random() < 0.25:  # a blob missing from a frame: single-frame neighbours
                    continue
                c = centers[b] + drift * f
                k = rng.integers(per // 2, per + 1)
                xs.append(c + rng.normal(0, spread, (k, 2)))
                ts.append(np.full(k, f, np.float32))
            k = rng.integers(0, noise + 1)
            xs.append(rng.random((k, 2)) * 140.0)
            ts.append(np.full(k, f, np.float32))
        xy = np.vstack(xs).astype(np.float32)
        t = np.concatenate(ts).astype(np.float32)
        perm = rng.permutation(len(t)) if rng.random() < 0.5 else np.arange(len(t))
        return xy[perm], t[perm]

    for i, (eps, et, ms, mf) in enumerate([(8.0, 2.0, 15, 2), (6.0, 1.0, 8, 2), (5.0, 2.0, 6, 3),
                                          (8.0, 0.0, 10, 1), (7.0, 2.5, 12, 2), (4.0, 1.0, 4, 2),
                                          (9.0, 3.0, 20, 4), (6.0, 2.0, 5, 1)]):
        xy, t = blobs(6 + i, 7, 30, 2.5 + 0.3 * i, rng.normal(0, 0.8, 2), 25,
                      skip=(2,) if i % 3 == 0 else ())
        cases.append((f"blobs{i}", xy, t, eps, et, ms, mf))
    # dense single-frame blobs next to multi-frame ones (the min_frames condition decides)
    xy1, t1 = blobs(1, 5, 60, 1.5, np.zeros(2), 10)
    xy2, t2 = blobs(4, 4, 20, 2.0, np.zeros(2), 10)
    xy2 = xy2 + 200.0
    cases.append(("single_vs_multi", np.vstack([xy1, xy2]), np.concatenate([t1, t2 + 10]),
                  6.0, 2.0, 8, 2))
    # lattice: many equal distances, border points shared by several clusters
    g = np.stack(np.meshgrid(np.arange(14), np.arange(14)), -1).reshape(-1, 2).astype(np.float32)
    xy = np.vstack([g * 2.0 + f * 0.5 for f in range(3)]).astype(np.float32)
    t = np.repeat(np.arange(3, dtype=np.float32), len(g))
    cases.append(("lattice", xy, t, 2.0, 1.0, 5, 2))
    # float times (not frame ids): int32 truncation decides the frames
    xy, t = blobs(5, 6, 25, 2.0, np.zeros(2), 15)
    t = (t * 0.7 + rng.random(len(t)).astype(np.float32) * 0.6).astype(np.float32)
    cases.append(("float_time", xy, t, 6.0, 1.2, 8, 2))
    # a NaN time (never a neighbour) and an empty cloud
    xy, t = blobs(3, 3, 20, 2.0, np.zeros(2), 5)
    t = t.copy()
    t[::37] = np.nan
    cases.append(("nan_time", xy, t, 6.0, 2.0, 6, 2))
    cases.append(("empty", np.zeros((0, 2), np.float32), np.zeros(0, np.float32), 8.0, 2.0, 15, 2))
    return cases


def g9_denoise(den):
    rec = {}
    names = []
    for name, xy, t, eps, et, ms, mf in _denoise_cases():
        lab = den.st_dbscan(xy.astype(np.float32), t.astype(np.float32), eps, et, ms, mf)
        rec[f"{name}_xy"], rec[f"{name}_t"] = xy.astype(np.float32), t.astype(np.float32)
        rec[f"{name}_labels"] = np.asarray(lab, np.int32)
        rec[f"{name}_params"] = np.array([eps, et, ms, mf], np.float64)
        names.append(name)
    rec["names"] = np.array(names)
    np.savez_compressed(OUT / "g9_denoise.npz", **rec)
    return len(names)


def g10_denoise_pipeline(den, tmp: Path):
    data = synth_csv_stack(tmp / "stack")
    out = tmp / "out"
    buf = io.StringIO()
    with redirect_stdout(buf):
        den.run_pipeline(data, out, eps_space=8.0, eps_time=2.0, min_samples=15, min_frames=2,
                         max_frames=0, no_viz=True, parallel=False)
    rec = {"stdout": np.array(buf.getvalue())}
    for name in ("denoised_point_cloud.ply", "raw_point_cloud.ply"):
        rec[name.replace(".", "_")] = np.frombuffer((out / name).read_bytes(), np.uint8)
    for name in ("denoising_stats.csv", "clusters.csv"):
        rec[name.replace(".", "_")] = np.array((out / name).read_text())
    np.savez_compressed(OUT / "g10_denoise_pipeline.npz", **rec)


def corrupt_csv_stack(root: Path, denoise: bool = False):
    """synth_csv_stack with malformed files (regenerated by the tests, never stored):
    frame 3 gain 50: a last row with two fields too many (read_csv's tokenizing error; the
    tracker prints "Error loading ...", the denoise loader fails the whole frame); frame 5 gain
    40: one data row (genfromtxt's 1-D array: an empty sweep for the denoise loader); frame 6
    gain 75: a comment line after row 10; frame 8 gain 40: empty echo fields in row 4; with
    denoise=True also an empty Scale field in frame 6 gain 75's row 7 (genfromtxt fills 0.0;
    pandas' NaN would reach the tracker's BallTree, which raises)."""
    synth_csv_stack(root)
    files = {g: sorted((root / f"gain_{g}").glob("*.csv")) for g in (40, 50, 75)}

    def edit(path, fn):
        lines = path.read_text().splitlines()
        path.write_text("\n".join(fn(lines)) + "\n")

    edit(files[50][3], lambda L: L + [L[-1] + ",7,7"])
    edit(files[40][5], lambda L: L[:2])

    def f6(L):
        if denoise:
            row = L[1 + 7].split(",")
            row[1] = ""
            L[1 + 7] = ",".join(row)
        return L[:11] + ["# note: gain check"] + L[11:]
    edit(files[75][6], f6)

    def f8(L):
        row = L[1 + 4].split(",")
        for c in (5, 6, 300, 301, 302):
            row[c] = ""
        L[1 + 4] = ",".join(row)
        return L
    edit(files[40][8], f8)
    return root


def g11_corrupt(trk, den, tmp: Path):
    rec = {}
    data = corrupt_csv_stack(tmp / "stack")
    buf = io.StringIO()
    with redirect_stdout(buf):
        trk.run_pipeline(data, tmp / "out", visualize=False)
    rec["tracker_stdout"] = np.array(buf.getvalue())
    for name in ("tracked_objects.csv", "trajectories.csv", "clusters.csv"):
        rec["tracker_" + name.replace(".csv", "")] = np.array((tmp / "out" / name).read_text())
    data = corrupt_csv_stack(tmp / "dstack", denoise=True)
    out = tmp / "dout"
    buf = io.StringIO()
    with redirect_stdout(buf):
        den.run_pipeline(data, out, eps_space=8.0, eps_time=2.0, min_samples=15, min_frames=2,
                         max_frames=0, no_viz=True, parallel=True)
    rec["denoise_stdout"] = np.array(buf.getvalue())
    for name in ("denoised_point_cloud.ply", "raw_point_cloud.ply"):
        rec["denoise_" + name.replace(".", "_")] = np.frombuffer((out / name).read_bytes(),
                                                                 np.uint8)
    for name in ("denoising_stats.csv", "clusters.csv"):
        rec["denoise_" + name.replace(".", "_")] = np.array((out / name).read_text())
    np.savez_compressed(OUT / "g11_corrupt.npz", **rec)


def main():
    if not REF.exists():
        raise SystemExit("make_golden.py must run where /root/reference exists (build container)")
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.path.insert(0, str(REF / "radar-pipeline" / "src"))
    trk = _load("ref_tracker4", REF / "PointCloudWork" / "4_temporal_object_tracker.py")
    ref3 = _load("ref_stdbscan3", REF / "PointCloudWork" / "3_stdbscan_point_clouds.py")
    from radar_pipeline.core import loaders as rp_loaders, transforms as rp_transforms
    only = set(sys.argv[1:])
    want = lambda name: not only or name in only  # noqa: E731
    n = None
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        if want("g1"):
            g1_polar(trk, rp_loaders, rp_transforms, tmp / "g1")
        if want("g2"):
            n = g2_stdbscan(ref3)
        if want("g3"):
            g3_land(trk)
        if want("g4"):
            g4_clusters(trk)
        if want("g5"):
            g5_tracker(trk)
        if want("g6"):
            g6_pipeline(trk, tmp / "g6")
        if want("g7"):
            g7_ply(ref3, tmp / "g7")
        if want("g8"):
            g8_fuse_max(tmp / "g8")
        if want("g9") or want("g10") or want("g11"):
            den = _load("ref_denoise", REF / "PointCloudWorkF" / "stdbscan_denoising_pipeline.py")
            if want("g9"):
                g9_denoise(den)
            if want("g10"):
                g10_denoise_pipeline(den, tmp / "g10")
            if want("g11"):
                g11_corrupt(trk, den, tmp / "g11")
    import scipy
    import sklearn
    mp = OUT / "meta.json"
    meta = json.loads(mp.read_text()) if mp.exists() else {}
    meta.update({"numpy": np.__version__, "scipy": scipy.__version__,
                 "sklearn": sklearn.__version__, "python": platform.python_version(),
                 "cpu": platform.processor() or platform.machine()})
    if n is not None:
        meta["g2_cases"] = n
    (OUT / "meta.json").write_text(json.dumps(meta, indent=1) + "\n")
    for p in sorted(OUT.glob("*.npz")):
        print(f"{p.name}: {p.stat().st_size / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
