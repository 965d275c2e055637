"""Pin the oracle: every oracle function reproduces the vectors produced by running the reference
itself (tests/golden/make_golden.py).  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oracle import path as op


def test_stdbscan_oracle_matches_reference_labels(golden):
    g = golden("g2_stdbscan.npz")
    for k in range(int(g["n_cases"])):
        eps, et, ms = g[f"c{k}_params"]
        lab = oracle.stdbscan(g[f"c{k}_coords"], g[f"c{k}_times"], eps, et, int(ms))
        np.testing.assert_array_equal(lab, g[f"c{k}_labels"], err_msg=f"case {k} {g[f'c{k}_kind']}")
        lab = oracle.stdbscan_uf(g[f"c{k}_coords"], g[f"c{k}_times"], eps, et, int(ms))
        np.testing.assert_array_equal(lab, g[f"c{k}_labels"], err_msg=f"uf case {k}")


def test_reference_structure_baseline_matches_reference_labels(golden):
    """oracle/refpath.py (bench.py's cpu_baseline: whole-stack BallTree + per-neighbour time
    filter + seed-set expansion, the reference's structure) gives the reference's labels."""
    from oracle.refpath import stdbscan_structure

    g = golden("g2_stdbscan.npz")
    for k in range(int(g["n_cases"])):
        c, t = g[f"c{k}_coords"], g[f"c{k}_times"]
        if len(c) == 0:
            continue
        eps, et, ms = g[f"c{k}_params"]
        lab, _ = stdbscan_structure(c, t, eps, et, int(ms))
        np.testing.assert_array_equal(lab, g[f"c{k}_labels"], err_msg=f"case {k}")


def test_stdbscan_uf_matches_bfs_on_dense_stacks():
    """The set-formulation checker (used at full stack sizes) against the BFS oracle on dense
    multi-frame clouds: chained clusters, border points between clusters, frame-id gaps, NaN
    times, lattice ties, D=3."""
    rng = np.random.default_rng(31)
    for case in range(12):
        F = int(rng.integers(2, 9))
        pts, ts = [], []
        for f in range(F):
            if case % 4 == 1 and f == F // 2:
                continue  # frame-id gap
            c = rng.random((int(rng.integers(3, 10)), 2)) * 150
            for cc in c:
                m = int(rng.integers(5, 120))
                pts.append(cc + rng.normal(0, rng.choice([1.0, 3.0, 6.0]), (m, 2)))
                ts.append(np.full(m, f))
            m = int(rng.integers(50, 400))
            pts.append(rng.random((m, 2)) * 150)
            ts.append(np.full(m, f))
        xy = np.vstack(pts).astype(np.float32)
        if case % 3 == 2:
            xy = np.round(xy)  # lattice: exact-boundary distances
        t = np.concatenate(ts).astype(np.float32)
        if case % 4 == 3:
            t[rng.random(len(t)) < 0.01] = np.nan
        if case % 5 == 4:
            xy = np.column_stack([xy, rng.integers(0, 30, len(xy))]).astype(np.float32)
        eps, et, ms = float(rng.choice([3.0, 5.0, 8.0])), float(rng.choice([0.0, 1.0, 2.0])), \
            int(rng.choice([1, 4, 10, 15]))
        np.testing.assert_array_equal(oracle.stdbscan_uf(xy, t, eps, et, ms),
                                      oracle.stdbscan(xy, t, eps, et, ms), err_msg=f"case {case}")


def test_polar_oracle_matches_load_radar_csv(golden):
    g = golden("g1_polar.npz")
    for k in range(3):
        cos_t, sin_t = op.trig_tables(g[f"f{k}_angle"])
        x, y, v = op.polar_scatter(g[f"f{k}_echo"], g[f"f{k}_scale"], cos_t, sin_t)
        np.testing.assert_array_equal(x, g[f"f{k}_x"])
        np.testing.assert_array_equal(y, g[f"f{k}_y"])
        np.testing.assert_array_equal(v, g[f"f{k}_i"])
        # package form (radar_pipeline sweep_to_point_cloud: threshold 0, stride 16)
        xp, yp, zp = op.polar_scatter(g[f"f{k}_echo"], g[f"f{k}_scale"], cos_t, sin_t,
                                      threshold=0.0, stride=16)
        np.testing.assert_array_equal(xp, g[f"f{k}_pkg_x"])
        np.testing.assert_array_equal(yp, g[f"f{k}_pkg_y"])
        np.testing.assert_array_equal(zp, g[f"f{k}_pkg_z"])


def test_build_frames_oracle_matches_build_frame(golden):
    g = golden("g1_polar.npz")
    per_gain = {}
    for k in range(3):
        cos_t, sin_t = op.trig_tables(g[f"f{k}_angle"])
        per_gain[int(g[f"f{k}_gain"])] = op.polar_scatter(g[f"f{k}_echo"], g[f"f{k}_scale"],
                                                          cos_t, sin_t)
    frames = op.build_frames([per_gain])
    assert len(frames) == 1
    _, pts, gains = frames[0]
    np.testing.assert_array_equal(pts, g["frame_points"])
    np.testing.assert_array_equal(gains, g["frame_gains"])


def _g3_frames(g):
    n = int(g["n_frames"])
    return [(int(g[f"in{k}_fid"]), g[f"in{k}_points"], g[f"in{k}_gains"]) for k in range(n)]


def test_land_oracle_matches_reference(golden):
    g = golden("g3_land.npz")
    frames = _g3_frames(g)
    out, cnt, tot, land, (xe, ye) = op.land_filter(frames)
    np.testing.assert_array_equal(xe, g["x_edges"])
    np.testing.assert_array_equal(ye, g["y_edges"])
    np.testing.assert_array_equal(cnt, g["count"])
    np.testing.assert_array_equal(tot, g["intensity"])
    np.testing.assert_array_equal(land, g["land"])
    assert land.any(), "fixture should contain land cells"
    for k, (_, p, gg) in enumerate(out):
        np.testing.assert_array_equal(p, g[f"out{k}_points"])
        np.testing.assert_array_equal(gg, g[f"out{k}_gains"])


def _g4_case(g, k):
    frames = [(int(g[f"c{k}_f{j}_fid"]), g[f"c{k}_f{j}_points"], None)
              for j in range(int(g[f"c{k}_nframes"]))]
    eps, et, ms = g[f"c{k}_params"]
    return frames, float(eps), float(et), int(ms)


def test_frame_clusters_oracle_matches_reference(golden):
    g = golden("g4_clusters.npz")
    for k in range(int(g["n_cases"])):
        frames, eps, et, ms = _g4_case(g, k)
        xy, t = op.stack_coords(frames)
        labels = oracle.stdbscan(xy, t, eps, et, ms)
        res = op.frame_clusters(frames, labels)
        rows = [(fid, *c) for fid, _, _ in frames for c in res.get(fid, [])]
        assert len(rows) == len(g[f"c{k}_frame"])
        np.testing.assert_array_equal([r[0] for r in rows], g[f"c{k}_frame"])
        np.testing.assert_array_equal([r[1] for r in rows], g[f"c{k}_label"])
        np.testing.assert_array_equal([r[2] for r in rows], g[f"c{k}_count"])
        np.testing.assert_array_equal(np.array([r[3][0] for r in rows], np.float32), g[f"c{k}_cx"])
        np.testing.assert_array_equal(np.array([r[3][1] for r in rows], np.float32), g[f"c{k}_cy"])
        np.testing.assert_array_equal([r[4] for r in rows], g[f"c{k}_mean_i"])


def replay_tracker(g, s, make):
    """Feed sequence s of g5 into a tracker built by make(); returns (tracker, alive lists)."""
    frames = g[f"s{s}_frames"]
    off = g[f"s{s}_offsets"]
    cents = g[f"s{s}_cents"]
    trk = make()
    alive = []
    for i, f in enumerate(frames):
        cl = [(cents[j], int(f)) for j in range(off[i], off[i + 1])]
        objs = trk.update(cl, int(f))
        alive.append([o.object_id for o in objs])
    return trk, alive


def test_tracker_oracle_matches_reference(golden):
    g = golden("g5_tracker.npz")
    for s in range(int(g["n_seqs"])):
        trk, alive = replay_tracker(g, s, oracle.Tracker)
        ao = g[f"s{s}_alive_off"]
        for i, a in enumerate(alive):
            assert a == list(g[f"s{s}_alive"][ao[i]:ao[i + 1]])
        objs = list(trk.objects.values())
        np.testing.assert_array_equal([o.object_id for o in objs], g[f"s{s}_obj_id"])
        np.testing.assert_array_equal([o.object_type for o in objs], g[f"s{s}_obj_type"])
        pos = np.vstack([np.vstack(o.positions) for o in objs]).astype(np.float32)
        np.testing.assert_array_equal(pos, g[f"s{s}_obj_pos"])
        vel = np.vstack([np.vstack(o.velocities).astype(np.float64) for o in objs])
        np.testing.assert_array_equal(vel, g[f"s{s}_obj_vel"])
        np.testing.assert_array_equal([float(o.average_velocity) for o in objs],
                                      g[f"s{s}_obj_avgv"])
        np.testing.assert_array_equal([isinstance(o.average_velocity, np.float32) for o in objs],
                                      g[f"s{s}_obj_avgv_f32"])
        np.testing.assert_array_equal([o.color for o in objs], g[f"s{s}_obj_color"])


def test_denoise_oracle_matches_reference(golden):
    """oracle.stdbscan_denoise against PointCloudWorkF st_dbscan run in the build container
    (g9: blobs with missing frames, single- vs multi-frame blobs, lattice, float times, a NaN
    time, an empty cloud; min_frames 1-4)."""
    g = golden("g9_denoise.npz")
    for name in g["names"]:
        eps, et, ms, mf = g[f"{name}_params"]
        lab = oracle.stdbscan_denoise(g[f"{name}_xy"], g[f"{name}_t"], eps, et, int(ms), int(mf))
        np.testing.assert_array_equal(lab, g[f"{name}_labels"], err_msg=str(name))


def _denoise_sets(xy, t, eps, et, ms, mf):
    """The set formulation the device path computes (csrc/stdbscan.hip k_frames_* and
    k_label_fifo), brute force: core = count >= ms and >= mf distinct int32(t) frames among the
    neighbours; components of core points numbered by minimum index; a non-core point p takes
    the smallest component m adjacent through a core point with p > m or p adjacent to m."""
    n = len(t)
    x64 = xy.astype(np.float64)
    d2 = (x64[:, None, 0] - x64[None, :, 0]) ** 2 + (x64[:, None, 1] - x64[None, :, 1]) ** 2
    with np.errstate(invalid="ignore"):
        adj = (d2 <= eps * eps) & (np.abs(t[:, None] - t[None, :]) <= np.float32(et))
    with np.errstate(invalid="ignore"):
        fr = t.astype(np.int32)
    core = np.array([adj[i].sum() >= ms and len(np.unique(fr[adj[i]])) >= mf for i in range(n)],
                    bool) if n else np.zeros(0, bool)
    comp = np.full(n, -1)
    for i in range(n):
        if core[i] and comp[i] < 0:
            stack, comp[i] = [i], i
            while stack:
                a = stack.pop()
                for b in np.nonzero(adj[a] & core)[0]:
                    if comp[b] < 0:
                        comp[b] = i
                        stack.append(b)
    mins = sorted(set(comp[core].tolist()))
    cid = {m: k for k, m in enumerate(mins)}
    lab = np.full(n, -1, np.int32)
    for i in range(n):
        if core[i]:
            lab[i] = cid[comp[i]]
        else:
            ms_ = [m for m in set(comp[adj[i] & core].tolist()) if i > m or adj[i, m]]
            if ms_:
                lab[i] = cid[min(ms_)]
    return lab


def test_denoise_set_formulation_matches_fifo_oracle():
    """The order-free formulation of the FIFO expansion (what the GPU computes) equals the
    sequential restatement on random clouds with many shared border points."""
    rng = np.random.default_rng(41)
    for k in range(30):
        n = int(rng.integers(50, 500))
        xy = (rng.random((n, 2)) * rng.uniform(20, 80)).astype(np.float32)
        t = rng.integers(0, 5, n).astype(np.float32)
        if k % 5 == 4:
            t = (t + rng.random(n) * 0.9).astype(np.float32)
        eps, et = float(rng.uniform(2, 8)), float(rng.choice([0.0, 1.0, 1.5, 2.0]))
        ms, mf = int(rng.integers(1, 12)), int(rng.integers(0, 4))
        a = oracle.stdbscan_denoise(xy, t, eps, et, ms, mf)
        b = _denoise_sets(xy, t, eps, et, ms, mf)
        np.testing.assert_array_equal(a, b, err_msg=f"case {k}")
