"""Parity of the HIP path stages (through the C-ABI) with the reference's golden vectors and the
pinned oracle: K1 polar scatter + fusion, synthetic echo, land filter, cluster summaries +
reference cluster order, and the whole stack -> tracker path."""
from __future__ import annotations

import sys

import numpy as np
import pytest
import torch

import oracle
from oracle import path as op

from _stack_check import check_stack_vs_oracle as _check_stack_vs_oracle
from _stack_check import oracle_stack as _oracle_stack

pytestmark = pytest.mark.gpu


def _k1(dev, echo, scale, angle, gains=(0,), threshold=10.0, stride=4, f32=False, staged=False):
    """Run rpt_polar_count/write (or their staged-entry variants) on a batch of equally shaped
    sweeps."""
    from rpt import _abi
    from rpt._device import stream_handle
    from rpt.core.transforms import trig_tables

    lib = _abi.load()
    echo = np.ascontiguousarray(echo)
    nf, rows, bins = echo.shape
    ed = torch.from_numpy(echo.astype(np.float32) if f32 else echo.astype(np.uint8)).to(dev)
    c, s = [], []
    for a in angle:
        ct, st_ = trig_tables(a)
        c.append(ct)
        s.append(st_)
    cd = torch.from_numpy(np.concatenate(c)).to(dev)
    sd = torch.from_numpy(np.concatenate(s)).to(dev)
    sc = torch.from_numpy(np.concatenate(scale).astype(np.float32)).to(dev)
    gl = list(gains) * (nf // len(gains)) if nf % len(gains) == 0 else list(gains)
    gd = torch.tensor(gl, dtype=torch.int32, device=dev)
    rp = torch.empty(nf * rows + 1, dtype=torch.int64, device=dev)
    fo = torch.empty(nf + 1, dtype=torch.int64, device=dev)
    tot = _abi.C.c_int64(0)
    dt = _abi.ECHO_F32 if f32 else _abi.ECHO_U8
    st = stream_handle(dev)
    mk = torch.zeros(max(int(lib.rpt_polar_stage_words(nf, rows)), 1), dtype=torch.int32,
                     device=dev) if staged else None
    if staged:
        _abi.check(lib.rpt_polar_count_staged(ed.data_ptr(), dt, nf, rows, bins, threshold,
                                              stride, rp.data_ptr(), fo.data_ptr(),
                                              _abi.C.byref(tot), mk.data_ptr(), st))
    else:
        _abi.check(lib.rpt_polar_count(ed.data_ptr(), dt, nf, rows, bins, threshold, stride,
                                       rp.data_ptr(), fo.data_ptr(), _abi.C.byref(tot), st))
    n = tot.value
    x = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    y, v = torch.empty_like(x), torch.empty_like(x)
    g = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    pf = torch.empty_like(g)
    args = (ed.data_ptr(), dt, nf, rows, bins, sc.data_ptr(), cd.data_ptr(), sd.data_ptr(),
            gd.data_ptr(), threshold, stride, rp.data_ptr(), fo.data_ptr(), len(gains),
            x.data_ptr(), y.data_ptr(), v.data_ptr(), g.data_ptr(), pf.data_ptr())
    if staged:
        _abi.check(lib.rpt_polar_write_staged(*args, mk.data_ptr(), st))
    else:
        _abi.check(lib.rpt_polar_write(*args, st))
    return (x[:n].cpu().numpy(), y[:n].cpu().numpy(), v[:n].cpu().numpy(), g[:n].cpu().numpy(),
            pf[:n].cpu().numpy(), fo.cpu().numpy())


@pytest.mark.parametrize("f32", [False, True])
def test_polar_scatter_matches_load_radar_csv(gpu, golden, f32):
    g = golden("g1_polar.npz")
    parts = []
    for k in range(3):
        x, y, v, gg, _, _ = _k1(gpu, g[f"f{k}_echo"][None], [g[f"f{k}_scale"]],
                                [g[f"f{k}_angle"]], gains=(int(g[f"f{k}_gain"]),), f32=f32)
        np.testing.assert_array_equal(x, g[f"f{k}_x"])
        np.testing.assert_array_equal(y, g[f"f{k}_y"])
        np.testing.assert_array_equal(v, g[f"f{k}_i"])
        parts.append((x, y, v, gg))
    # build_frame fusion = concatenation in ascending gain order
    pts = np.column_stack([np.concatenate([p[0] for p in parts]),
                           np.concatenate([p[1] for p in parts]),
                           np.concatenate([p[2] for p in parts])])
    np.testing.assert_array_equal(pts, g["frame_points"])
    np.testing.assert_array_equal(np.concatenate([p[3] for p in parts]), g["frame_gains"])


def test_sweep_to_point_cloud_matches_package(gpu, golden):
    from rpt.core.loaders import RadarSweep
    from rpt.core.transforms import sweep_to_point_cloud

    g = golden("g1_polar.npz")
    for k in range(3):
        sw = RadarSweep(angles_rad=g[f"f{k}_pkg_angles"], ranges=g[f"f{k}_pkg_ranges"],
                        intensities=g[f"f{k}_echo"].astype(np.float32),
                        scale=g[f"f{k}_scale"])
        pc = sweep_to_point_cloud(sw)
        np.testing.assert_array_equal(pc.x, g[f"f{k}_pkg_x"])
        np.testing.assert_array_equal(pc.y, g[f"f{k}_pkg_y"])
        np.testing.assert_array_equal(pc.z, g[f"f{k}_pkg_z"])


def test_polar_to_cartesian_reference_known_answers(gpu):
    """radar-pipeline/tests/test_transforms.py:15-45 known answers."""
    from rpt.core.transforms import polar_to_cartesian

    angles = np.array([0, np.pi / 2, np.pi], dtype=np.float32)
    x, y = polar_to_cartesian(angles, np.array([[1], [1], [1]], dtype=np.float32))
    np.testing.assert_allclose(x[:, 0], [1, 0, -1], atol=1e-6)
    np.testing.assert_allclose(y[:, 0], [0, 1, 0], atol=1e-6)
    x, y = polar_to_cartesian(np.array([0, np.pi / 2], np.float32),
                              np.array([[1, 2, 3], [1, 2, 3]], dtype=np.float32))
    assert x.shape == (2, 3)
    np.testing.assert_allclose(x[0], [1, 2, 3], atol=1e-6)
    np.testing.assert_allclose(y[1], [1, 2, 3], atol=1e-6)


def test_infer_time_from_colors(gpu):
    from rpt.processors import infer_time_from_colors

    cols = np.array([[0, 114, 255], [0, 200, 83], [255, 87, 34], [5, 110, 250], [10, 195, 88],
                     [128, 128, 128], [0, 0, 0], [255, 255, 255]], np.uint8)
    pal = np.array([[0, 114, 255], [0, 200, 83], [255, 87, 34]], np.float32)
    d = cols[:, None, :].astype(np.float32) - pal[None]
    exp = np.argmin(np.sum(d * d, axis=2), axis=1).astype(np.float32)
    np.testing.assert_array_equal(infer_time_from_colors(cols), exp)
    rng = np.random.default_rng(2)
    cols = rng.integers(0, 256, (5000, 3)).astype(np.uint8)
    d = cols[:, None, :].astype(np.float32) - pal[None]
    exp = np.argmin(np.sum(d * d, axis=2), axis=1).astype(np.float32)
    np.testing.assert_array_equal(infer_time_from_colors(cols), exp)


def _small_synth(n_frames=3, rows=512, targets=12, frame0=0):
    from rpt.synth import SynthConfig

    return SynthConfig(n_frames=n_frames, rows=rows, n_targets=targets, frame0=frame0,
                       clutter_density=0.03)


def test_synth_echo_bit_identical(gpu):
    from rpt.synth import DeviceSynth, numpy_echo

    for cfg in (_small_synth(), _small_synth(n_frames=2, rows=4096, targets=40, frame0=5)):
        ds = DeviceSynth(cfg, gpu)
        dev = ds.echo().cpu().numpy()
        ref = numpy_echo(cfg, ds.geo)
        np.testing.assert_array_equal(dev, ref)
        assert (ref >= 60).sum() > 0 and (ref >= 150).sum() > 0 and ((ref > 10) & (ref < 40)).sum() > 0


def test_k1_batch_matches_oracle_on_synth(gpu):
    """Multi-file batch (3 gains x 3 frames, 4096 rows): per-file stride ranks and fusion."""
    from rpt.synth import DeviceSynth, SynthConfig

    cfg = SynthConfig(n_frames=3, n_targets=40)
    ds = DeviceSynth(cfg, gpu)
    echo = ds.echo().cpu().numpy()
    F, G, R, B = echo.shape
    x, y, v, g, pf, fo = _k1(gpu, echo.reshape(F * G, R, B), [np.full(R, cfg.scale, np.float32)] * (F * G),
                             [ds.geo.angle] * (F * G), gains=cfg.gains)
    per_frame = []
    for f in range(F):
        per_frame.append({gain: op.polar_scatter(echo[f, k], np.full(R, cfg.scale, np.float32),
                                                 ds.geo.cos_t, ds.geo.sin_t)
                          for k, gain in enumerate(cfg.gains)})
    frames = op.build_frames(per_frame)
    pts = np.vstack([p for _, p, _ in frames])
    np.testing.assert_array_equal(np.column_stack([x, y, v]), pts)
    np.testing.assert_array_equal(g, np.concatenate([gg for _, _, gg in frames]))
    np.testing.assert_array_equal(pf, np.concatenate([np.full(len(p), fid) for fid, p, _ in frames]))


def _land_device(dev, frames):
    """Run the device land filter on oracle-format frames; returns (cnt, tot, land, edges, kept)."""
    from rpt import _abi
    from rpt._device import stream_handle

    lib = _abi.load()
    st = stream_handle(dev)
    pts = np.vstack([p for _, p, _ in frames])
    gains = np.concatenate([g for _, _, g in frames]).astype(np.int32)
    pf = np.concatenate([np.full(len(p), k, np.int32) for k, (_, p, _) in enumerate(frames)])
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for _, p, _ in frames])
    n = len(pts)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    x, y, v = T(pts[:, 0]), T(pts[:, 1]), T(pts[:, 2])
    gd, pfd, offd = T(gains), T(pf), T(off)
    b4 = (_abi.C.c_float * 4)()
    _abi.check(lib.rpt_bounds_xy(x.data_ptr(), y.data_ptr(), n, b4, st))
    x0, x1, y0, y1 = (np.float32(b4[k]) for k in range(4))
    xe = np.arange(x0, x1 + 5.0, 5.0)
    ye = np.arange(y0, y1 + 5.0, 5.0)
    xed, yed = T(xe), T(ye)
    cells = (len(xe) - 1) * (len(ye) - 1)
    cnt = torch.empty(cells, dtype=torch.int32, device=dev)
    tot = torch.empty(cells, dtype=torch.float64, device=dev)
    land = torch.empty(cells, dtype=torch.uint8, device=dev)
    _abi.check(lib.rpt_land_grid(x.data_ptr(), y.data_ptr(), v.data_ptr(), n, xed.data_ptr(),
                                 len(xe), yed.data_ptr(), len(ye), cnt.data_ptr(), tot.data_ptr(),
                                 st))
    nl = _abi.C.c_int64(0)
    _abi.check(lib.rpt_land_mask(cnt.data_ptr(), tot.data_ptr(), cells, len(frames), 0.8, 100.0,
                                 land.data_ptr(), _abi.C.byref(nl), st))
    outs = [torch.empty(n, dtype=d, device=dev) for d in
            (torch.float32, torch.float32, torch.float32, torch.int32, torch.int32)]
    noff = torch.empty(len(frames) + 1, dtype=torch.int64, device=dev)
    kept = _abi.C.c_int64(0)
    _abi.check(lib.rpt_land_filter(x.data_ptr(), y.data_ptr(), v.data_ptr(), gd.data_ptr(),
                                   pfd.data_ptr(), n, offd.data_ptr(), len(frames),
                                   xed.data_ptr(), len(xe), yed.data_ptr(), len(ye),
                                   land.data_ptr(), *[o.data_ptr() for o in outs],
                                   noff.data_ptr(), _abi.C.byref(kept), st))
    k = kept.value
    shape = (len(xe) - 1, len(ye) - 1)
    return (cnt.cpu().numpy().reshape(shape), tot.cpu().numpy().reshape(shape),
            land.cpu().numpy().reshape(shape).astype(bool), (xe, ye), int(nl.value),
            [o[:k].cpu().numpy() for o in outs], noff.cpu().numpy())


def test_land_filter_matches_reference(gpu, golden):
    g = golden("g3_land.npz")
    n = int(g["n_frames"])
    frames = [(int(g[f"in{k}_fid"]), g[f"in{k}_points"], g[f"in{k}_gains"]) for k in range(n)]
    cnt, tot, land, (xe, ye), nl, outs, noff = _land_device(gpu, frames)
    np.testing.assert_array_equal(xe, g["x_edges"])
    np.testing.assert_array_equal(ye, g["y_edges"])
    np.testing.assert_array_equal(cnt, g["count"])
    np.testing.assert_array_equal(tot, g["intensity"])
    np.testing.assert_array_equal(land, g["land"])
    assert nl == int(g["land"].sum())
    exp = np.vstack([g[f"out{k}_points"] for k in range(n)])
    np.testing.assert_array_equal(np.column_stack(outs[:3]), exp)
    np.testing.assert_array_equal(outs[3], np.concatenate([g[f"out{k}_gains"] for k in range(n)]))
    np.testing.assert_array_equal(np.diff(noff), [len(g[f"out{k}_points"]) for k in range(n)])


def _summaries_device(dev, frames, labels_np, n_clusters):
    from rpt import _abi
    from rpt._device import stream_handle

    lib = _abi.load()
    st = stream_handle(dev)
    pts = np.vstack([p for _, p, _ in frames])
    pf = np.concatenate([np.full(len(p), k, np.int32) for k, (_, p, _) in enumerate(frames)])
    n = len(pts)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    x, y, v, pfd, lab = T(pts[:, 0]), T(pts[:, 1]), T(pts[:, 2]), T(pf), T(labels_np.astype(np.int32))
    F = len(frames)
    outs = {k: torch.empty(max(n, 1), dtype=d, device=dev) for k, d in
            (("frame", torch.int32), ("label", torch.int32), ("count", torch.int64),
             ("first", torch.int64), ("cx", torch.float32), ("cy", torch.float32),
             ("mi", torch.float32))}
    ffn = torch.empty(F, dtype=torch.int64, device=dev)
    ns = _abi.C.c_int64(0)
    _abi.check(lib.rpt_cluster_summaries(lab.data_ptr(), x.data_ptr(), y.data_ptr(), v.data_ptr(),
                                         pfd.data_ptr(), n, F, n_clusters,
                                         *[outs[k].data_ptr() for k in
                                           ("frame", "label", "count", "first", "cx", "cy", "mi")],
                                         ffn.data_ptr(), _abi.C.byref(ns), st))
    S = ns.value
    seg = {k: t[:S].cpu().numpy() for k, t in outs.items()}
    fn = ffn.cpu().numpy()
    fo = np.empty(F + 1, np.int64)
    order = np.empty(max(S, 1), np.int64)
    _abi.check(lib.rpt_order_clusters(F, S, seg["frame"].ctypes.data_as(_abi.c_i32p),
                                      seg["label"].ctypes.data_as(_abi.c_i32p),
                                      seg["first"].ctypes.data_as(_abi.c_i64p),
                                      fn.ctypes.data_as(_abi.c_i64p),
                                      fo.ctypes.data_as(_abi.c_i64p),
                                      order.ctypes.data_as(_abi.c_i64p)))
    return seg, fo, order[:S]


def test_cluster_summaries_and_order_match_reference(gpu, golden):
    from rpt.processors.clustering import st_dbscan

    g = golden("g4_clusters.npz")
    for k in range(int(g["n_cases"])):
        frames = [(int(g[f"c{k}_f{j}_fid"]), g[f"c{k}_f{j}_points"], None)
                  for j in range(int(g[f"c{k}_nframes"]))]
        eps, et, ms = g[f"c{k}_params"]
        xy, t = op.stack_coords(frames)
        labels = st_dbscan(xy, t, eps, et, int(ms))
        seg, fo, order = _summaries_device(gpu, frames, labels, int(labels.max()) + 1)
        rows = []
        for j, (fid, _, _) in enumerate(frames):
            for s in order[fo[j]:fo[j + 1]]:
                rows.append((fid, seg["label"][s], seg["count"][s], seg["cx"][s], seg["cy"][s],
                             float(seg["mi"][s])))
        assert len(rows) == len(g[f"c{k}_frame"])
        np.testing.assert_array_equal([r[0] for r in rows], g[f"c{k}_frame"])
        np.testing.assert_array_equal([r[1] for r in rows], g[f"c{k}_label"])
        np.testing.assert_array_equal([r[2] for r in rows], g[f"c{k}_count"])
        np.testing.assert_array_equal(np.array([r[3] for r in rows], np.float32), g[f"c{k}_cx"])
        np.testing.assert_array_equal(np.array([r[4] for r in rows], np.float32), g[f"c{k}_cy"])
        np.testing.assert_array_equal([r[5] for r in rows], g[f"c{k}_mean_i"])


def test_mean_intensity_pairwise_chunks(gpu):
    """Non-integer intensities in clusters of 1..20000 points: numpy's chunked pairwise mean."""
    rng = np.random.default_rng(12)
    sizes = [1, 2, 7, 8, 9, 127, 128, 129, 1000, 8191, 8192, 8193, 20000]
    pts, labs = [], []
    for k, m in enumerate(sizes):
        p = np.column_stack([rng.normal(k * 100, 1, m), rng.normal(0, 1, m),
                             rng.random(m) * 250]).astype(np.float32)
        pts.append(p)
        labs.append(np.full(m, k, np.int32))
    p = np.vstack(pts)
    lab = np.concatenate(labs)
    perm = rng.permutation(len(p))
    p, lab = p[perm], lab[perm]
    seg, fo, order = _summaries_device(gpu, [(0, p, None)], lab, len(sizes))
    for s in range(len(seg["label"])):
        m = lab == seg["label"][s]
        assert seg["count"][s] == m.sum()
        assert seg["first"][s] == np.nonzero(m)[0][0]
        c = np.mean(p[m][:, :2], axis=0)
        assert seg["cx"][s] == c[0] and seg["cy"][s] == c[1]
        assert float(seg["mi"][s]) == float(np.mean(p[m][:, 2]))


def _radix_summaries_in_child(frames, lab, ncl):
    """_summaries_device in a child process on the A/B build (librpt_ab.so, built by
    __graft_entry__.build(): the only build that reads RPT_* switches) with RPT_K9_RADIX=1."""
    import os
    import subprocess
    import tempfile

    from rpt import _build

    assert _build.LIB_AB.exists(), "librpt_ab.so missing: run __graft_entry__.build()"

    with tempfile.TemporaryDirectory() as d:
        np.savez(os.path.join(d, "in.npz"), lab=lab, ncl=ncl,
                 **{f"p{k}": p for k, (_, p, _) in enumerate(frames)})
        code = (
            "import sys, numpy as np, torch\n"
            f"sys.path[:0] = {sys.path!r}\n"
            "from test_path_gpu import _summaries_device\n"
            f"g = np.load({os.path.join(d, 'in.npz')!r})\n"
            f"frames = [(k, g[f'p{{k}}'], None) for k in range({len(frames)})]\n"
            "seg, fo, order = _summaries_device(torch.device('cuda:0'), frames, g['lab'],"
            " int(g['ncl']))\n"
            f"np.savez({os.path.join(d, 'out.npz')!r}, fo=fo, order=order,"
            " **{'s_' + k: v for k, v in seg.items()})\n")
        env = dict(os.environ, RPT_K9_RADIX="1", RPT_LIB=str(_build.LIB_AB))
        subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=240,
                       cwd=os.path.dirname(os.path.abspath(__file__)))
        o = np.load(os.path.join(d, "out.npz"))
        seg = {k[2:]: o[k] for k in o.files if k.startswith("s_")}
        return seg, o["fo"], o["order"]


@pytest.mark.parametrize("crowded", [False, True])
def test_summaries_chunked_frame_sort_matches_radix_path(gpu, crowded):
    """Frames of hundreds of thousands of points (the dense share's shape) take the frame sort
    with several blocks per frame (k_fsc_count / k_fsc_merge / k_fsc_scatter: a run spans
    chunks, each chunk's part placed after the earlier chunks'): the same segments, first
    points, counts and float32 centroids as the radix path and numpy, runs interleaved point by
    point across chunk boundaries, an empty frame, a giant run per frame; `crowded` puts more
    labels in one frame than the frame sort takes (redone on the radix path)."""
    rng = np.random.default_rng(33)
    sizes = [300000, 0, 250000, 180000, 70000, 3]
    frames, labs = [], []
    for k, m in enumerate(sizes):
        p = np.column_stack([rng.normal(0, 50, m), rng.normal(0, 50, m),
                             rng.integers(0, 255, m)]).astype(np.float32)
        lab = rng.integers(-1, 12 + 3 * k, m).astype(np.int32)
        lab[rng.random(m) < 0.7] = 5 + k  # one giant run per frame
        if crowded and k == 3:
            lab = rng.integers(-1, 4000, m).astype(np.int32)
        frames.append((k, p, None))
        labs.append(lab)
    lab = np.concatenate(labs)
    ncl = int(lab.max()) + 1
    a = _summaries_device(gpu, frames, lab, ncl)
    b = _radix_summaries_in_child(frames, lab, ncl)
    ka = np.lexsort((a[0]["label"], a[0]["frame"]))
    kb = np.lexsort((b[0]["label"], b[0]["frame"]))
    assert np.all(np.diff(a[0]["frame"]) >= 0) != crowded  # frame-major unless redone
    for key in a[0]:
        np.testing.assert_array_equal(a[0][key][ka], b[0][key][kb], err_msg=key)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0]["label"][a[2]], b[0]["label"][b[2]])
    pf = np.concatenate([np.full(m, k, np.int32) for k, m in enumerate(sizes)])
    pts = np.vstack([p for _, p, _ in frames])
    order = np.lexsort((np.arange(len(lab)), lab, pf))  # (frame, label) runs in index order
    key = pf.astype(np.int64)[order] * (ncl + 2) + lab[order] + 1
    heads = np.flatnonzero(np.r_[True, key[1:] != key[:-1]])
    ends = np.r_[heads[1:], len(key)]
    runs = {(int(pf[order[h]]), int(lab[order[h]])): order[h:e] for h, e in zip(heads, ends)
            if lab[order[h]] >= 0}
    assert len(runs) == len(a[0]["label"])
    for s in range(len(a[0]["label"])):
        idx = runs[(int(a[0]["frame"][s]), int(a[0]["label"][s]))]
        assert a[0]["count"][s] == len(idx) and a[0]["first"][s] == idx[0]
        c = np.mean(pts[idx][:, :2], axis=0)
        assert a[0]["cx"][s] == c[0] and a[0]["cy"][s] == c[1]


@pytest.mark.parametrize("crowded", [False, True])
def test_summaries_frame_sort_matches_radix_path(gpu, crowded):
    """K9's per-frame counting sort and its radix path (RPT_K9_RADIX=1, in a child process) give
    the same segments — frame-major vs label-major — on frames of ragged sizes, empty frames,
    noise-only frames, runs interleaved point by point, a run longer than a lane summarises and
    non-integer intensities (both checked against numpy); `crowded` adds a frame with more
    labels than the frame sort takes (the sync entry point then redoes K9 on the radix path)."""
    rng = np.random.default_rng(21)
    sizes = [0, 1, 63, 64, 65, 3000, 0, 517, 20000, 5, 0] + ([6000] if crowded else [])
    frames = []
    labs = []
    for k, m in enumerate(sizes):
        p = np.column_stack([rng.normal(0, 50, m), rng.normal(0, 50, m),
                             rng.integers(0, 255, m)]).astype(np.float32)
        lab = rng.integers(-1, 3000 if k == 11 else 40 + k, m).astype(np.int32)
        if k == 9:
            lab[:] = -1
        if k == 8:  # one run far longer than a lane takes (summarised by whole waves)
            lab[rng.random(m) < 0.6] = 7
        if k in (3, 8):  # non-integer intensities: numpy's pairwise sum (lane / wave forms)
            p[:, 2] = rng.random(m).astype(np.float32) * 255
        frames.append((k, p, None))
        labs.append(lab)
    lab = np.concatenate(labs)
    ncl = int(lab.max()) + 1
    a = _summaries_device(gpu, frames, lab, ncl)
    b = _radix_summaries_in_child(frames, lab, ncl)
    ka = np.lexsort((a[0]["label"], a[0]["frame"]))
    kb = np.lexsort((b[0]["label"], b[0]["frame"]))
    assert np.all(np.diff(a[0]["frame"]) >= 0) != crowded  # frame-major unless redone
    for key in a[0]:
        np.testing.assert_array_equal(a[0][key][ka], b[0][key][kb], err_msg=key)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0]["label"][a[2]], b[0]["label"][b[2]])
    pf = np.concatenate([np.full(m, k, np.int32) for k, m in enumerate(sizes)])
    pts = np.vstack([p for _, p, _ in frames])
    for s in range(len(a[0]["label"])):
        m = (pf == a[0]["frame"][s]) & (lab == a[0]["label"][s])
        assert a[0]["count"][s] == m.sum()
        assert a[0]["first"][s] == np.nonzero(m)[0][0]
        c = np.mean(pts[m][:, :2], axis=0)
        assert a[0]["cx"][s] == c[0] and a[0]["cy"][s] == c[1]
        assert float(a[0]["mi"][s]) == float(np.mean(pts[m][:, 2]))
    assert len(a[0]["label"]) == len({(f, l) for f, l in zip(pf, lab) if l >= 0})


@pytest.mark.parametrize("n_frames,land", [(6, True), (14, True), (14, False)])
def test_stack_path_matches_oracle(gpu, n_frames, land):
    """echo in HBM -> K1 -> land -> ST-DBSCAN -> K9 -> order -> C++ tracker, against the oracle
    run of the same stages (oracle.run_path)."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    cfg = SynthConfig(n_frames=n_frames, rows=1024, n_targets=14, clutter_density=0.01)
    ds = DeviceSynth(cfg, gpu)
    echo_d = ds.echo()
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(land_filter=land), gpu)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      n_frames * len(cfg.gains))
    frames = _oracle_stack(echo_d.cpu().numpy(), cfg, ds.geo)
    o_frames, o_labels, o_clusters, o_trk = op.run_path(frames, land=land)
    # twice: the second run reuses the driver's buffers
    for _ in range(2):
        res = pipe.run(echo_d, keep_points=True)
        _check_stack_vs_oracle(res, n_frames, frames, o_frames, o_labels, o_clusters, o_trk)


def test_k1_grouped_u8_matches_generic_rows(gpu):
    """The grouped u8 kernels (1024 bins: keep bits by SWAR + dot4 mask, group prefix) against the
    generic per-row kernels on the same samples (a 2048-bin sweep runs the generic u8 path, and
    its two 1024-bin halves as separate sweeps the grouped one) at thresholds on both sides of 127,
    with short last groups (rows % 4 != 0) and strides 1, 3, 4."""
    rng = np.random.default_rng(5)
    for rows in (4093, 8):
        wide = rng.integers(0, 256, (2, rows, 2048)).astype(np.uint8)
        scale = [np.full(rows, 30.0, np.float32)] * 2
        angle = [np.linspace(0, 359, rows).astype(np.float32)] * 2
        for thr in (-3.0, 10.0, 127.5, 128.0, 200.0, 254.9, 255.0):
            for stride in (1, 3, 4):
                a = _k1(gpu, wide, scale, angle, threshold=thr, stride=stride)
                # same samples as 1024-bin sweeps: per-row keep order is bins 0..2047 of a row
                # in the wide layout vs two rows here, so compare kept (value) streams and counts
                narrow = wide.reshape(2, rows * 2, 1024)
                b = _k1(gpu, narrow, [np.repeat(sc, 2) for sc in scale],
                        [np.repeat(an, 2) for an in angle], threshold=thr, stride=stride)
                np.testing.assert_array_equal(a[2], b[2])  # intensities, in rank order
                np.testing.assert_array_equal(a[5], b[5])  # file offsets
                ref = _k1(gpu, narrow.astype(np.float32), [np.repeat(sc, 2) for sc in scale],
                          [np.repeat(an, 2) for an in angle], threshold=thr, stride=stride,
                          f32=True)
                for i in range(5):
                    np.testing.assert_array_equal(b[i], ref[i])


def test_k1_staged_entries_match_two_full_reads(gpu):
    """The staged K1 (the count pass stores the kept samples of every group keeping <= 128 of
    them, the write pass reads those instead of the echo; denser groups read the echo again)
    against the two-full-read kernels: thresholds on both sides of 127 and at the ends, strides
    1/3/4/7, short last groups, an empty file between others, and densities from all-staged to
    none-staged with mixed groups in between, and a nearly empty stack whose 1024-output tiles
    span more groups than the expand write's LDS window (its global-search fallback)."""
    rng = np.random.default_rng(17)
    for rows, p in ((4096, 0.02), (1023, 0.5), (6, 1.0), (37, 0.0), (512, 0.03), (4096, 2e-5)):
        echo = np.where(rng.random((6, rows, 1024)) < p, rng.integers(0, 256, (6, rows, 1024)),
                        0).astype(np.uint8)
        echo[2] = 0
        scale = [np.full(rows, 231.5, np.float32)] * 6
        angle = [np.linspace(0, 8000, rows).astype(np.float32)] * 6
        for thr in (-3.0, 10.0, 127.5, 200.0, 255.0):
            for stride in (1, 3, 4, 7):
                a = _k1(gpu, echo, scale, angle, gains=(40, 50, 75), threshold=thr, stride=stride)
                b = _k1(gpu, echo, scale, angle, gains=(40, 50, 75), threshold=thr, stride=stride,
                        staged=True)
                for i in range(6):
                    np.testing.assert_array_equal(a[i], b[i])


def test_speculative_k1_write_regrows(gpu):
    """The stack driver queues K1's write with the capacity of the previous run; a denser stack
    after a sparse one overflows it, and the driver must grow the buffers and write again: same
    result as a fresh pipeline."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    sparse = SynthConfig(n_frames=12, rows=1024, clutter_density=0.002)
    dense = SynthConfig(n_frames=12, rows=1024, clutter_density=0.03)
    e_sparse = DeviceSynth(sparse, gpu).echo()
    ds = DeviceSynth(dense, gpu)
    e_dense = ds.echo()
    torch.cuda.synchronize(gpu)
    pipes = []
    for _ in range(2):
        p = FrameStackPipeline(dense.gains, dense.rows, dense.bins, PathParams(), gpu)
        p.set_geometry(np.full(dense.rows, dense.scale, np.float32), ds.geo.cos_t,
                       ds.geo.sin_t, dense.n_frames * 3)
        pipes.append(p)
    a0 = pipes[0].run(e_sparse, keep_points=True)
    a = pipes[0].run(e_dense, keep_points=True)   # capacity from the sparse run: regrow
    b = pipes[1].run(e_dense, keep_points=True)   # fresh
    assert a.n_points > a0.n_points
    assert a.n_points == b.n_points
    for k in a.points:
        assert torch.equal(a.points[k], b.points[k]), k
    assert torch.equal(a.labels, b.labels)
    for k in a.seg:
        np.testing.assert_array_equal(a.seg[k], b.seg[k])


@pytest.mark.parametrize("rows,thr,stride,p", [(1000, 10.0, 1, 0.02), (1000, 127.5, 3, 0.1),
                                               (4093, 200.0, 4, 0.08), (16, -3.0, 1, 1.0),
                                               (1000, 10.0, 1, 0.25)])
def test_k1_stack_driver_matches_public_k1(gpu, rows, thr, stride, p):
    """The stack driver's K1 (staged count, speculative capacity-bounded write, regrow) against
    the public rpt_polar_count/write on the same sparse random sweeps: thresholds on both sides of
    127, strides 1 / 3 / 4, row counts that are not multiples of the 4-row group or 64, densities
    from sparse to dense (the last case keeps more than 256 samples in most groups: the unstaged
    write), every pipeline run twice (buffers regrown on the first run, reused on the second)."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.core.transforms import trig_tables

    rng = np.random.default_rng(rows + int(thr) + stride)
    F, gains = 2, (40, 50, 75)
    vals = rng.integers(0, 256, (F * 3, rows, 1024))
    echo = np.where(rng.random((F * 3, rows, 1024)) < p, vals, 0).astype(np.uint8)
    scale = np.full(rows, 231.5, np.float32)
    angle = np.floor(np.arange(rows) * 8196 / rows).astype(np.float32)
    ref = _k1(gpu, echo, [scale] * (F * 3), [angle] * (F * 3), gains=gains, threshold=thr,
              stride=stride)
    ct, st_ = trig_tables(angle)
    pipe = FrameStackPipeline(gains, rows, 1024, PathParams(threshold=thr, stride=stride,
                                                           land_filter=False), gpu)
    pipe.set_geometry(scale, ct, st_, F * 3)
    ed = torch.from_numpy(echo.reshape(F, 3, rows, 1024)).to(gpu)
    for _ in range(2):
        res = pipe.run(ed, keep_points=True)
        assert res.n_points == len(ref[0])
        got = [res.points[k].cpu().numpy() for k in ("x", "y", "v", "gain", "frame")]
        for a, b, name in zip(got, ref[:5], ("x", "y", "v", "gain", "frame")):
            np.testing.assert_array_equal(a, b, err_msg=name)


@pytest.mark.parametrize("lanes,k1_gate", [(2, False), (3, True)])
def test_concurrent_lanes_match_single_lane(gpu, lanes, k1_gate):
    """Two or three lanes (native handles on their own streams, submitted from as many threads,
    the library's scratch, scan state and zeroed counters per stream; with k1_gate the lanes'
    K1 passes take turns, rpt_k1_gate) give the same results as one lane, run after run: four
    stacks of different content spread over the lanes."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    stacks = []
    for k in range(4):
        cfg = SynthConfig(n_frames=14, rows=1024, frame0=100 * k)
        ds = DeviceSynth(cfg, gpu)
        stacks.append(ds.echo())
    torch.cuda.synchronize(gpu)
    one = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), gpu)
    two = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), gpu, lanes=lanes,
                             async_host=True, k1_gate=k1_gate)
    for p in (one, two):
        p.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                       cfg.n_frames * 3)
    ref = [one.run(e, keep_points=True) for e in stacks]
    futs = [two.submit(e, keep_points=True) for e in stacks]
    got = [f.result().finish() for f in futs]
    for a, b in zip(ref, got):
        assert a.n_points == b.n_points and a.n_clusters == b.n_clusters
        assert torch.equal(a.labels, b.labels)
        for k in a.seg:
            np.testing.assert_array_equal(a.seg[k], b.seg[k])
        oa, ob = a.tracker.objects(), b.tracker.objects()
        assert [o.object_id for o in oa] == [o.object_id for o in ob]


def test_full_size_partition_is_order_invariant(gpu):
    """Bench-size frames (4096x1024, 3 gains): the ST-DBSCAN partition must not depend on point
    order (size-independent property; labels renumber by first core index)."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.processors.clustering import st_dbscan_soa
    from rpt.synth import DeviceSynth, SynthConfig

    cfg = SynthConfig(n_frames=12)
    ds = DeviceSynth(cfg, gpu)
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), gpu)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      cfg.n_frames * 3)
    res = pipe.run(ds.echo(), keep_points=True)
    x, y = res.points["x"], res.points["y"]
    t = res.points["frame"].to(torch.float32)
    lab = res.labels.cpu().numpy()
    perm = torch.randperm(x.numel(), device=gpu, generator=torch.Generator(gpu).manual_seed(0))
    lab2 = st_dbscan_soa(x[perm].contiguous(), y[perm].contiguous(), t[perm].contiguous(),
                         8.0, 2.0, 15).cpu().numpy()
    back = np.empty_like(lab2)
    back[perm.cpu().numpy()] = lab2
    # noise/border status is order-free; ids and ties between clusters are not (the reference
    # numbers clusters by first core point and gives a border point the smallest adjacent id)
    assert ((lab < 0) == (back < 0)).all()
    m = np.nonzero(lab >= 0)[0]
    pairs, cnt = np.unique(np.stack([lab[m], back[m]], 1), axis=0, return_counts=True)
    major = {}
    for (a, b), c in zip(pairs.tolist(), cnt.tolist()):
        if c > major.get(a, (None, -1))[1]:
            major[a] = (b, c)
    assert len({v[0] for v in major.values()}) == len(major)  # bijection between partitions
    dev = m[np.array([back[i] != major[lab[i]][0] for i in m], bool)]
    assert len(dev) < 0.001 * len(m)
    if len(dev):  # every disagreement must be a border point (fewer than min_samples nbrs)
        xh, yh, th = x.cpu().numpy(), y.cpu().numpy(), t.cpu().numpy()
        for i in dev[:200]:
            w = np.abs(th - th[i]) <= 2.0
            d2 = (xh[w].astype(np.float64) - xh[i]) ** 2 + (yh[w].astype(np.float64) - yh[i]) ** 2
            assert int((d2 <= 64.0).sum()) < 15
    assert res.n_clusters > 10 and res.n_segments > 100


def test_stack_points_gain_needs_gain_table(gpu):
    """Without keep_points the pipeline runs rpt_stack_run with no gain table (no per-point gains
    are written); rpt_stack_points must then refuse a gain output instead of copying stale
    values, and still hand back the other arrays."""
    from rpt import _abi
    from rpt._device import stream_handle
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    cfg = SynthConfig(n_frames=12, rows=512)
    ds = DeviceSynth(cfg, gpu)
    echo = ds.echo()
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), gpu)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      cfg.n_frames * 3)
    a = pipe.run(echo, keep_points=True)
    res = pipe.run(echo)  # no gain table
    n = res.n_clustered_input
    assert n == a.n_clustered_input
    lib = _abi.load()
    g = torch.empty(n, dtype=torch.int32, device=gpu)
    x = torch.empty(n, dtype=torch.float32, device=gpu)
    st = stream_handle(gpu)
    assert lib.rpt_stack_points(pipe._h, None, None, None, g.data_ptr(), None, None, st) == \
        _abi.RPT_EINVAL
    assert lib.rpt_stack_points(pipe._h, x.data_ptr(), None, None, None, None, None, st) == 0
    torch.cuda.synchronize(gpu)
    assert torch.equal(x, a.points["x"])
