"""Parity of the HIP ST-DBSCAN (rpt_stdbscan through the C-ABI) with the reference: the golden
labels produced by running the reference, and the pinned C oracle on seeded clouds.  Labels must
be bit-identical (same ids, not just the same partition)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _st(coords, times, eps, et, ms):
    from rpt.processors import st_dbscan

    return st_dbscan(coords, times, eps, et, ms)


def test_golden_reference_labels(gpu, golden):
    g = golden("g2_stdbscan.npz")
    for k in range(int(g["n_cases"])):
        eps, et, ms = g[f"c{k}_params"]
        lab = _st(g[f"c{k}_coords"], g[f"c{k}_times"], eps, et, int(ms))
        np.testing.assert_array_equal(lab, g[f"c{k}_labels"], err_msg=f"case {k} {g[f'c{k}_kind']}")


def _blobs(rng, F, n_blobs, per, noise, spread=2.0, box=200.0, dim=2):
    pts, ts = [], []
    centers = rng.random((n_blobs, dim)) * box - box / 2
    vel = rng.normal(0, 1.5, (n_blobs, dim))
    for f in range(F):
        for c, v in zip(centers, vel):
            m = int(rng.integers(per // 2, per * 2))
            pts.append(c + v * f + rng.normal(0, spread, (m, dim)))
            ts.append(np.full(m, f))
        pts.append(rng.random((noise, dim)) * box * 1.2 - box * 0.6)
        ts.append(np.full(noise, f))
    return np.vstack(pts).astype(np.float32), np.concatenate(ts).astype(np.float32)


CASES = []
for seed in range(12):
    CASES.append(("blobs2d", seed))
for seed in range(6):
    CASES.append(("uniform2d", seed))
for seed in range(6):
    CASES.append(("ply3d", seed))
for seed in range(4):
    CASES.append(("floattime", seed))
for seed in range(4):
    CASES.append(("lattice", seed))
for seed in range(4):
    CASES.append(("widetime2d", seed))


def _make(kind, seed):
    rng = np.random.default_rng(1000 + seed)
    if kind == "blobs2d":
        F = int(rng.integers(1, 12))
        c, t = _blobs(rng, F, int(rng.integers(2, 15)), int(rng.integers(10, 120)),
                      int(rng.integers(10, 200)), spread=float(rng.choice([1.0, 2.5, 4.0])))
        return c, t, float(rng.choice([3.0, 5.0, 8.0])), float(rng.choice([0.0, 1.0, 2.0, 3.0])), \
            int(rng.choice([1, 2, 5, 10, 15, 40]))
    if kind == "uniform2d":
        n = int(rng.integers(1000, 20000))
        c = (rng.random((n, 2)) * rng.choice([50, 200, 1000])).astype(np.float32)
        t = rng.integers(0, int(rng.integers(1, 20)), n).astype(np.float32)
        return c, t, float(rng.choice([1.0, 4.0, 8.0, 15.0])), float(rng.choice([0.0, 1.0, 2.0])), \
            int(rng.choice([2, 4, 8, 15]))
    if kind == "ply3d":
        c, t = _blobs(rng, 3, int(rng.integers(2, 10)), 80, 150, spread=2.0, dim=3)
        return c, t, float(rng.choice([3.0, 5.0])), 1.0, int(rng.choice([5, 10]))
    if kind == "floattime":
        n = int(rng.integers(500, 5000))
        c = (rng.random((n, 2)) * 60).astype(np.float32)
        t = (rng.random(n) * rng.choice([3, 10, 100])).astype(np.float32)
        return c, t, 3.0, float(rng.choice([0.25, 0.5, 1.3, 2.7])), int(rng.choice([3, 6]))
    if kind == "lattice":
        s = int(rng.integers(20, 60))
        gx, gy = np.meshgrid(np.arange(s), np.arange(s))
        c = (np.column_stack([gx.ravel(), gy.ravel()]) * float(rng.choice([1, 2, 0.5]))).astype(np.float32)
        keep = rng.random(len(c)) < 0.6
        c = c[keep]
        t = rng.integers(0, 4, len(c)).astype(np.float32)
        return c, t, float(rng.choice([1.0, 2.0, 3.0])), float(rng.choice([0.0, 1.0])), \
            int(rng.choice([2, 3, 5, 7]))
    if kind == "widetime2d":  # forward slab windows of >= 128 cells (the union passes' walk)
        F = int(rng.integers(12, 30))
        c, t = _blobs(rng, F, int(rng.integers(3, 10)), int(rng.integers(10, 60)), 60,
                      spread=2.5)
        return c, t, float(rng.choice([5.0, 8.0])), float(rng.choice([4.0, 6.0, 9.0])), \
            int(rng.choice([10, 30, 60]))
    raise ValueError(kind)


@pytest.mark.parametrize("kind,seed", CASES)
def test_matches_oracle_seeded(gpu, kind, seed):
    c, t, eps, et, ms = _make(kind, seed)
    exp = oracle.stdbscan(c, t, eps, et, ms)
    got = _st(c, t, eps, et, ms)
    np.testing.assert_array_equal(got, exp, err_msg=f"{kind}/{seed} n={len(c)} eps={eps} et={et} ms={ms}")


def test_torch_in_torch_out(gpu):
    rng = np.random.default_rng(7)
    c, t = _blobs(rng, 4, 6, 50, 50)
    exp = oracle.stdbscan(c, t, 8.0, 2.0, 15)
    got = _st(torch.from_numpy(c).to(gpu), torch.from_numpy(t).to(gpu), 8.0, 2.0, 15)
    assert isinstance(got, torch.Tensor) and got.dtype == torch.int32 and got.is_cuda
    np.testing.assert_array_equal(got.cpu().numpy(), exp)


def test_large_stack_vs_oracle(gpu):
    """Radar-like stack: 40 frames of dense targets + clutter (~120k points); exercises multi-pass
    radix sort, thousands of cells and long union chains across frames."""
    rng = np.random.default_rng(99)
    c, t = _blobs(rng, 40, 25, 100, 400, spread=2.5, box=400.0)
    exp = oracle.stdbscan(c, t, 8.0, 2.0, 15)
    got = _st(c, t, 8.0, 2.0, 15)
    np.testing.assert_array_equal(got, exp)


def test_identical_points_single_cell(gpu):
    c = np.zeros((5000, 2), np.float32)
    t = np.zeros(5000, np.float32)
    np.testing.assert_array_equal(_st(c, t, 1.0, 0.0, 10), np.zeros(5000, np.int32))
    np.testing.assert_array_equal(_st(c, t, 0.0, 0.0, 10), np.zeros(5000, np.int32))
    np.testing.assert_array_equal(_st(c[:5], t[:5], 1.0, 0.0, 10), np.full(5, -1, np.int32))


def test_degenerate_parameters(gpu):
    rng = np.random.default_rng(3)
    c = (rng.random((300, 2)) * 10).astype(np.float32)
    t = np.zeros(300, np.float32)
    for eps, et, ms in [(-1.0, 1.0, 3), (2.0, -1.0, 3), (-1.0, 1.0, 0), (2.0, 1.0, 0),
                        (2.0, 1.0, 1), (0.0, 0.0, 1), (1e9, 1e9, 5), (1e-6, 0.0, 2)]:
        np.testing.assert_array_equal(_st(c, t, eps, et, ms), oracle.stdbscan(c, t, eps, et, ms),
                                      err_msg=f"eps={eps} et={et} ms={ms}")


def test_nonfinite_times_are_isolated(gpu):
    rng = np.random.default_rng(4)
    c = (rng.random((400, 2)) * 10).astype(np.float32)
    t = rng.integers(0, 3, 400).astype(np.float32)
    t[::7] = np.nan
    t[::11] = np.inf
    for ms in (0, 1, 4):
        np.testing.assert_array_equal(_st(c, t, 2.0, 1.0, ms), oracle.stdbscan(c, t, 2.0, 1.0, ms))


def test_wide_extent_coarsened_grid(gpu):
    """Extent / eps far beyond the dense-grid budget: the grid coarsens, results stay exact."""
    rng = np.random.default_rng(5)
    c = np.vstack([(rng.random((2000, 2)) * 3).astype(np.float32),
                   np.array([[1e6, -1e6], [-1e6, 1e6]], np.float32)])
    t = np.zeros(len(c), np.float32)
    np.testing.assert_array_equal(_st(c, t, 0.05, 0.0, 3), oracle.stdbscan(c, t, 0.05, 0.0, 3))


def test_errors(gpu):
    with pytest.raises(ValueError):
        _st(np.zeros((0, 2), np.float32), np.zeros(0, np.float32), 1.0, 1.0, 2)
    bad = np.zeros((10, 2), np.float32)
    bad[3, 1] = np.nan
    with pytest.raises(ValueError):
        _st(bad, np.zeros(10, np.float32), 1.0, 1.0, 2)


def test_integer_and_f64_times(gpu):
    rng = np.random.default_rng(6)
    c, t = _blobs(rng, 5, 5, 40, 30)
    exp = oracle.stdbscan(c, t, 5.0, 1.0, 8)
    np.testing.assert_array_equal(_st(c, t.astype(np.int64), 5.0, 1.0, 8), exp)
    np.testing.assert_array_equal(_st(c, t.astype(np.float64), 5.0, 1.9, 8), exp)
