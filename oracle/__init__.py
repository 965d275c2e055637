"""TEST INFRASTRUCTURE ONLY — the parity oracle for the rpt hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the timed CPU baseline; the product (``rpt`` +
``librpt.so``) never imports or links it.

Contents — a CPU restatement of the reference algorithm for every row of SURVEY.md §8a, each
function citing the reference file:line it follows (paths relative to the reference root):

* ``stdbscan``          BFS ST-DBSCAN, C (``stdbscan_oracle.c``) — 3_stdbscan_point_clouds.py:101-136
* ``stdbscan_uf``       the same labels by the set formulation, OpenMP (large stacks)
* ``stdbscan_denoise``  the denoise variant, C — PointCloudWorkF/stdbscan_denoising_pipeline.py:264-369
* ``polar_scatter``     4_temporal_object_tracker.py:200-232 arithmetic on an echo matrix
* ``build_frames``      build_frame :312-352 concatenation
* ``land_filter``       :359-436
* ``frame_clusters``    :508-536 (per-frame Cluster list in CPython set order)
* ``Tracker``           ObjectTracker :543-688 with the exact numpy dtype flow
* ``run_path``          stage order of run_pipeline :941-991 (no file I/O)

Pinned by ``tests/golden/*.npz`` — vectors produced by running the reference itself in the
build container (``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks every
function here against them.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from .path import (  # noqa: F401
    ANGLE_SCALE,
    build_frames,
    frame_clusters,
    land_filter,
    polar_scatter,
    run_path,
    trig_tables,
)
from .tracker import Tracker  # noqa: F401

_HERE = Path(__file__).resolve().parent
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        so = _HERE / "liboracle.so"
        if not so.exists():
            import subprocess

            subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
        lib = C.CDLL(str(so))
        lib.oracle_stdbscan.restype = C.c_int32
        lib.oracle_stdbscan.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64,
                                        C.c_double, C.c_double, C.c_int32, C.c_void_p]
        lib.oracle_stdbscan_uf.restype = C.c_int32
        lib.oracle_stdbscan_uf.argtypes = lib.oracle_stdbscan.argtypes
        lib.oracle_stdbscan_denoise.restype = C.c_int32
        lib.oracle_stdbscan_denoise.argtypes = lib.oracle_stdbscan.argtypes[:7] + [
            C.c_int32, C.c_void_p]
        lib.oracle_sample_check.restype = C.c_int32
        lib.oracle_sample_check.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64,
                                            C.c_double, C.c_double, C.c_void_p, C.c_int64,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p]
        lib.oracle_neighbour_counts.restype = C.c_int32
        lib.oracle_neighbour_counts.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64,
                                                C.c_double, C.c_double, C.c_void_p]
        _LIB = lib
    return _LIB


def _prep(coords, times):
    c = np.ascontiguousarray(coords, dtype=np.float32)
    if c.ndim != 2:
        raise ValueError("coords must be 2-D")
    t = np.ascontiguousarray(times, dtype=np.float32)
    return c, t


def stdbscan(coords, times, eps_space: float, eps_time: float, min_samples: int) -> np.ndarray:
    """Reference BFS labels (3_stdbscan_point_clouds.py:101-136) for float32 coords/times."""
    c, t = _prep(coords, times)
    n = c.shape[0]
    if n == 0:
        raise ValueError("Found array with 0 sample(s)")
    labels = np.empty(n, dtype=np.int32)
    r = _lib().oracle_stdbscan(c.ctypes.data, c.shape[1], t.ctypes.data, n, float(eps_space),
                               float(eps_time), int(min_samples), labels.ctypes.data)
    if r < 0:
        raise MemoryError("oracle_stdbscan failed")
    return labels


def stdbscan_uf(coords, times, eps_space: float, eps_time: float, min_samples: int) -> np.ndarray:
    """The same labels by the set formulation (core counts, core-core components numbered by
    minimum index, border = smallest adjacent id), OpenMP-parallel: the checker for stacks too
    large for the sequential BFS.  Pinned to ``stdbscan`` by tests/test_oracle_golden.py."""
    c, t = _prep(coords, times)
    n = c.shape[0]
    if n == 0:
        raise ValueError("Found array with 0 sample(s)")
    labels = np.empty(n, dtype=np.int32)
    r = _lib().oracle_stdbscan_uf(c.ctypes.data, c.shape[1], t.ctypes.data, n, float(eps_space),
                                  float(eps_time), int(min_samples), labels.ctypes.data)
    if r < 0:
        raise MemoryError("oracle_stdbscan_uf failed")
    return labels


def stdbscan_denoise(coords, times, eps_space: float, eps_time: float, min_samples: int,
                     min_frames: int = 2) -> np.ndarray:
    """Labels of the denoise variant (PointCloudWorkF/stdbscan_denoising_pipeline.py:264-369:
    min_frames core condition, FIFO expansion), the reference's loop restated in C."""
    c, t = _prep(coords, times)
    n = c.shape[0]
    labels = np.empty(n, dtype=np.int32)
    if n == 0:
        return labels
    r = _lib().oracle_stdbscan_denoise(c.ctypes.data, c.shape[1], t.ctypes.data, n,
                                       float(eps_space), float(eps_time), int(min_samples),
                                       int(min_frames), labels.ctypes.data)
    if r < 0:
        raise MemoryError("oracle_stdbscan_denoise failed")
    return labels


def sample_check(coords, times, eps_space: float, eps_time: float, idx, core, labels):
    """For the sample points idx: exact neighbour counts (self included) and the smallest /
    largest label among their core neighbours under the CLAIMED core flags and labels of every
    point (-1 when none) -- the checker for full-size runs the oracle cannot label whole."""
    c, t = _prep(coords, times)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    core = np.ascontiguousarray(core, dtype=np.uint8)
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    assert core.shape[0] == labels.shape[0] == c.shape[0]
    cnt = np.empty(len(idx), np.int64)
    lo = np.empty(len(idx), np.int32)
    hi = np.empty(len(idx), np.int32)
    r = _lib().oracle_sample_check(c.ctypes.data, c.shape[1], t.ctypes.data, c.shape[0],
                                   float(eps_space), float(eps_time), idx.ctypes.data, len(idx),
                                   core.ctypes.data, labels.ctypes.data, cnt.ctypes.data,
                                   lo.ctypes.data, hi.ctypes.data)
    if r < 0:
        raise ValueError("oracle_sample_check needs integral finite times (grid mode)")
    return cnt, lo, hi


def neighbour_counts(coords, times, eps_space: float, eps_time: float) -> np.ndarray:
    c, t = _prep(coords, times)
    out = np.empty(c.shape[0], dtype=np.int64)
    _lib().oracle_neighbour_counts(c.ctypes.data, c.shape[1], t.ctypes.data, c.shape[0],
                                   float(eps_space), float(eps_time), out.ctypes.data)
    return out
