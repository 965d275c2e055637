"""Synthetic 1024-echo radar sweeps for the benchmark and the parity tests.

A frame is n_gains sweeps (gains 40/50/75) of rows=4096 azimuths x bins=1024 range samples of
u8 echo, generated ON DEVICE by ``rpt_synth_echo`` from integer hashes (splitmix64), so the input
is bit-reproducible and ``numpy_echo`` below restates the generator exactly for small cases.

Scene (seeded): K disc targets (radius 2.5-5.5 m, 40-215 m range) — half stationary buoys, half
boats moving 0.5-2 m/frame and bouncing inside that annulus — echo 60-99 with fill 0.8; a
persistent land sector (echo 150-255, fill ~0.1, > 180 m) that the reference's land filter
removes; Cartesian-uniform clutter (echo 11-39) kept below the density at which ST-DBSCAN would
chain it into one component.  Target echoes stay below LAND_MIN_INTENSITY=100 on purpose: the
reference's land filter counts points, not frames (4_temporal_object_tracker.py:388, :401), so
any dense bright target persisting over a 5 m cell would otherwise be classified as land.

Geometry (per-row Angle, Scale, cos/sin tables; per-frame target discs and their polar
bounding boxes) is computed on the host once, like the Scale/Angle columns of a CSV.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np

from .core.transforms import ANGLE_SCALE, trig_tables

M64 = (1 << 64) - 1


@dataclass
class SynthConfig:
    n_frames: int = 100
    rows: int = 4096
    bins: int = 1024
    gains: Tuple[int, ...] = (40, 50, 75)
    scale: float = 231.5
    n_targets: int = 56
    seed: int = 0
    target_seed: int = 123
    clutter_density: float = 0.012          # kept echo cells per m^2 per sweep (before stride)
    gain_sensitivity: Tuple[float, ...] = (0.7, 0.85, 1.0)
    target_fill: float = 0.8
    land_fill: float = 0.1
    land_deg: Tuple[float, float] = (300.0, 330.0)
    land_min_range: float = 181.0
    frame0: int = 0                          # absolute index of the first frame (sharding)


# BASELINE.json configs[4] ("dense full sweep, ~500k pts/frame"): Cartesian-uniform clutter at
# ~4.2 kept echo cells per m^2 per sweep.  Expected points per frame ~= density * 107k (3 gains,
# sensitivities 0.7/0.85/1.0, stride 4, 231.5 m) + ~48k target/land points.  At this density every
# clutter point is core and ST-DBSCAN chains the whole stack into one component: a stress case
# for the union-find and the per-(frame, label) reductions, as SURVEY.md §8(d) describes it.
DENSE_CLUTTER_DENSITY = 4.2


def dense_config(n_frames: int = 125, **kw) -> "SynthConfig":
    return SynthConfig(n_frames=n_frames, clutter_density=DENSE_CLUTTER_DENSITY, **kw)


@dataclass
class SynthGeometry:
    angle: np.ndarray          # Angle column (float32 units of 360/8196 deg)
    cos_t: np.ndarray          # float32 [rows]
    sin_t: np.ndarray
    clutter_thresh: np.ndarray  # uint32 [n_gains][bins]
    targets: np.ndarray         # float32 [n_frames][K][4]: tx, ty, r^2, 0
    target_rows: np.ndarray     # int32 [n_frames][K][2]
    target_bins: np.ndarray     # int32 [n_frames][K][2]
    land_rows: Tuple[int, int]
    land_bin0: int
    target_fill_u8: int
    land_fill_u8: int
    info: dict = field(default_factory=dict)


def _angles(rows: int) -> np.ndarray:
    return np.floor(np.arange(rows) * 8196 / rows).astype(np.float32)


def _trajectories(cfg: SynthConfig, n_total: int):
    """Target centres for absolute frames [0, n_total): float64 [n_total][K][2], radii [K]."""
    rng = np.random.default_rng(cfg.target_seed)
    K = cfg.n_targets
    rho = rng.uniform(45.0, 210.0, K)
    th = rng.uniform(0.35, 2 * np.pi - 0.35, K)
    rad = rng.uniform(2.5, 5.5, K)
    speed = np.where(np.arange(K) % 2 == 0, 0.0, rng.uniform(0.5, 2.0, K))
    head = rng.uniform(0, 2 * np.pi, K)
    p = np.column_stack([rho * np.cos(th), rho * np.sin(th)])
    v = np.column_stack([speed * np.cos(head), speed * np.sin(head)])
    out = np.empty((n_total, K, 2))
    for f in range(n_total):
        out[f] = p
        p = p + v
        r = np.hypot(p[:, 0], p[:, 1])
        bad = (r > 215.0) | (r < 40.0)
        if bad.any():
            nrm = p[bad] / r[bad, None]
            vb = v[bad]
            v[bad] = vb - 2 * np.sum(vb * nrm, axis=1)[:, None] * nrm
            p[bad] = p[bad] + 2 * v[bad]
    return out, rad


def make_geometry(cfg: SynthConfig) -> SynthGeometry:
    rows, bins = cfg.rows, cfg.bins
    angle = _angles(rows)
    cos_t, sin_t = trig_tables(angle)
    theta = angle.astype(np.float64) * (2 * np.pi / 8196.0)  # row azimuth (rad), increasing
    dr = cfg.scale / bins
    dth = 2 * np.pi / rows
    # clutter: Bernoulli per cell with p = density * cell area (Cartesian-uniform)
    area = np.arange(bins, dtype=np.float64) * dr * dth * dr
    thr = np.zeros((len(cfg.gains), bins), dtype=np.uint32)
    for g in range(len(cfg.gains)):
        sens = cfg.gain_sensitivity[g] if g < len(cfg.gain_sensitivity) else 1.0
        pr = np.clip(cfg.clutter_density * sens * area, 0.0, 1.0 - 2.0**-32)
        thr[g] = np.floor(pr * 2.0**32).astype(np.uint32)
    n_total = cfg.frame0 + cfg.n_frames
    cen, rad = _trajectories(cfg, n_total)
    cen = cen[cfg.frame0:]
    K = cfg.n_targets
    tg = np.zeros((cfg.n_frames, K, 4), np.float32)
    tg[:, :, 0] = cen[:, :, 0].astype(np.float32)
    tg[:, :, 1] = cen[:, :, 1].astype(np.float32)
    tg[:, :, 2] = (rad.astype(np.float32) ** 2)[None, :]
    rho = np.hypot(cen[:, :, 0], cen[:, :, 1])
    phi = np.mod(np.arctan2(cen[:, :, 1], cen[:, :, 0]), 2 * np.pi)
    half = np.arcsin(np.clip((rad[None, :] + 1.0) / rho, 0.0, 1.0)) + 3 * dth
    r_lo = np.searchsorted(theta, phi - half, side="left")
    r_hi = np.searchsorted(theta, phi + half, side="right") - 1
    trows = np.stack([np.clip(r_lo, 0, rows - 1), np.clip(r_hi, 0, rows - 1)], -1).astype(np.int32)
    b_lo = np.floor((rho - rad[None, :] - 1.0) / dr)
    b_hi = np.ceil((rho + rad[None, :] + 1.0) / dr)
    tbins = np.stack([np.clip(b_lo, 0, bins - 1), np.clip(b_hi, 0, bins - 1)], -1).astype(np.int32)
    l0 = int(np.searchsorted(theta, math.radians(cfg.land_deg[0])))
    l1 = int(np.searchsorted(theta, math.radians(cfg.land_deg[1])))
    lb0 = int(math.ceil(cfg.land_min_range / dr))
    return SynthGeometry(angle=angle, cos_t=cos_t, sin_t=sin_t, clutter_thresh=thr, targets=tg,
                         target_rows=trows, target_bins=tbins, land_rows=(l0, l1), land_bin0=lb0,
                         target_fill_u8=int(round(cfg.target_fill * 256)),
                         land_fill_u8=int(round(cfg.land_fill * 256)),
                         info={"radius": rad})


# ----------------------------------------------------------------- numpy restatement (tests)
def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def numpy_echo(cfg: SynthConfig, geo: SynthGeometry, frames: Optional[range] = None
               ) -> np.ndarray:
    """Bit-identical numpy restatement of k_synth (csrc/polar.hip) for local frames `frames`."""
    frames = range(cfg.n_frames) if frames is None else frames
    G, R, B = len(cfg.gains), cfg.rows, cfg.bins
    out = np.zeros((len(frames), G, R, B), np.uint8)
    rr = np.arange(R, dtype=np.uint64)[:, None]
    bb = np.arange(B, dtype=np.uint64)[None, :]
    step = np.float32(cfg.scale) / np.float32(B)
    rng_f = step * np.arange(B, dtype=np.float32)
    xx = rng_f[None, :] * geo.cos_t[:, None]
    yy = rng_f[None, :] * geo.sin_t[:, None]
    land = np.zeros((R, B), bool)
    land[geo.land_rows[0]:geo.land_rows[1], geo.land_bin0:] = True
    with np.errstate(over="ignore"):
        for li, fl in enumerate(frames):
            fa = cfg.frame0 + fl
            for gi in range(G):
                idx = ((np.uint64(fa * G + gi) * np.uint64(R) + rr) * np.uint64(B)) + bb
                h = _splitmix64(np.uint64(cfg.seed) ^ (idx * np.uint64(0xD1B54A32D192ED03)))
                v = np.zeros((R, B), np.uint32)
                clut = (h >> np.uint64(32)).astype(np.uint32) < geo.clutter_thresh[gi][None, :]
                cval = (np.uint32(11) + ((h >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.uint32)
                        % np.uint32(29))
                v[clut] = cval[clut]
                lmask = land & ((h & np.uint64(0xFF)).astype(np.uint32) < geo.land_fill_u8)
                lval = np.uint32(150) + ((h >> np.uint64(8)) & np.uint64(0xFF)).astype(np.uint32) % np.uint32(106)
                v[lmask] = lval[lmask]
                decided = np.zeros((R, B), bool)
                tfill = ((h >> np.uint64(40)) & np.uint64(0xFF)).astype(np.uint32) < geo.target_fill_u8
                tval = np.uint32(60) + ((h >> np.uint64(48)) & np.uint64(0xFF)).astype(np.uint32) % np.uint32(40)
                for k in range(cfg.n_targets):
                    r0, r1 = geo.target_rows[fl, k]
                    b0, b1 = geo.target_bins[fl, k]
                    if r1 < r0 or b1 < b0:
                        continue
                    sl = (slice(r0, r1 + 1), slice(b0, b1 + 1))
                    tx, ty, r2 = geo.targets[fl, k, :3]
                    dx = xx[sl] - tx
                    dy = yy[sl] - ty
                    d2 = dx * dx + dy * dy
                    inside = (d2 <= r2) & ~decided[sl]
                    sub = v[sl]
                    put = inside & tfill[sl]
                    sub[put] = tval[sl][put]
                    v[sl] = sub
                    decided[sl] |= inside
                out[li, gi] = v.astype(np.uint8)
    return out


# ----------------------------------------------------------------- device generation
class DeviceSynth:
    """Holds the geometry on device and fills u8 echo tensors with rpt_synth_echo."""

    def __init__(self, cfg: SynthConfig, device=None):
        import torch

        from . import _abi
        from ._device import require_gpu

        self.cfg = cfg
        self.dev = require_gpu(device)
        self.geo = make_geometry(cfg)
        g = self.geo
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)  # noqa: E731
        self.cos_t = t(g.cos_t, None)
        self.sin_t = t(g.sin_t, None)
        self.thresh = t(g.clutter_thresh.view(np.int32), None)
        self.targets = t(g.targets, None)
        self.trows = t(g.target_rows, None)
        self.tbins = t(g.target_bins, None)
        p = _abi.SynthParams()
        p.seed = cfg.seed
        p.rows, p.bins, p.n_gains, p.n_targets = cfg.rows, cfg.bins, len(cfg.gains), cfg.n_targets
        p.scale = cfg.scale
        p.target_fill_u8 = g.target_fill_u8
        p.land_fill_u8 = g.land_fill_u8
        p.land_row0, p.land_row1 = g.land_rows
        p.land_bin0 = g.land_bin0
        self.params = p
        self._abi = _abi

    def echo(self, out=None):
        import torch

        from ._device import stream_handle

        cfg = self.cfg
        shape = (cfg.n_frames, len(cfg.gains), cfg.rows, cfg.bins)
        if out is None:
            out = torch.empty(shape, dtype=torch.uint8, device=self.dev)
        # frame0 = 0 relative to this geometry (its targets already start at cfg.frame0); the
        # hash uses absolute frame numbers: pass frame0 so shards reproduce the full stack.
        st = self._abi.load().rpt_synth_echo(self.params, cfg.frame0, cfg.n_frames,
                                             self.cos_t.data_ptr(), self.sin_t.data_ptr(),
                                             self.thresh.data_ptr(), self.targets.data_ptr(),
                                             self.trows.data_ptr(), self.tbins.data_ptr(),
                                             out.data_ptr(), stream_handle(self.dev))
        self._abi.check(st, "rpt_synth_echo")
        return out
