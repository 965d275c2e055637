#!/usr/bin/env python3
"""CPU model of the K5 slow pass on a small synthetic stack (kernel design aid, not a test):
which points the cell pass leaves undecided, and how many dependent point-load rounds a wave
spends on each of them -- per undecided candidate cell 64 points at a time (k_core_slow before
the flattened form) vs the flattened candidate list, U loads per lane per round.
    python tools/k5_sim.py [frames] [U]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "radar-point-cloud-tracking_amd"), str(ROOT)):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

from oracle import path as op  # noqa: E402
from rpt.synth import SynthConfig, make_geometry, numpy_echo  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 12
U = int(sys.argv[2]) if len(sys.argv) > 2 else 4
EPS, EPST, NEED = 8.0, 2.0, 15
cfg = SynthConfig(n_frames=F)
geo = make_geometry(cfg)
t0 = time.time()
echo = numpy_echo(cfg, geo)
per_frame = [{g: op.polar_scatter(echo[f, k], np.full(cfg.rows, cfg.scale, np.float32),
                                  geo.cos_t, geo.sin_t) for k, g in enumerate(cfg.gains)}
             for f in range(F)]
frames = op.build_frames(per_frame)
if len(frames) > 10:
    frames = op.land_filter(frames)[0]
xy, t = op.stack_coords(frames)
print(f"stack {len(xy)} points, {time.time() - t0:.1f} s")
x = xy[:, 0].astype(np.float64)
y = xy[:, 1].astype(np.float64)
tt = t.astype(np.float64)
side = 0.7 * EPS * (1 + 2**-20)
cx = np.floor((x - x.min()) / side).astype(np.int64)
cy = np.floor((y - y.min()) / side).astype(np.int64)
cs = (tt - tt.min()).astype(np.int64)
nx, ny = int(cx.max()) + 1, int(cy.max()) + 1
key = (cs * ny + cy) * nx + cx
order = np.argsort(key, kind="stable")
key_s = key[order]
xs, ys, ts = x[order], y[order], tt[order]
u, first, cnt = np.unique(key_s, return_index=True, return_counts=True)
cell_of = {int(k): i for i, k in enumerate(u)}
b = first
e = first + cnt
bx0 = np.minimum.reduceat(xs, first)
bx1 = np.maximum.reduceat(xs, first)
by0 = np.minimum.reduceat(ys, first)
by1 = np.maximum.reduceat(ys, first)
bt0 = np.minimum.reduceat(ts, first)
bt1 = np.maximum.reduceat(ts, first)
E2 = EPS * EPS


def gap(a0, a1, b0, b1):
    return np.where(b0 > a1, b0 - a1, np.where(a0 > b1, a0 - b1, 0.0))


def span(a0, a1, b0, b1):
    return np.maximum(np.abs(b1 - a0), np.abs(a1 - b0))


def classify(ax0, ax1, ay0, ay1, at0, at1, ci):
    dmin = gap(ax0, ax1, bx0[ci], bx1[ci]) ** 2 + gap(ay0, ay1, by0[ci], by1[ci]) ** 2
    dmax = span(ax0, ax1, bx0[ci], bx1[ci]) ** 2 + span(ay0, ay1, by0[ci], by1[ci]) ** 2
    tg = gap(at0, at1, bt0[ci], bt1[ci])
    tm = span(at0, at1, bt0[ci], bt1[ci])
    c = np.where((dmin <= E2) & (tg <= EPST), np.where((dmax <= E2) & (tm <= EPST), 1, 2), 0)
    return c


def window(k):
    s, r = divmod(int(k), nx * ny)
    yy, xx = divmod(r, nx)
    out = []
    for ds in range(-3, 4):
        for dy in range(-2, 3):
            for dx in range(-2, 3):
                X, Y, S = xx + dx, yy + dy, s + ds
                if 0 <= X < nx and 0 <= Y < ny and S >= 0:
                    c = cell_of.get((S * ny + Y) * nx + X)
                    if c is not None:
                        out.append(c)
    return np.array(out, np.int64)


mutual = (span(bx0, bx1, bx0, bx1) ** 2 + span(by0, by1, by0, by1) ** 2 <= E2)
und = []
n_dec_whole = 0
for i in range(len(u)):
    if mutual[i] and cnt[i] >= NEED:
        n_dec_whole += 1
        continue
    w = window(u[i])
    c = classify(bx0[i], bx1[i], by0[i], by1[i], bt0[i], bt1[i], w)
    lo = cnt[w][c == 1].sum()
    hi = cnt[w][c != 0].sum()
    if lo >= NEED or hi < NEED:
        continue
    und.append(i)
und = np.array(und, np.int64)
q_pts = np.concatenate([np.arange(b[i], e[i]) for i in und]) if len(und) else np.zeros(0, int)
print(f"occupied {len(u)} cells, whole {n_dec_whole}, undecided {len(und)} cells with "
      f"{len(q_pts)} points ({len(q_pts) / len(xs):.3%})")
old_rounds, new_rounds, Ts, cores, lists = [], [], [], [], []
for s in q_pts:
    w = window(key_s[s])
    c = classify(xs[s], xs[s], ys[s], ys[s], ts[s], ts[s], w)
    count = int(cnt[w][c == 1].sum())
    und_c = w[c == 2]
    T = int(cnt[und_c].sum())
    Ts.append(T)
    lists.append(len(und_c))
    # per candidate cell, 64 points per round, stop at NEED
    k = count
    rounds = 0
    for ci in und_c:
        if k >= NEED:
            break
        for j0 in range(b[ci], e[ci], 64):
            if k >= NEED:
                break
            j = np.arange(j0, min(j0 + 64, e[ci]))
            d2 = (xs[j] - xs[s]) ** 2 + (ys[j] - ys[s]) ** 2
            k += int(np.sum((d2 <= E2) & (np.abs(ts[j] - ts[s]) <= EPST)))
            rounds += 1
    old_rounds.append(rounds)
    # flattened: 64*U points per round
    if und_c.size:
        j = np.concatenate([np.arange(b[ci], e[ci]) for ci in und_c])
        d2 = (xs[j] - xs[s]) ** 2 + (ys[j] - ys[s]) ** 2
        adj = (d2 <= E2) & (np.abs(ts[j] - ts[s]) <= EPST)
        csum = count + np.cumsum(adj)
        hit = np.nonzero(csum >= NEED)[0]
        last = hit[0] if (count < NEED and hit.size) else (len(j) - 1 if count < NEED else -1)
        new_rounds.append(0 if last < 0 else last // (64 * U) + 1)
    else:
        new_rounds.append(0)
    cores.append(k >= NEED)
old_rounds, new_rounds, Ts = map(np.array, (old_rounds, new_rounds, Ts))
cores = np.array(cores)
print(f"queued points: core {cores.mean():.3f}; undecided candidate cells mean {np.mean(lists):.1f}; "
      f"T (their points) mean {Ts.mean():.0f} p50 {np.median(Ts):.0f} p90 {np.percentile(Ts, 90):.0f}")
for name, r in (("per-cell 64", old_rounds), (f"flattened 64x{U}", new_rounds)):
    print(f"{name:>16}: rounds mean {r.mean():.2f} p50 {np.median(r):.0f} p90 "
          f"{np.percentile(r, 90):.0f} max {r.max()}  (core {r[cores].mean():.2f}, "
          f"non-core {r[~cores].mean() if (~cores).any() else 0:.2f})")
