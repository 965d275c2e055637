"""TEST-ONLY CPU implementation of the per-device stage interface of rpt/stages.py::HipOps,
built from the pinned oracle, so that the multi-GPU protocol of rpt/dist.py can be exercised
with torch.distributed gloo on CPU (tests/test_dist_cpu.py).  Never used by the product."""
from __future__ import annotations

import numpy as np
import torch

import oracle
from oracle import path as op
from rpt.stages import Points


def _t(a, dt=None):
    a = np.ascontiguousarray(a)
    if dt is not None:
        a = a.astype(dt)
    return torch.from_numpy(a)


class CpuOps:
    def __init__(self, scale: float, cos_t, sin_t):
        self.scale, self.cos_t, self.sin_t = scale, cos_t, sin_t
        self._xy = None

    def polar(self, echo, dt, rows, bins, geo, gain_d, threshold, stride, files_per_frame,
              prefix=""):
        e = echo.numpy() if isinstance(echo, torch.Tensor) else echo
        F, G = e.shape[:2]
        gains = [int(g) for g in gain_d[:G].tolist()]
        xs, ys, vs, gs, pfs, off = [], [], [], [], [], [0]
        for f in range(F):
            n = 0
            for k in range(G):
                x, y, v = op.polar_scatter(e[f, k], np.full(rows, self.scale, np.float32),
                                           self.cos_t, self.sin_t, threshold, stride)
                xs.append(x); ys.append(y); vs.append(v)
                gs.append(np.full(len(x), gains[k], np.int32))
                pfs.append(np.full(len(x), f, np.int32))
                n += len(x)
            off.append(off[-1] + n)
        cat = lambda l, d: _t(np.concatenate(l) if l else np.zeros(0, d), d)  # noqa: E731
        return Points(cat(xs, np.float32), cat(ys, np.float32), cat(vs, np.float32),
                      cat(gs, np.int32), cat(pfs, np.int32), np.array(off, np.int64))

    def bounds(self, pts):
        x, y = pts.x.numpy(), pts.y.numpy()
        return np.array([x.min(), x.max(), y.min(), y.max()], np.float32)

    def land_grid(self, pts, xe, ye):
        x, y, v = pts.x.numpy(), pts.y.numpy(), pts.v.numpy()
        cnt = np.zeros((len(xe) - 1, len(ye) - 1), np.int32)
        tot = np.zeros((len(xe) - 1, len(ye) - 1), np.float64)
        ix = np.clip(np.digitize(x, xe) - 1, 0, len(xe) - 2)
        iy = np.clip(np.digitize(y, ye) - 1, 0, len(ye) - 2)
        np.add.at(cnt, (ix, iy), 1)
        np.add.at(tot, (ix, iy), v)
        return _t(cnt.reshape(-1)), _t(tot.reshape(-1))

    def land_apply(self, pts, cnt, tot, num_frames, xe, ye):
        shape = (len(xe) - 1, len(ye) - 1)
        c = cnt.numpy().reshape(shape)
        s = tot.numpy().reshape(shape)
        with np.errstate(divide="ignore", invalid="ignore"):
            avg = np.where(c > 0, s / c, 0)
        land = (c / max(num_frames, 1) >= 0.8) & (avg >= 100)
        x, y = pts.x.numpy(), pts.y.numpy()
        ix = np.clip(np.digitize(x, xe) - 1, 0, shape[0] - 1)
        iy = np.clip(np.digitize(y, ye) - 1, 0, shape[1] - 1)
        keep = ~land[ix, iy]
        k = torch.from_numpy(keep)
        newoff = np.concatenate([[0], np.cumsum([keep[a:b].sum() for a, b in
                                                 zip(pts.frame_off[:-1], pts.frame_off[1:])])])
        return Points(pts.x[k], pts.y[k], pts.v[k], pts.g[k], pts.pf[k],
                      newoff.astype(np.int64)), int(land.sum())

    def frame_times(self, pts, frame0, name="t"):
        return (pts.pf.to(torch.int64) + frame0).to(torch.float32)

    def dbscan_core(self, x, y, t, eps, eps_t, min_samples):
        xy = np.column_stack([x.numpy(), y.numpy()]).astype(np.float32)
        self._xy, self._t, self._eps, self._et = xy, t.numpy().astype(np.float32), eps, eps_t
        cnt = oracle.neighbour_counts(xy, self._t, eps, eps_t)
        return _t((cnt >= min_samples).astype(np.uint8))

    def _adj(self, i):
        d = self._xy.astype(np.float64) - self._xy[i].astype(np.float64)
        d2 = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]
        dt = np.abs(self._t - self._t[i])
        return np.nonzero((d2 <= self._eps * self._eps) & (dt <= np.float32(self._et)))[0]

    def dbscan_components(self, core):
        c = core.numpy().astype(bool)
        self._core = c
        n = len(c)
        comp = np.full(n, -1, np.int64)
        for i in range(n):
            if not c[i] or comp[i] >= 0:
                continue
            stack = [i]
            comp[i] = i
            while stack:
                u = stack.pop()
                for w in self._adj(u):
                    if c[w] and comp[w] < 0:
                        comp[w] = i
                        stack.append(w)
        return _t(comp, np.int32)

    def remap(self, comp, base, keys, vals):
        c = comp.numpy().astype(np.int64)
        g = np.where(c >= 0, c + base, -1)
        m = dict(zip(keys.tolist(), vals.tolist()))
        return _t(np.array([m.get(v, v) if v >= 0 else -1 for v in g.tolist()], np.int64))

    def select_roots(self, rep, base, lo, hi):
        r = rep.numpy()[lo:hi]
        g = base + np.arange(lo, hi)
        return _t(g[r == g].astype(np.int64))

    def dbscan_labels_global(self, rep, reps_sorted):
        r = rep.numpy()
        reps = reps_sorted.numpy()
        pos = {int(v): k for k, v in enumerate(reps.tolist())}
        out = np.full(len(r), -1, np.int32)
        for i in range(len(r)):
            if r[i] >= 0:
                out[i] = pos[int(r[i])]
            else:
                adj = [int(r[w]) for w in self._adj(i) if r[w] >= 0]
                if adj:
                    out[i] = pos[min(adj)]
        return _t(out)

    def summaries(self, pts, labels, n_clusters):
        lab = labels.numpy()
        x, y, v, pf = pts.x.numpy(), pts.y.numpy(), pts.v.numpy(), pts.pf.numpy()
        F = len(pts.frame_off) - 1
        rows = []
        for l in sorted(set(lab.tolist()) - {-1}):
            idx = np.nonzero(lab == l)[0]
            for f in sorted(set(pf[idx].tolist())):
                m = idx[pf[idx] == f]
                c = np.mean(np.column_stack([x[m], y[m]]), axis=0)
                rows.append((f, l, len(m), m[0], c[0], c[1], np.mean(v[m])))
        seg = {"frame": np.array([r[0] for r in rows], np.int32),
               "label": np.array([r[1] for r in rows], np.int32),
               "count": np.array([r[2] for r in rows], np.int64),
               "first": np.array([r[3] for r in rows], np.int64),
               "cx": np.array([r[4] for r in rows], np.float32),
               "cy": np.array([r[5] for r in rows], np.float32),
               "mi": np.array([r[6] for r in rows], np.float32)}
        fn = np.full(F, -1, np.int64)
        for f in range(F):
            nz = np.nonzero((pf == f) & (lab < 0))[0]
            if len(nz):
                fn[f] = nz[0]
        return seg, fn
