"""Frame-sharded multi-GPU run of the path: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" with host staging for CPU tests / several
ranks sharing one GPU).

Rank r owns the contiguous frame range [r*F, (r+1)*F) of one global stack.  ST-DBSCAN is global
over the stack (the reference clusters all frames at once, 4_temporal_object_tracker.py:466-506)
so the ranks cooperate; the result is identical to a single-device run:

  1. K1 on own frames.                                                     (local)
  2. land filter when the GLOBAL number of built frames exceeds 10: bounds all_reduce MIN/MAX,
     identical float64 edges everywhere, count / intensity grids all_reduce SUM (integer-valued,
     so exact), mask, local compaction.                                   (2 all_reduce rounds)
  3. global point numbering: all_gather of kept counts (frames are in rank order).
  4. halo: h = floor(eps_t) frames to each neighbour (points of the first / last h frames,
     send/recv), so every owned point sees all its space-time neighbours.      (P2P)
  5. core flags on [halo | own | halo]; halo flags replaced by their owners' flags.  (P2P)
  6. local components (min-index union-find); halo points' component ids exchanged with their
     owners, equivalences all_gather'ed, merged on the host (tiny), every component mapped to
     its global minimum core index.                                       (P2P + all_gather)
  7. global representatives: each rank lists the ones it owns, all_gather -> sorted; labels =
     rank of the representative; border points take the smallest adjacent one.  (all_gather)
  8. K9 summaries on own frames, gathered to rank 0, which runs the sequential tracker.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .pipeline import PathParams
from .stages import LAND_GRID_RESOLUTION, Points, order_frames, track_ordered

_MIN, _MAX, _SUM = dist.ReduceOp.MIN, dist.ReduceOp.MAX, dist.ReduceOp.SUM


class Comm:
    """torch.distributed helpers; tensors are staged through host memory for gloo."""

    def __init__(self, dev: torch.device, group=None, force_collectives: bool | None = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.dev = dev
        self.host = dist.get_backend(group) == "gloo"
        self.cdev = torch.device("cpu") if self.host else dev
        if force_collectives is None:
            force_collectives = os.environ.get("RPT_COMM_FORCE_COLLECTIVES", "0") == "1"
        # solo: a one-member group's collectives are the identity (no device round trip).
        # force_collectives (tests): run them through the backend anyway, so that on a one-GPU
        # box the RCCL branch (device tensors, stream order, lanes) executes end to end
        self.solo = self.world == 1 and not force_collectives

    def _c(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.cdev).contiguous()

    def all_reduce(self, t: torch.Tensor, op, inplace: bool = False) -> torch.Tensor:
        """inplace: reduce t itself when it already lives on the backend's device (no copy;
        the caller gives up its values)."""
        if self.solo:
            return t
        c = self._c(t)
        if not (inplace and c.data_ptr() == t.data_ptr()):
            c = c.clone()
        dist.all_reduce(c, op=op, group=self.group)
        return c.to(t.device)

    def all_gather_fixed(self, t: torch.Tensor) -> torch.Tensor:
        """all_gather of a 1-D tensor of the same length on every rank -> [world][len] (host)."""
        if self.solo:
            return t.reshape(1, -1).cpu()
        c = self._c(t).reshape(-1)
        out = torch.empty(self.world * c.numel(), dtype=c.dtype, device=self.cdev)
        dist.all_gather_into_tensor(out, c, group=self.group)
        return out.cpu().reshape(self.world, -1)

    def all_gather_fixed_issue(self, t: torch.Tensor) -> torch.Tensor:
        """all_gather_fixed without the wait: the gathered [world][len] tensor on the backend's
        device (RCCL: in stream order); the caller's .cpu() waits.  Several stacks in flight
        issue the collective inside their sequencer slot and wait outside it."""
        if self.solo:
            return t.reshape(1, -1)
        c = self._c(t).reshape(-1)
        out = torch.empty(self.world * c.numel(), dtype=c.dtype, device=self.cdev)
        dist.all_gather_into_tensor(out, c, group=self.group)
        return out.reshape(self.world, -1)

    def all_gather_dev(self, t: torch.Tensor) -> torch.Tensor:
        """all_gather of a 1-D tensor of the same length on every rank -> [world * len] on the
        input's device (RCCL: stays in stream order, no host wait)."""
        if self.solo:
            return t.reshape(-1)
        c = self._c(t).reshape(-1)
        out = torch.empty(self.world * c.numel(), dtype=c.dtype, device=self.cdev)
        dist.all_gather_into_tensor(out, c, group=self.group)
        return out.to(t.device)

    def all_gather_var(self, t: torch.Tensor) -> List[torch.Tensor]:
        """all_gather of 1-D tensors of different lengths (returned on the input's device)."""
        if self.solo:
            return [t.reshape(-1)]
        c = self._c(t).reshape(-1)
        n = torch.tensor([c.numel()], dtype=torch.int64, device=self.cdev)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(ns, n, group=self.group)
        ns = [int(v.item()) for v in ns]
        m = max(ns) if ns else 0
        pad = torch.zeros(max(m, 1), dtype=c.dtype, device=self.cdev)
        pad[:c.numel()] = c
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(outs, pad, group=self.group)
        return [o[:k].to(t.device) for o, k in zip(outs, ns)]

    def all_gather_capped(self, t: torch.Tensor, cap: int) -> Tuple[List[torch.Tensor], int]:
        """all_gather_var in ONE collective when every rank's length fits cap: each rank sends
        [length | first min(length, cap) elements] padded to 1 + cap (the length as the dtype:
        exact below 2^53), everyone reads the lengths from the same gathered block, and only when
        some length exceeds cap do all ranks (consistently) fall back to the two-round form.
        Returns (pieces on the input's device, longest length)."""
        if self.solo:
            t = t.reshape(-1)
            return [t], int(t.numel())
        c = self._c(t).reshape(-1)
        n = int(c.numel())
        buf = torch.zeros(1 + cap, dtype=c.dtype, device=self.cdev)
        buf[0] = n
        k = min(n, cap)
        if k:
            buf[1:1 + k] = c[:k]
        out = torch.empty(self.world * (1 + cap), dtype=c.dtype, device=self.cdev)
        dist.all_gather_into_tensor(out, buf, group=self.group)
        out = out.reshape(self.world, 1 + cap)
        lens = [int(v) for v in out[:, 0].cpu().tolist()]
        m = max(lens) if lens else 0
        if m > cap:
            return self.all_gather_var(t), m
        return [out[r, 1:1 + lens[r]].to(t.device) for r in range(self.world)], m

    def exchange_known(self, to_prev: torch.Tensor, to_next: torch.Tensor, n_from_prev: int,
                       n_from_next: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """exchange() when every rank already knows what its neighbours send (one P2P round):
        returns (from_prev, from_next) with n_from_prev / n_from_next elements (empty at the
        ends of the rank chain)."""
        r, w = self.rank, self.world
        dev, dt = to_prev.device, to_prev.dtype
        bp = torch.empty(n_from_prev if r > 0 else 0, dtype=dt, device=self.cdev)
        bn = torch.empty(n_from_next if r < w - 1 else 0, dtype=dt, device=self.cdev)
        ops = []
        if r > 0 and to_prev.numel():
            ops.append(dist.P2POp(dist.isend, self._c(to_prev), r - 1, self.group))
        if r < w - 1 and to_next.numel():
            ops.append(dist.P2POp(dist.isend, self._c(to_next), r + 1, self.group))
        if bp.numel():
            ops.append(dist.P2POp(dist.irecv, bp, r - 1, self.group))
        if bn.numel():
            ops.append(dist.P2POp(dist.irecv, bn, r + 1, self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return bp.to(dev), bn.to(dev)

    def exchange(self, to_prev: Optional[torch.Tensor], to_next: Optional[torch.Tensor]
                 ) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
        """Send to_prev to rank-1 and to_next to rank+1; receive what they send back (the
        neighbour's to_next / to_prev).  1-D tensors of one dtype; sizes are exchanged first."""
        r, w = self.rank, self.world
        has_prev, has_next = r > 0, r < w - 1
        ref = to_prev if to_prev is not None else to_next
        if ref is None:
            return None, None
        dt = ref.dtype

        def p2p(sends, recvs):
            ops = []
            for peer, t in sends:
                ops.append(dist.P2POp(dist.isend, t, peer, self.group))
            for peer, t in recvs:
                ops.append(dist.P2POp(dist.irecv, t, peer, self.group))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()

        sz = lambda t: torch.tensor([t.numel() if t is not None else 0],  # noqa: E731
                                    dtype=torch.int64, device=self.cdev)
        rp = torch.zeros(1, dtype=torch.int64, device=self.cdev)
        rn = torch.zeros(1, dtype=torch.int64, device=self.cdev)
        sends, recvs = [], []
        if has_prev:
            sends.append((r - 1, sz(to_prev)))
            recvs.append((r - 1, rp))
        if has_next:
            sends.append((r + 1, sz(to_next)))
            recvs.append((r + 1, rn))
        p2p(sends, recvs)
        bp = torch.empty(int(rp.item()), dtype=dt, device=self.cdev) if has_prev else None
        bn = torch.empty(int(rn.item()), dtype=dt, device=self.cdev) if has_next else None
        sends, recvs = [], []
        if has_prev and to_prev is not None and to_prev.numel():
            sends.append((r - 1, self._c(to_prev)))
        if has_next and to_next is not None and to_next.numel():
            sends.append((r + 1, self._c(to_next)))
        if bp is not None and bp.numel():
            recvs.append((r - 1, bp))
        if bn is not None and bn.numel():
            recvs.append((r + 1, bn))
        p2p(sends, recvs)
        dev = ref.device
        return (bp.to(dev) if bp is not None else None), (bn.to(dev) if bn is not None else None)


class _UF:
    def __init__(self):
        self.p: Dict[int, int] = {}

    def find(self, a: int) -> int:
        p = self.p
        p.setdefault(a, a)
        root = a
        while p[root] != root:
            root = p[root]
        while p[a] != root:
            p[a], a = root, p[a]
        return root

    def union(self, a: int, b: int):
        ra, rb = self.find(a), self.find(b)
        if ra != rb:
            if ra < rb:
                self.p[rb] = ra
            else:
                self.p[ra] = rb


def merge_equivalences(pairs: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """pairs [k][2] of global component ids known to be one component -> (keys, reps) sorted,
    rep = minimum id of each class (= the global minimum core index)."""
    uf = _UF()
    for a, b in pairs.tolist():
        uf.union(int(a), int(b))
    keys = np.array(sorted(uf.p.keys()), dtype=np.int64)
    reps = np.array([uf.find(int(k)) for k in keys], dtype=np.int64)
    return keys, reps


@dataclass
class ShardResult:
    n_points_local: int
    n_points_global: int
    n_clustered_local: int
    n_clusters: int
    labels_local: Optional[torch.Tensor]        # labels of this rank's kept points
    n_segments: int = 0
    tracker: object = None                      # rank 0 only
    frame_order_offsets: Optional[np.ndarray] = None
    frame_order: Optional[np.ndarray] = None
    seg: Optional[Dict[str, np.ndarray]] = None  # rank 0: all segments, global frame slots
    built_global: Optional[np.ndarray] = None
    stage_ms: Dict[str, float] = field(default_factory=dict)
    t_done: float = 0.0                         # perf_counter when the device part ended
    _pending: Optional[Future] = None
    lane: int = -1                              # ShardLanes: the lane that ran the step

    def finish(self) -> "ShardResult":
        """Wait for rank 0's host stage when it runs asynchronously (async_host=True)."""
        if self._pending is not None:
            (self.seg, self.built_global, self.frame_order_offsets, self.frame_order,
             self.tracker, ms) = self._pending.result()
            if self.stage_ms:
                self.stage_ms["tracker"] = ms
            self._pending = None
        return self


class ShardedStackPipeline:
    """The path over a global stack whose frames are split across ranks (see module doc)."""

    def __init__(self, ops, comm: Comm, gains: Sequence[int], rows: int, bins: int,
                 params: PathParams = None, timing: bool = False, async_host: bool = False,
                 host_workers: int = 2):
        """async_host: rank 0's host stage (the reference cluster order of every frame and the
        tracker over the whole stack) runs on a pool of host_workers threads while the ranks go
        on to the next runs (runs are independent, so their host stages may overlap each other
        too); ShardResult.finish() waits and fills seg / frame_order / tracker."""
        self._host = ThreadPoolExecutor(max_workers=host_workers) if async_host else None
        self.ops = ops
        self.comm = comm
        self.gains = [int(g) for g in gains]
        self.rows, self.bins = rows, bins
        self.p = params or PathParams()
        self.timing = timing

    def set_geometry(self, geo, gain_d):
        self.geo, self.gain_d = geo, gain_d

    def run(self, echo, dt: int, frame0: int) -> ShardResult:
        dev = getattr(self.ops, "dev", None)
        if dev is None or torch.device(dev).type != "cuda":  # the oracle-backed CPU test ops
            return self._run(echo, dt, frame0)
        with torch.cuda.device(dev):  # librpt works on the thread's current device
            return self._run(echo, dt, frame0)

    def _run(self, echo, dt: int, frame0: int) -> ShardResult:
        p, ops, comm = self.p, self.ops, self.comm
        G = len(self.gains)
        F = int(echo.shape[0])
        W, r = comm.world, comm.rank
        marks = [("start", time.perf_counter())]

        def mark(name):
            if self.timing:
                marks.append((name, time.perf_counter()))
        # 1. K1; counts and bounds of every rank in one all_gather
        pts = ops.polar(echo, dt, self.rows, self.bins, self.geo, self.gain_d, p.threshold,
                        p.stride, G)
        n_local = pts.n
        built_local = np.nonzero(np.diff(pts.frame_off) > 0)[0]
        b = ops.bounds(pts) if n_local else np.array([np.inf, -np.inf, np.inf, -np.inf],
                                                     np.float32)
        info = comm.all_gather_fixed(torch.tensor(
            [n_local, len(built_local), *b.astype(np.float64)], dtype=torch.float64)).numpy()
        n_global = int(info[:, 0].sum())
        n_built = int(info[:, 1].sum())
        mark("polar")
        # 2. land filter (global grid): one all_reduce of [counts | intensity sums] in float64
        #    (integer-valued, so the sums are exact in any order)
        if p.land_filter and n_built > 10 and n_global > 0:
            x0, x1 = np.float32(info[:, 2].min()), np.float32(info[:, 3].max())
            y0, y1 = np.float32(info[:, 4].min()), np.float32(info[:, 5].max())
            xe = np.arange(x0, x1 + LAND_GRID_RESOLUTION, LAND_GRID_RESOLUTION)
            ye = np.arange(y0, y1 + LAND_GRID_RESOLUTION, LAND_GRID_RESOLUTION)
            cnt, tot = ops.land_grid(pts, xe, ye)
            cells = cnt.numel()
            both = comm.all_reduce(torch.cat([cnt.to(torch.float64), tot.to(torch.float64)]),
                                   _SUM)
            cnt = both[:cells].to(torch.int32)
            tot = both[cells:].contiguous()
            pts, _ = ops.land_apply(pts, cnt, tot, n_built, xe, ye)
        mark("land")
        # 3. global numbering and halo sizes: [kept, points of the first h frames, of the last h]
        h = int(np.floor(p.eps_time)) if np.isfinite(p.eps_time) and p.eps_time >= 0 else 0
        if W > 1 and h > F:
            raise ValueError(f"each rank needs at least floor(eps_time)={h} frames")
        h = min(h, F)
        fo = pts.frame_off
        n_own = pts.n
        a_first, a_last = int(fo[min(h, F)]), int(fo[F - h]) if h else n_own
        kinfo = comm.all_gather_fixed(torch.tensor([n_own, a_first, n_own - a_last],
                                                   dtype=torch.int64)).numpy()
        kept = kinfo[:, 0]
        P = int(kept[:r].sum())
        n_in_global = int(kept.sum())
        if n_in_global == 0:
            raise ValueError("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 "
                             "is required.")
        halo = W > 1 and h > 0
        n_prev = int(kinfo[r - 1, 2]) if halo and r > 0 else 0      # rank r-1's last h frames
        n_next = int(kinfo[r + 1, 1]) if halo and r < W - 1 else 0  # rank r+1's first h frames
        t_own = ops.frame_times(pts, frame0)
        # 4. halo exchange: points of the first / last h frames (sizes known: one P2P round)
        own_xyt = torch.stack([pts.x, pts.y, t_own]) if n_own else \
            torch.zeros((3, 0), dtype=torch.float32, device=pts.x.device)
        if halo:
            hp, hn = comm.exchange_known(own_xyt[:, :a_first].reshape(-1),
                                         own_xyt[:, a_last:].reshape(-1), 3 * n_prev, 3 * n_next)
            allxyt = torch.cat([hp.reshape(3, -1), own_xyt, hn.reshape(3, -1)], dim=1)
        else:
            allxyt = own_xyt
        allxyt = allxyt.contiguous()
        base = P - n_prev
        mark("halo")
        # 5. core flags, halo flags from their owners
        X, Y, T = allxyt[0].contiguous(), allxyt[1].contiguous(), allxyt[2].contiguous()
        core = ops.dbscan_core(X, Y, T, p.eps_space, p.eps_time, p.min_samples)
        if halo:
            c_own = core[n_prev:n_prev + n_own]
            cp, cn = comm.exchange_known(c_own[:a_first].contiguous(),
                                         c_own[a_last:].contiguous(), n_prev, n_next)
            if n_prev:
                core[:n_prev] = cp
            if n_next:
                core[n_prev + n_own:] = cn
        # 6. components + equivalences across ranks
        comp = ops.dbscan_components(core)
        compg = torch.where(comp >= 0, comp.to(torch.int64) + base,
                            torch.full_like(comp, -1, dtype=torch.int64))
        pairs = np.zeros((0, 2), np.int64)
        if halo:
            g_own = compg[n_prev:n_prev + n_own]
            op_, on_ = comm.exchange_known(g_own[:a_first].contiguous(),
                                           g_own[a_last:].contiguous(), n_prev, n_next)
            pr = torch.cat([torch.stack([compg[:n_prev], op_], 1),
                            torch.stack([compg[n_prev + n_own:], on_], 1)]).cpu().numpy()
            pr = pr[(pr[:, 0] >= 0) & (pr[:, 1] >= 0) & (pr[:, 0] != pr[:, 1])]
            pr = np.unique(pr, axis=0) if len(pr) else pairs
            # every rank's pair list padded to the largest possible one (halo sizes are known)
            cap = int(max((kinfo[q - 1, 2] if q > 0 else 0) +
                          (kinfo[q + 1, 1] if q < W - 1 else 0) for q in range(W)))
            buf = np.zeros(1 + 2 * cap, np.int64)
            buf[0] = len(pr)
            buf[1:1 + 2 * len(pr)] = pr.reshape(-1)
            allp = comm.all_gather_fixed(torch.from_numpy(buf)).numpy()
            pairs = np.concatenate([row[1:1 + 2 * int(row[0])] for row in allp]).reshape(-1, 2)
        keys, vals = merge_equivalences(pairs)
        rep = ops.remap(comp, base, keys, vals)
        # 7. global representatives and labels
        roots = ops.select_roots(rep, base, n_prev, n_prev + n_own)
        all_roots = comm.all_gather_var(roots) if not comm.solo else [roots]
        reps_sorted = torch.cat([a.to(rep.device) for a in all_roots])
        labels_all = ops.dbscan_labels_global(rep, reps_sorted)
        labels = labels_all[n_prev:n_prev + n_own]
        n_clusters = int(reps_sorted.numel())
        mark("stdbscan")
        # 8. summaries of the own frames, then ONE gather of everything rank 0's host stage
        #    needs (float64 carries the int32 / int64 fields and the float32 values exactly);
        #    the per-frame cluster order is computed there, off every rank's critical path
        seg, first_noise = ops.summaries(pts, labels, n_clusters)
        S = len(seg["frame"])
        packed = np.concatenate([
            [S, frame0], built_local.astype(np.float64), [-1.0] * (F - len(built_local)),
            first_noise, seg["frame"], seg["label"], seg["count"], seg["first"], seg["cx"],
            seg["cy"], seg["mi"]]).astype(np.float64)
        parts = comm.all_gather_var(torch.from_numpy(packed)) if not comm.solo else \
            [torch.from_numpy(packed)]
        mark("summaries")
        res = ShardResult(n_points_local=n_local, n_points_global=n_global,
                          n_clustered_local=n_own, n_clusters=n_clusters, labels_local=labels)
        if r == 0:
            res.n_segments = int(sum(float(t[0]) for t in parts))

            def host_stage():
                t0 = time.perf_counter()
                all_seg, built, fo_g, order_g = _unpack_parts(parts, F)
                trk = track_ordered(built - frame0, fo_g, order_g, all_seg, p, built)
                return all_seg, built, fo_g, order_g, trk, (time.perf_counter() - t0) * 1e3

            if self._host is not None:
                res._pending = self._host.submit(host_stage)
            else:
                (res.seg, res.built_global, res.frame_order_offsets, res.frame_order,
                 res.tracker, _) = host_stage()
        mark("tracker")
        if self.timing:
            for (a, ta), (b, tb) in zip(marks[:-1], marks[1:]):
                res.stage_ms[b] = (tb - ta) * 1e3
        return res


def _unpack_parts(parts, F: int):
    """Rank 0: the per-rank packed summaries (rank order = frame order) -> global seg arrays
    (frame = global slot), built frame ids, and per frame slot the reference cluster order
    (offsets + indices into the global seg), computed rank part by rank part."""
    segs = {k: [] for k in ("frame", "label", "count", "first", "cx", "cy", "mi")}
    built, fos, orders = [], [np.zeros(1, np.int64)], []
    s_base = 0
    for t in parts:
        a = t.cpu().numpy()
        S, f0 = int(a[0]), int(a[1])
        o = 2
        bl = a[o:o + F]
        o += F
        built.append(bl[bl >= 0].astype(np.int64) + f0)
        first_noise = a[o:o + F].astype(np.int64)
        o += F
        part = {}
        for k, dt in (("frame", np.int32), ("label", np.int32), ("count", np.int64),
                      ("first", np.int64), ("cx", np.float32), ("cy", np.float32),
                      ("mi", np.float32)):
            part[k] = a[o:o + S].astype(dt)
            o += S
        fo, order = order_frames(F, part, first_noise)   # frames of the part: local slots
        fos.append(fo[1:] + s_base)
        orders.append(order[:S] + s_base)
        part["frame"] = part["frame"] + np.int32(f0)
        for k in segs:
            segs[k].append(part[k])
        s_base += S
    seg = {k: np.concatenate(v) for k, v in segs.items()}
    return seg, np.concatenate(built), np.concatenate(fos), np.concatenate(orders)


class CommSequencer:
    """Orders the collectives of several stacks in flight on ONE communicator.

    Each step (a stack run) passes through `phases` collective slots in order.  The slots of
    all steps follow one fixed software-pipeline order: step s starts its phase 0 at slot time
    s * d (d = ceil(phases / lanes): the lanes' stagger) and takes phase p at time s * d + p;
    slots are entered by time, ties by step.  In steady state the lanes are thus a fraction of a
    step apart -- while one lane waits on a collective or a readback another runs device work --
    instead of moving phase by phase together.  The order depends only on the sequence of
    submissions, which is the same on every rank, so every rank issues the same collectives in
    the same order on the same process group (no second communicator whose kernels could be
    ordered differently on different GPUs).  A slot may have to wait for a step that is not
    submitted yet; when the submitter stops submitting to wait for results (close_group()) the
    steps submitted so far form a closed epoch and later submissions start a new one after it.
    A step that fails poisons the sequencer so the other lanes raise instead of waiting."""

    def __init__(self, lanes: int, phases: int, stagger: Optional[int] = None,
                 offsets: Optional[Sequence[int]] = None):
        """stagger / offsets: step s takes phase p at slot time s * stagger + offsets[p]
        (default stagger ceil(phases / lanes), offsets 0, 1, ..., phases - 1).  Any
        non-decreasing offsets give a valid order (the same on every rank); they only move where
        the lanes wait."""
        self.L, self.P = int(lanes), int(phases)
        self.d = max(1, -(-self.P // self.L)) if stagger is None else max(1, int(stagger))
        self.off = list(range(self.P)) if offsets is None else [int(v) for v in offsets]
        if len(self.off) != self.P or self.off[0] < 0 or \
                any(b < a for a, b in zip(self.off, self.off[1:])):
            raise ValueError("offsets: one non-decreasing slot time per phase")
        # a lane runs its steps one after another: step s's last slot must come before step
        # s + lanes' first (that step waits behind s on the same lane thread)
        if self.off[-1] - self.off[0] >= self.L * self.d:
            raise ValueError(f"offsets span {self.off[-1] - self.off[0]} >= lanes x stagger "
                             f"({self.L} x {self.d}): a step would wait on a later step of its "
                             f"own lane")
        self.cv = threading.Condition()
        self.failed: Optional[BaseException] = None
        # the open (last) epoch [first step, base time, closed (0/1)]; a step keeps a reference
        # to its own epoch until its last slot is released, so nothing here grows with the
        # number of steps run (a long-running service submits steps without bound)
        self.epoch: Optional[List[int]] = None
        self.epoch_of: Dict[int, List[int]] = {}  # steps not done -> their epoch
        self.next_phase: Dict[int, int] = {}  # step -> its next phase (steps not done)
        self.n_reg = 0
        self.t_end = 0                         # one past the last slot time of any step
        # slot-wait accounting (seconds a step's thread waited for its turn, per phase)
        self.wait_s = [0.0] * self.P
        self.wait_n = [0] * self.P

    def register(self, step: int):
        """Called by the submitter, in step order, before the step runs."""
        with self.cv:
            e = self.epoch
            if e is None or e[2]:
                e = self.epoch = [step, self.t_end, 0]
            self.epoch_of[step] = e
            self.next_phase[step] = 0
            self.n_reg = step + 1
            self.t_end = max(self.t_end, self._time(step, self.P - 1) + 1)
            # (a later epoch starts after every slot of this one: its first step's phase 0 must
            # not precede them)
            self.cv.notify_all()

    def close_group(self):
        """No more steps join the open epoch (the submitter is about to wait on a result)."""
        with self.cv:
            if self.epoch is not None and not self.epoch[2]:
                self.epoch[2] = 1
                self.cv.notify_all()

    def _time(self, step: int, phase: int) -> int:
        e = self.epoch_of[step]
        return e[1] + (step - e[0]) * self.d + self.off[phase]

    def _blocked(self, step: int, phase: int) -> bool:  # under self.cv
        key = (self._time(step, phase), step)
        for s, q in self.next_phase.items():
            if s != step and (self._time(s, q), s) < key:
                return True
        e = self.epoch
        if e is not None and not e[2]:  # the open epoch's next (unsubmitted) step could come first
            t = e[1] + (self.n_reg - e[0]) * self.d + self.off[0]
            if (t, self.n_reg) < key:
                return True
        return False

    def _acquire(self, step: int, phase: int):
        with self.cv:
            t0 = None
            while self.failed is None and self._blocked(step, phase):
                if t0 is None:
                    t0 = time.perf_counter()
                self.cv.wait()
            if t0 is not None:
                self.wait_s[phase] += time.perf_counter() - t0
            self.wait_n[phase] += 1
            if self.failed is not None:
                raise RuntimeError("collective sequence aborted by another stack") \
                    from self.failed

    def _skip(self, step: int, phase: int):
        """A slot the step does not use: it issues no collective, so it needs no turn (waiting
        for it could wait on a step that is not submitted yet); the step just moves past it."""
        self._release(step, phase)

    def _release(self, step: int, phase: int):
        with self.cv:
            if phase + 1 >= self.P:
                self.next_phase.pop(step, None)
                self.epoch_of.pop(step, None)
            else:
                self.next_phase[step] = phase + 1
            self.cv.notify_all()

    def abort(self, exc: BaseException):
        with self.cv:
            if self.failed is None:
                self.failed = exc
            self.cv.notify_all()

    def step(self, step: int) -> "_StepSlots":
        return _StepSlots(self, step)

    def order(self, steps: int) -> List[Tuple[int, int]]:
        """The (step, phase) slot order of `steps` steps submitted without a wait."""
        return sorted(((s, q) for s in range(steps) for q in range(self.P)),
                      key=lambda a: (a[0] * self.d + self.off[a[1]], a[0]))


class _StepSlots:
    """One step's walk through its slots: slot(k) first moves past the skipped slots < k
    without taking their turns (no collective runs in them), close() past the remaining ones
    (e.g. the rare redo slot) -- so a finished step never waits on later submissions."""

    def __init__(self, seq: CommSequencer, step: int):
        self.seq, self.step, self.next = seq, step, 0

    def _pass(self, upto: int):
        while self.next < upto:
            self.seq._skip(self.step, self.next)
            self.next += 1

    @contextlib.contextmanager
    def slot(self, k: int):
        self._pass(k)
        self.seq._acquire(self.step, k)
        try:
            yield
        finally:
            self.seq._release(self.step, k)
            self.next = k + 1

    def close(self):
        self._pass(self.seq.P)


class _NoSlots:
    @contextlib.contextmanager
    def slot(self, k: int):
        yield

    def close(self):
        pass


class NativeShardPipeline:
    """The frame-sharded path with every per-rank stage in librpt's shard driver (rpt_shard_*,
    csrc/shard.cpp) and the collectives between them here (torch.distributed: RCCL over xGMI, or
    gloo).  Per step (csrc/shard.cpp's header has the phases):

      polar* [all_gather info*] land_grid [all_reduce grid] halo [P2P x/y/t] window*
      [P2P core flags] link [P2P component ids] pairs [all_gather pairs] finish
      [all_gather packed results*]

    -- three host waits (*), the other collectives stay in stream order.  Sizes the host does
    not know when it issues a collective are capacities: the halo buffers take the neighbour's
    K1 count of its edge frames (from the info gather), the pair and result buffers capacities
    grown from earlier steps; a step whose pairs or results did not fit (every rank sees every
    header) is finished again with larger ones, in the same order on every rank.  Rank 0's host
    stage (the global label numbering, the reference cluster order and the tracker) is ONE
    native call that releases the GIL.  Same results as ShardedStackPipeline (module doc), which
    stays as the CPU-testable restatement (tests/test_dist_cpu.py)."""

    N_SLOTS = 8  # collective phases of one step (CommSequencer slots): 7 + the rare redo
    # the lanes' slot order (CommSequencer): step s takes phase p at time 4 s + SLOT_OFFSETS[p].
    # Info, land and halo (0-2) together; flags and component ids (3, 4) after the window
    # readback; the pair gather (5) before the NEXT step's info / land / halo, the result gather
    # (6) after them -- so a step's pair gather does not wait for the next step's K1, and its
    # label / K9 work is queued while the next step's K1 runs.  Measured at one rank with every
    # collective forced through RCCL (profiles/r6/rccl_lanes/sq_*): 1.41 ms per 125-frame step at
    # 4 lanes against 1.46-1.54 in the round-5 order (3 lanes)
    SLOT_STAGGER = 4
    SLOT_OFFSETS = (0, 0, 0, 2, 2, 3, 5, 5)

    def __init__(self, comm: Comm, gains: Sequence[int], rows: int, bins: int,
                 params: PathParams = None, timing: bool = False, async_host: bool = False,
                 host_workers: int = 2):
        from . import _abi
        from .stages import _Ws

        self.comm = comm
        self.dev = comm.dev
        self.gains = [int(g) for g in gains]
        self.rows, self.bins = rows, bins
        self.p = params or PathParams()
        self.timing = timing
        self.lib = _abi.load()
        self._abi = _abi
        self.h = self.lib.rpt_shard_create()
        self.ws = _Ws(self.dev)
        self._host = ThreadPoolExecutor(max_workers=host_workers) if async_host else None
        self.core_points = 0
        self._core_ms = False
        # capacities (grown from what earlier steps needed; a step that exceeds one is finished
        # again with a larger one, consistently on every rank)
        self._cap_pairs, self._cap_out = 1024, 1 << 15
        self._last = None  # (gathered results on the device, rows, words per row) of the last run
        # the info vector's host staging: pinned, so its upload for the RCCL gather is an async
        # copy in stream order instead of a synchronous pageable one (reused: the next step's
        # polar readback synchronises the lane's stream after this upload)
        self._info_pin = torch.empty(8, dtype=torch.float64, pin_memory=True) \
            if self.dev.type == "cuda" and not comm.host else None

    def set_geometry(self, scale, cos_t, sin_t, n_files: int):
        def rep(a):
            a = np.ascontiguousarray(a, dtype=np.float32)
            if a.size == self.rows:
                a = np.tile(a, n_files)
            return torch.from_numpy(a).to(self.dev)
        self.geo = (rep(scale), rep(cos_t), rep(sin_t))
        self.gain_d = torch.tensor(self.gains * (n_files // len(self.gains)), dtype=torch.int32,
                                   device=self.dev)

    def last_core_ms(self) -> Optional[float]:
        """hipEvent duration of the last run's core-flag pass (timing=True), else None."""
        if not self._core_ms:
            return None
        ms = float(self.lib.rpt_shard_core_ms(self.h))
        return ms if ms >= 0 else None

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.rpt_shard_destroy(h)
            self.h = None

    def run(self, echo: torch.Tensor, frame0: int, slots=None) -> ShardResult:
        """slots: a CommSequencer step (several stacks in flight on one communicator) or None."""
        slots = slots if slots is not None else _NoSlots()
        with torch.cuda.device(self.dev):
            try:
                return self._run(echo, frame0, slots)
            finally:
                slots.close()

    def _run(self, echo: torch.Tensor, frame0: int, slots) -> ShardResult:
        from ._device import stream_handle
        from .stages import LAND_MIN_INTENSITY, LAND_PERSISTENCE_THRESHOLD

        A, lib, comm, p, ws = self._abi, self.lib, self.comm, self.p, self.ws
        C_ = A.C
        G = len(self.gains)
        F = int(echo.shape[0])
        W, r = comm.world, comm.rank
        st = stream_handle(self.dev)
        marks = [("start", time.perf_counter())]

        def mark(name):
            if self.timing:
                marks.append((name, time.perf_counter()))

        def chk(status, what):
            A.check(status, what)

        def ptr(t):
            return t.data_ptr() if t is not None and t.numel() else None

        if W > 1 and not (np.isfinite(p.eps_time) and p.eps_time >= 0):
            raise ValueError("the frame-sharded path needs a finite eps_time >= 0")
        if W > 1 and int(np.floor(p.eps_time)) > F:
            raise ValueError(f"each rank needs at least floor(eps_time)="
                             f"{int(np.floor(p.eps_time))} frames")
        dt = {torch.uint8: A.ECHO_U8, torch.float32: A.ECHO_F32}[echo.dtype]
        echo = echo.contiguous()
        sp = A.StackParams(F, G, self.rows, self.bins, dt, float(np.float32(p.threshold)),
                           int(p.stride), 1 if p.land_filter else 0, LAND_GRID_RESOLUTION,
                           LAND_PERSISTENCE_THRESHOLD, float(LAND_MIN_INTENSITY),
                           float(p.eps_space), float(p.eps_time), int(p.min_samples),
                           1 if self.timing else 0)
        info = A.ShardInfo()
        scale_d, cos_d, sin_d = self.geo
        # 1. K1 + bounds + edge-frame counts (one readback), then every rank's
        chk(lib.rpt_shard_polar(self.h, C_.byref(sp), echo.data_ptr(), scale_d.data_ptr(),
                                cos_d.data_ptr(), sin_d.data_ptr(), None,  # no per-point gains
                                C_.byref(info), st), "rpt_shard_polar")
        n_points = int(info.n_points)
        # issued inside the slot, waited for outside it: the other lanes' collectives go on
        vals = [n_points, info.n_built, *[float(b) for b in info.bounds], info.n_head_k1,
                info.n_tail_k1]
        if self._info_pin is not None and not comm.solo:
            self._info_pin.numpy()[:] = vals
            info_t = self._info_pin.to(self.dev, non_blocking=True)
        else:
            info_t = torch.tensor(vals, dtype=torch.float64)
        with slots.slot(0):
            allinfo = comm.all_gather_fixed_issue(info_t)
        allinfo = allinfo.cpu().numpy()
        n_global = int(allinfo[:, 0].sum())
        n_built = int(allinfo[:, 1].sum())
        mark("polar")
        # 2. land grid over the global bounds, all-reduced (integer-valued float64: exact)
        grid, cells = None, 0
        if p.land_filter and n_built > 10 and n_global > 0:
            gb = np.array([allinfo[:, 2].min(), allinfo[:, 3].max(), allinfo[:, 4].min(),
                           allinfo[:, 5].max()], np.float32)
            gbp = gb.ctypes.data_as(A.c_f32p)
            cells = int(lib.rpt_shard_land_cells(gbp, LAND_GRID_RESOLUTION))
            if cells <= 0:
                raise ValueError("degenerate land grid")
            grid = ws.get("grid", 2 * cells, torch.float64)
            chk(lib.rpt_shard_land_grid(self.h, gbp, grid.data_ptr(), cells, st),
                "rpt_shard_land_grid")
            with slots.slot(1):
                grid = comm.all_reduce(grid, _SUM, inplace=True)
        # 3. mask + compaction; the own edge frames for the neighbours (capacities: K1 counts)
        hf = int(info.halo_frames)
        halo = W > 1 and hf > 0
        has_p, has_n = halo and r > 0, halo and r < W - 1
        cap_sp = int(info.n_head_k1) if has_p else 0     # my first hf frames, to rank r - 1
        cap_sn = int(info.n_tail_k1) if has_n else 0     # my last hf frames, to rank r + 1
        cap_rp = int(allinfo[r - 1, 7]) if has_p else 0  # rank r - 1's last hf frames
        cap_rn = int(allinfo[r + 1, 6]) if has_n else 0  # rank r + 1's first hf frames
        hsp = ws.get("hsp", 4 + 3 * cap_sp, torch.int32) if has_p else None
        hsn = ws.get("hsn", 4 + 3 * cap_sn, torch.int32) if has_n else None
        chk(lib.rpt_shard_halo(self.h, ptr(grid), cells, n_built, r, int(frame0), ptr(hsp),
                               ptr(hsn), cap_rp, cap_rn, st), "rpt_shard_halo")
        rp = rn = None
        if halo:
            empty = torch.empty(0, dtype=torch.int32, device=self.dev)
            with slots.slot(2):
                rp, rn = comm.exchange_known(hsp if has_p else empty, hsn if has_n else empty,
                                             4 + 3 * cap_rp if has_p else 0,
                                             4 + 3 * cap_rn if has_n else 0)
        mark("land")
        # 4. window, its grid build and core flags (one readback); own edge flags for the
        #    neighbours
        fsp = ws.get("fsp", max(cap_sp, 1), torch.uint8)
        fsn = ws.get("fsn", max(cap_sn, 1), torch.uint8)
        chk(lib.rpt_shard_window(self.h, ptr(rp), cap_rp, ptr(rn), cap_rn,
                                 fsp.data_ptr() if has_p else None,
                                 fsn.data_ptr() if has_n else None, C_.byref(info), st),
            "rpt_shard_window")
        n_own, n_head, n_tail = int(info.n_kept), int(info.n_head), int(info.n_tail)
        self._n_own = n_own
        n_prev, n_next = int(info.n_prev), int(info.n_next)
        n_tot = n_prev + n_own + n_next
        self._core_ms = self.timing and n_tot > 0
        self.core_points = n_tot
        mark("halo")
        # 5. halo core flags from their owners, components, own edge component ids
        flp = fln = None
        if halo:
            with slots.slot(3):
                flp, fln = comm.exchange_known(fsp[:n_head] if has_p else fsp[:0],
                                               fsn[:n_tail] if has_n else fsn[:0],
                                               n_prev, n_next)
        csp = ws.get("csp", max(n_head, 1), torch.int64)
        csn = ws.get("csn", max(n_tail, 1), torch.int64)
        chk(lib.rpt_shard_link(self.h, ptr(flp), ptr(fln), csp.data_ptr() if has_p else None,
                               csn.data_ptr() if has_n else None, st), "rpt_shard_link")
        owp = own_ = None
        if halo:
            with slots.slot(4):
                owp, own_ = comm.exchange_known(csp[:n_head] if has_p else csp[:0],
                                                csn[:n_tail] if has_n else csn[:0],
                                                n_prev, n_next)
        # 6.-7. pairs, gathered; merge, labels, K9 and the packed results, gathered
        g_host, gathered, cap_out = self._finish(slots, owp, own_, W, r)
        mark("stdbscan")
        if int(g_host[:, 7].sum()) == 0 and n_built > 0:   # BallTree on 0 samples
            raise ValueError("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 "
                             "is required.")
        self._last = (gathered, W, cap_out)
        res = ShardResult(n_points_local=n_points, n_points_global=n_global,
                          n_clustered_local=n_own, n_clusters=-1, labels_local=None)
        if r == 0:
            sizes = np.zeros(4, np.int64)
            gh = np.ascontiguousarray(g_host)
            chk(lib.rpt_shard_gathered_sizes(gh.ctypes.data_as(A.c_i64p), W, cap_out,
                                             sizes.ctypes.data_as(A.c_i64p)),
                "rpt_shard_gathered_sizes")
            res.n_segments, res.n_clusters = int(sizes[0]), int(sizes[3])
            host_stage = self._host_stage(gh, W, cap_out, sizes, p)
            if self._host is not None:
                res._pending = self._host.submit(host_stage)
            else:
                (res.seg, res.built_global, res.frame_order_offsets, res.frame_order,
                 res.tracker, _) = host_stage()
        mark("summaries")
        if self.timing:
            for (a, ta), (b, tb) in zip(marks[:-1], marks[1:]):
                res.stage_ms[b] = (tb - ta) * 1e3
        res.t_done = time.perf_counter()
        return res

    def _finish(self, slots, owp, own_, W: int, r: int):
        """pairs -> [all_gather] -> finish -> [all_gather] -> readback; finished again (slot 7,
        every rank alike) while some rank's pairs or results did not fit their capacity, the
        merge needs the host, or K9 must take the radix path."""
        A, lib, comm, ws = self._abi, self.lib, self.comm, self.ws
        from ._device import stream_handle
        st = stream_handle(self.dev)

        def ptr(t):
            return t.data_ptr() if t is not None and t.numel() else None

        def pairs_step():
            cap = self._cap_pairs
            pb = ws.get("pairs", 1 + 2 * cap, torch.int64)
            A.check(lib.rpt_shard_pairs(self.h, ptr(owp), ptr(own_), pb.data_ptr(), cap, st),
                    "rpt_shard_pairs")
            return pb, cap

        def gather(t):
            return comm.all_gather_dev(t) if not comm.solo else t

        def finish_step(pb, gp, row, keys=None, vals=None, radix=False):
            cap_out = self._cap_out
            out = ws.get("out", cap_out, torch.int64)
            if keys is None:
                A.check(lib.rpt_shard_finish(self.h, gp.data_ptr(), W, row, pb.data_ptr(), None,
                                             None, 0, 1 if radix else 0, out.data_ptr(), cap_out,
                                             st), "rpt_shard_finish")
            else:
                A.check(lib.rpt_shard_finish(self.h, None, W, row, pb.data_ptr(),
                                             keys.ctypes.data_as(A.c_i64p),
                                             vals.ctypes.data_as(A.c_i64p), len(keys),
                                             1 if radix else 0, out.data_ptr(), cap_out, st),
                        "rpt_shard_finish")
            return out, cap_out

        def readback(g, cap_out):
            g2 = g.reshape(W, cap_out)
            if r == 0:
                return g2.cpu().numpy()
            h = np.zeros((W, cap_out), np.int64)   # the other ranks need the headers only
            h[:, :8] = g2[:, :8].cpu().numpy()
            return h

        pb, cap = pairs_step()
        with slots.slot(5):
            gp = gather(pb)
        out, cap_out = finish_step(pb, gp, 1 + 2 * cap)
        with slots.slot(6):
            g = gather(out)
        g_host = readback(g, cap_out)
        hdr = g_host[:, :8]
        bad = int(np.bitwise_or.reduce(hdr[:, 3])) or bool((hdr[:, 1] < 0).any())
        if not bad:
            return g_host, g, cap_out
        with slots.slot(7):   # rare: the same decisions on every rank (every header is seen)
            keys = vals = None
            for _ in range(4):
                hdr = g_host[:, :8]
                flags = int(np.bitwise_or.reduce(hdr[:, 3]))
                radix = bool(hdr[r, 1] < 0)
                if not flags and not (hdr[:, 1] < 0).any():
                    break
                if flags & 1:   # some rank's pairs exceeded the capacity
                    counts = gp.reshape(W, 1 + 2 * cap)[:, 0].cpu().numpy()
                    self._cap_pairs = int(counts.max()) + int(counts.max()) // 4 + 64
                    pb, cap = pairs_step()
                    gp = gather(pb)
                    keys = vals = None
                if flags & 2 or keys is not None:   # too many ids for the device merge
                    rows = gp.reshape(W, 1 + 2 * cap).cpu().numpy()
                    pairs = np.concatenate([row[1:1 + 2 * int(min(row[0], cap))]
                                            for row in rows]).astype(np.int64)
                    nk = int(lib.rpt_merge_equivalences(pairs.ctypes.data_as(A.c_i64p),
                                                        len(pairs) // 2, None, None, 0))
                    keys = np.empty(max(nk, 1), np.int64)
                    vals = np.empty(max(nk, 1), np.int64)
                    lib.rpt_merge_equivalences(pairs.ctypes.data_as(A.c_i64p), len(pairs) // 2,
                                               keys.ctypes.data_as(A.c_i64p),
                                               vals.ctypes.data_as(A.c_i64p), nk)
                    keys, vals = keys[:nk], vals[:nk]
                if flags & 4:   # some rank's results exceeded the capacity
                    need = int(hdr[:, 4].max())
                    self._cap_out = need + need // 4 + 1024
                out, cap_out = finish_step(pb, gp, 1 + 2 * cap, keys, vals, radix)
                g = gather(out)
                g_host = readback(g, cap_out)
            else:
                raise RuntimeError("rpt_shard: the packed results did not settle")
        return g_host, g, cap_out

    def _host_stage(self, gh: np.ndarray, W: int, cap_out: int, sizes: np.ndarray, p):
        """Rank 0: one native call (GIL released) -- global labels, every segment, the built
        frames, the reference cluster order and the tracker."""
        from .native_tracker import NativeTracker
        A, lib = self._abi, self.lib

        def host_stage():
            t0 = time.perf_counter()
            S, B, Ft = int(sizes[0]), int(sizes[1]), int(sizes[2])
            seg = {"frame": np.empty(S, np.int32), "label": np.empty(S, np.int32),
                   "count": np.empty(S, np.int64), "first": np.empty(S, np.int64),
                   "cx": np.empty(S, np.float32), "cy": np.empty(S, np.float32),
                   "mi": np.empty(S, np.float32)}
            built = np.empty(max(B, 1), np.int64)
            fo = np.empty(Ft + 1, np.int64)
            order = np.empty(max(S, 1), np.int64)
            trk = NativeTracker(p.max_association_distance, p.max_missed_frames,
                                p.motion_history_frames, p.stationary_velocity_threshold)
            P = lambda a, t: a.ctypes.data_as(t)  # noqa: E731
            A.check(lib.rpt_shard_host_stage(
                P(gh, A.c_i64p), W, cap_out, trk._h, P(seg["frame"], A.c_i32p),
                P(seg["label"], A.c_i32p), P(seg["count"], A.c_i64p), P(seg["first"], A.c_i64p),
                P(seg["cx"], A.c_f32p), P(seg["cy"], A.c_f32p), P(seg["mi"], A.c_f32p),
                P(built, A.c_i64p), P(fo, A.c_i64p), P(order, A.c_i64p), None, -1),
                "rpt_shard_host_stage")
            return seg, built[:B], fo, order[:S], trk, (time.perf_counter() - t0) * 1e3

        return host_stage

    def set_merge_limit(self, max_ids: int):
        """Ids the device equivalence merge takes (default and maximum 8192); a step whose
        gathered pairs hold more is merged on the host (rpt_merge_equivalences, the redo slot).
        0 sends every step with a pair there: tests use it to reach that path."""
        self._abi.check(self.lib.rpt_shard_set_merge_limit(self.h, int(max_ids)),
                        "rpt_shard_set_merge_limit")

    def points_local(self) -> Dict[str, torch.Tensor]:
        """The own kept points of the last run (device copies, for checks): x, y, v, frame slot
        and the K5 core flag of each."""
        from ._device import stream_handle
        n = int(getattr(self, "_n_own", 0))
        out = {"x": torch.empty(n, dtype=torch.float32, device=self.dev),
               "y": torch.empty(n, dtype=torch.float32, device=self.dev),
               "v": torch.empty(n, dtype=torch.float32, device=self.dev),
               "frame": torch.empty(n, dtype=torch.int32, device=self.dev),
               "core": torch.empty(n, dtype=torch.uint8, device=self.dev)}
        if n:
            self._abi.check(self.lib.rpt_shard_points(
                self.h, *[out[k].data_ptr() for k in ("x", "y", "v", "frame", "core")],
                stream_handle(self.dev)), "rpt_shard_points")
        return out

    def labels_local(self) -> torch.Tensor:
        """Global labels (device int32, a copy) of this rank's kept points of the last run (reads
        every rank's representative table back: for checks, not the hot path)."""
        from ._device import stream_handle
        A = self._abi
        gathered, W, cap = self._last
        gh = np.ascontiguousarray(gathered.reshape(W, cap).cpu().numpy())
        r = self.comm.rank
        nr = int(gh[r, 2])
        m = np.empty(max(nr, 1), np.int32)
        A.check(self.lib.rpt_shard_host_stage(gh.ctypes.data_as(A.c_i64p), W, cap, None, None,
                                              None, None, None, None, None, None, None, None,
                                              None, m.ctypes.data_as(A.c_i32p), r),
                "rpt_shard_host_stage")
        md = torch.from_numpy(m).to(self.dev)
        n = int(gh[r, 7])
        out = torch.empty(n, dtype=torch.int32, device=self.dev)
        if n:
            A.check(self.lib.rpt_shard_labels(self.h, md.data_ptr(), nr, out.data_ptr(),
                                              stream_handle(self.dev)), "rpt_shard_labels")
        return out


class ShardStepFuture(Future):
    """Future of one ShardLanes step: every way of waiting on it through its own methods closes
    the sequencer's open group first, so a partial group (fewer than `lanes` steps) is never
    left waiting for steps that will not be submitted."""

    def __init__(self, seq: "CommSequencer"):
        super().__init__()
        self._seq = seq

    def result(self, timeout=None):
        self._seq.close_group()
        return super().result(timeout)

    def exception(self, timeout=None):
        self._seq.close_group()
        return super().exception(timeout)

    def add_done_callback(self, fn):
        self._seq.close_group()
        super().add_done_callback(fn)


class ShardLanes:
    """Several stacks in flight on the frame-sharded path, through ONE communicator: lane i owns
    a NativeShardPipeline, a HIP stream and one worker thread; all lanes share the default
    process group, and a CommSequencer gives every rank the same global order of the lanes'
    collectives (step by step within a group of `lanes` consecutive steps, phase by phase), so
    no second RCCL communicator exists whose kernels could interleave differently on different
    GPUs.  submit() hands the stacks to the lanes in turn; every rank submits the same sequence.
    Step k+1's device phases then run while step k waits on collectives, readbacks or its host
    stage -- the sharded form of FrameStackPipeline(lanes=...)."""

    def __init__(self, dev: torch.device, lanes: int, gains: Sequence[int], rows: int,
                 bins: int, params: PathParams = None, timing: bool = False,
                 async_host: bool = False, host_workers: int = 2,
                 sequenced: Optional[bool] = None, free_lanes: bool = True,
                 keep_labels: bool = False):
        """sequenced: order the lanes' collective slots (default: with more than one rank; at
        one rank every collective is the identity -- True keeps the ordering anyway, to measure
        what it costs).  free_lanes: a step runs on whichever lane is free when its turn comes
        (steps still start in submission order, and the collective order depends only on the
        step numbers); False: step k on lane k % lanes.  keep_labels: each result also carries
        the global labels of this rank's points (result.labels_local, read on the lane before
        the lane takes its next step; for checks)."""
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self.dev = dev
        comm = Comm(dev)
        self.world = comm.world
        self.sequenced = not comm.solo if sequenced is None else bool(sequenced)
        self.pipes = [NativeShardPipeline(comm, gains, rows, bins, params, timing=timing,
                                          async_host=async_host, host_workers=host_workers)
                      for _ in range(lanes)]
        # (RPT_SEQ_STAGGER / RPT_SEQ_OFFSETS: other orders, for measurements)
        st_env = os.environ.get("RPT_SEQ_STAGGER")
        off_env = os.environ.get("RPT_SEQ_OFFSETS")
        offs = [int(v) for v in off_env.split(",")] if off_env else \
            list(NativeShardPipeline.SLOT_OFFSETS)
        # (one lane runs its steps one after another: a step's slots must all come before the
        # next step's, so the stagger grows to the offsets' span + 1 there)
        span = offs[-1] - offs[0]
        self.seq = CommSequencer(
            lanes, NativeShardPipeline.N_SLOTS,
            stagger=int(st_env) if st_env else
            max(NativeShardPipeline.SLOT_STAGGER, -(-(span + 1) // lanes)),
            offsets=offs)
        self.streams = [torch.cuda.Stream(dev) for _ in range(lanes)] if lanes > 1 else [None]
        self.free_lanes = bool(free_lanes)
        self.keep_labels = bool(keep_labels)
        if self.free_lanes:
            import queue

            # one pool of `lanes` workers takes the steps in submission order; each takes a free
            # lane (pipeline + stream) for its step
            self.pools = [ThreadPoolExecutor(max_workers=lanes)]
            self._free = queue.SimpleQueue()
            for i in range(lanes):
                self._free.put(i)
        else:
            self.pools = [ThreadPoolExecutor(max_workers=1) for _ in range(lanes)]
        self._step = 0

    def set_geometry(self, scale, cos_t, sin_t, n_files: int):
        for p in self.pipes:
            p.set_geometry(scale, cos_t, sin_t, n_files)

    def submit(self, echo: torch.Tensor, frame0: int) -> "ShardStepFuture":
        """Runs the next step on lane step % lanes; a future of its ShardResult (call finish()).
        Waiting on it through result() / exception() / add_done_callback() first closes the
        open group (the same on every rank); a caller waiting by other means
        (concurrent.futures.wait, as_completed) calls flush() first."""
        step = self._step
        self._step += 1
        # one rank: every collective is the identity, nothing to order (and nothing registered:
        # an unsequenced step never releases its sequencer entries)
        if self.sequenced:
            self.seq.register(step)
        slots = self.seq.step(step) if self.sequenced else _NoSlots()
        fut = ShardStepFuture(self.seq)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.dev))  # the echo's producer

        def work(li):
            pipe, s = self.pipes[li], self.streams[li]
            with torch.cuda.device(self.dev):
                if s is None:
                    r = pipe.run(echo, frame0, slots)
                    lab = pipe.labels_local() if self.keep_labels else None
                else:
                    s.wait_event(ready)  # the echo is ready
                    with torch.cuda.stream(s):
                        r = pipe.run(echo, frame0, slots)
                        lab = pipe.labels_local() if self.keep_labels else None
            r.lane = li
            if lab is not None:
                r.labels_local = lab
            return r

        def task(li=None):
            if not fut.set_running_or_notify_cancel():
                return
            lane = self._free.get() if li is None else li
            try:
                r = work(lane)
            except BaseException as e:
                self.seq.abort(e)
                fut.set_exception(e)
                return
            finally:
                if li is None:
                    self._free.put(lane)
            fut.set_result(r)

        if self.free_lanes:
            self.pools[0].submit(task)
        else:
            self.pools[step % len(self.pipes)].submit(task, step % len(self.pipes))
        return fut

    def flush(self):
        """Close the open group: its steps take their collective turns without waiting for more
        submissions (call before waiting on steps by any means other than the futures' own
        result() / exception() / add_done_callback(); every rank at the same point)."""
        self.seq.close_group()

    def close(self):
        self.seq.close_group()
        for p in self.pools:
            p.shutdown(wait=True)
