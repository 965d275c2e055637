#!/usr/bin/env python3
"""Multi-rank check of the frame-sharded path on GPU(s): every rank runs rpt.dist's
NativeShardPipeline (or, --impl python, ShardedStackPipeline) on its frame range; rank 0 also runs the single-GPU FrameStackPipeline over
the whole stack and asserts identical labels, per-frame cluster rows and tracked objects.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/dist_check.py --backend gloo --frames 14
(--backend gloo lets several ranks share one GPU; nccl = RCCL needs one GPU per rank.)

--digest std0[,std1]: the ranks run shares of the committed 1000-frame oracle workloads
(tests/golden/bigstack_<name>.json, tests/golden/make_bigstack.py) instead, alternating the named
workloads over the runs, and rank 0 compares every run's gathered result with the oracle digest.
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for _p in (str(ROOT / "radar-point-cloud-tracking_amd"), str(ROOT)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--frames", type=int, default=14, help="frames per rank")
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--lanes", type=int, default=1,
                    help="native: stacks in flight (rpt.dist.ShardLanes); every lane's result "
                         "is checked")
    ap.add_argument("--impl", default="native", choices=("native", "python"),
                    help="native: NativeShardPipeline (librpt shard driver); python: "
                         "ShardedStackPipeline over HipOps")
    ap.add_argument("--digest", default=None,
                    help="comma-separated bigstack workloads (tests/golden/bigstack_<name>.json): "
                         "compare with the oracle digests instead of the single-GPU pipeline")
    ap.add_argument("--dense", action="store_true",
                    help="configs[4] density (rpt.synth.dense_config): one giant component "
                         "crossing every rank boundary")
    ap.add_argument("--oracle", action="store_true",
                    help="rank 0 checks against the oracle's run_path (union-find ST-DBSCAN) "
                         "over the whole stack instead of the single-GPU pipeline")
    ap.add_argument("--tiny-caps", action="store_true",
                    help="native: one-pair / 16-word capacities for the pair and result gathers "
                         "(every step is finished again with grown ones)")
    ap.add_argument("--force-host-merge", action="store_true",
                    help="native: device equivalence-merge limit 0, so every step with a pair "
                         "is merged on the host (rpt_merge_equivalences, the redo slot)")
    ap.add_argument("--sample-check", action="store_true",
                    help="no whole-stack reference: every rank checks its own kept points' core "
                         "flags and labels with oracle.sample_check (every point of its first "
                         "and last floor(eps_t) frames + random frames), rank 0 the global "
                         "cluster numbering and its frames' K9 rows (configs[4] at 8 x 125)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="run world-1 collectives through the backend (rpt.dist.Comm.solo off): "
                         "with --backend nccl this executes the RCCL branch on one GPU")
    args = ap.parse_args()
    if args.force_collectives:
        os.environ["RPT_COMM_FORCE_COLLECTIVES"] = "1"
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")

    from rpt import _abi
    from rpt.dist import Comm, NativeShardPipeline, ShardedStackPipeline
    from rpt.pipeline import PathParams
    from rpt.stages import HipOps
    from rpt.synth import DeviceSynth, SynthConfig

    F = args.frames
    if args.digest:
        sys.exit(run_digest(args, rank, world, dev))
    if args.sample_check:
        sys.exit(run_sample_check(args, rank, world, dev))
    cfg = _config(args, F, rank * F)
    ds = DeviceSynth(cfg, dev)
    echo = ds.echo()
    runs = []  # (result, this rank's labels) per checked run
    if args.impl == "native" and args.lanes > 1:
        from rpt.dist import ShardLanes

        lanes = ShardLanes(dev, args.lanes, cfg.gains, cfg.rows, cfg.bins, PathParams(),
                           keep_labels=True)
        lanes.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t,
                           ds.geo.sin_t, F * 3)
        if args.force_host_merge:
            for p in lanes.pipes:
                p.set_merge_limit(0)
        futs = [lanes.submit(echo, rank * F) for _ in range(2 * args.lanes)]
        outs = [f.result().finish() for f in futs]
        torch.cuda.synchronize(dev)
        for r in outs[-args.lanes:]:  # the last `lanes` steps (whichever lanes ran them)
            runs.append((r, r.labels_local))
        lanes.close()
    elif args.impl == "native":
        pipe = NativeShardPipeline(Comm(dev), cfg.gains, cfg.rows, cfg.bins, PathParams())
        pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                          F * 3)
        if args.tiny_caps:
            pipe._cap_pairs, pipe._cap_out = 1, 16
        if args.force_host_merge:
            pipe.set_merge_limit(0)
        res = pipe.run(echo, rank * F)
        runs.append((res, pipe.labels_local()))
    else:
        ops = HipOps(dev)
        pipe = ShardedStackPipeline(ops, Comm(dev), cfg.gains, cfg.rows, cfg.bins, PathParams())
        geo = tuple(torch.from_numpy(np.tile(a, F * 3)).to(dev) for a in
                    (np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t))
        pipe.set_geometry(geo, torch.tensor(list(cfg.gains) * F, dtype=torch.int32, device=dev))
        res = pipe.run(echo, _abi.ECHO_U8, rank * F)
        runs.append((res, res.labels_local))
    ok = True
    for res, mine in runs:
        ok &= check(res, Comm(dev).all_gather_var(mine.to(torch.int64)), rank, world, args, dev)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    flag = Comm(dev).all_reduce(flag, dist.ReduceOp.MIN)
    dist.destroy_process_group()
    sys.exit(0 if int(flag.item()) == 1 else 1)


def run_digest(args, rank, world, dev):
    """Shares of the committed oracle workloads; every run checked against its digest."""
    import json

    sys.path.insert(0, str(ROOT / "tests"))
    from _digest import compare, shard_digest
    from rpt.dist import Comm, ShardLanes
    from rpt.pipeline import PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    F = args.frames
    names = args.digest.split(",")
    gold = {n: json.loads((ROOT / "tests" / "golden" / f"bigstack_{n}.json").read_text())
            for n in names}
    dss = {n: DeviceSynth(SynthConfig(**{**gold[n]["synth"], "n_frames": F, "frame0": rank * F}),
                          dev) for n in names}
    echoes = {n: dss[n].echo() for n in names}
    torch.cuda.synchronize(dev)
    c0 = dss[names[0]].cfg
    # (fixed lanes: the checks below read each lane's last run from its pipeline)
    lanes = ShardLanes(dev, args.lanes, c0.gains, c0.rows, c0.bins, PathParams(),
                       async_host=True, free_lanes=False)
    lanes.set_geometry(np.full(c0.rows, c0.scale, np.float32), dss[names[0]].geo.cos_t,
                       dss[names[0]].geo.sin_t, F * len(c0.gains))
    # run k goes to lane k % lanes; each lane alternates the workloads over its runs, so every
    # lane's last (checked) run differs from its previous one
    L = args.lanes
    seq = [names[(k % L + k // L) % len(names)] for k in range(2 * L)]
    futs = [lanes.submit(echoes[n], rank * F) for n in seq]
    outs = [f.result().finish() for f in futs]   # every lane idle before the checks' gathers
    torch.cuda.synchronize(dev)
    comm = Comm(dev)
    ok = True
    for i in range(L):
        k = len(seq) - L + i
        n, res, pipe = seq[k], outs[k], lanes.pipes[i]
        mine = pipe.labels_local().cpu().to(torch.int64)
        fo = np.empty(F + 1, np.int64)
        pipe._abi.check(pipe.lib.rpt_shard_frame_offsets(
            pipe.h, 1, fo.ctypes.data_as(pipe._abi.c_i64p)), "rpt_shard_frame_offsets")
        labels = comm.all_gather_var(mine)
        counts = comm.all_gather_fixed(torch.from_numpy(np.diff(fo)))
        if rank == 0:
            lab = torch.cat([l.cpu() for l in labels]).numpy().astype(np.int32)
            got = shard_digest(res, lab, counts.reshape(-1).numpy())
            try:
                compare(got, gold[n], f"run {k} ({n}, lane {i})")
                good = True
            except AssertionError as e:
                print(f"[dist_check] MISMATCH {e}", flush=True)
                good = False
            ok &= good
            print(f"[dist_check] digest run {k} {n} (lane {i}, after {seq[k - L] if k >= L else '-'}):"
                  f" world={world} frames/rank={F} points={res.n_points_global} "
                  f"clusters={res.n_clusters} objects={len(res.tracker.objects())} match={good}",
                  flush=True)
    lanes.close()
    flag = comm.all_reduce(torch.tensor([1 if ok else 0], dtype=torch.int32), dist.ReduceOp.MIN)
    if rank == 0:
        print(f"[dist_check] digest ok={bool(int(flag.item()) == 1)}", flush=True)
    dist.destroy_process_group()
    return 0 if int(flag.item()) == 1 else 1


def run_sample_check(args, rank, world, dev):
    """configs[4] (or any stack) at its real per-rank shape, where no whole-stack reference fits:
    every rank runs NativeShardPipeline on its F frames, then checks its own kept points against
    the exact neighbourhoods of oracle.sample_check (4_temporal_object_tracker.py:466-506):
      * core flag == (neighbour count >= min_samples); a core point's core neighbours all carry
        its label; a non-core point carries the smallest label among its core neighbours (-1
        without one) -- on EVERY point of its first and last floor(eps_t) frames (their
        neighbourhoods cross the rank boundary: the halo, the cross-rank merge and the global
        label numbering are all in these) and on 10,000 random points of each of 5 random inner
        frames; the neighbours' edge frames (points, flags, labels) come from them by P2P;
      * rank 0: the labels in order of their first core point over the whole stack (rank by rank)
        are exactly 0, 1, 2, ... (ids ascend with each cluster's minimum core index, dense), and
        its own frames' K9 rows: segment counts = the (frame, label) histogram, the largest and
        40 random segments' centroids / mean intensities = np.mean (:527-531)."""
    import oracle
    from rpt.dist import Comm, NativeShardPipeline
    from rpt.pipeline import PathParams
    from rpt.synth import DeviceSynth

    F, p = args.frames, PathParams()
    hf = int(np.floor(p.eps_time))
    cfg = _config(args, F, rank * F)
    ds = DeviceSynth(cfg, dev)
    echo = ds.echo()
    comm = Comm(dev)
    pipe = NativeShardPipeline(comm, cfg.gains, cfg.rows, cfg.bins, p)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      F * len(cfg.gains))
    if args.force_host_merge:
        pipe.set_merge_limit(0)
    res = pipe.run(echo, rank * F).finish()
    del echo
    lab = pipe.labels_local().cpu().numpy()
    pts = {k: v.cpu().numpy() for k, v in pipe.points_local().items()}
    torch.cuda.synchronize(dev)
    n = len(lab)
    pf = pts["frame"].astype(np.int64)
    gf = pf + rank * F                       # global frame ids
    fo = np.searchsorted(pf, np.arange(F + 1))
    assert len(pf) == n and (np.diff(pf) >= 0).all()

    def rows(a, b):   # [x bits, y bits, global frame, core, label] of own points a..b
        return np.column_stack([pts["x"][a:b].view(np.int32).astype(np.int64),
                                pts["y"][a:b].view(np.int32).astype(np.int64), gf[a:b],
                                pts["core"][a:b].astype(np.int64),
                                lab[a:b].astype(np.int64)]).reshape(-1)

    cpu = Comm(dev)
    rp, rn = cpu.exchange(torch.from_numpy(rows(0, fo[hf])),
                          torch.from_numpy(rows(fo[F - hf], n)))
    halo_p = rp.cpu().numpy().reshape(-1, 5) if rp is not None else np.zeros((0, 5), np.int64)
    halo_n = rn.cpu().numpy().reshape(-1, 5) if rn is not None else np.zeros((0, 5), np.int64)
    W = np.concatenate([halo_p, rows(0, n).reshape(-1, 5), halo_n])
    wx = W[:, 0].astype(np.int32).view(np.float32)
    wy = W[:, 1].astype(np.int32).view(np.float32)
    wf, wcore, wlab = W[:, 2], W[:, 3].astype(np.uint8), W[:, 4].astype(np.int32)
    off = len(halo_p)                        # window index of own point 0
    wfo = np.searchsorted(wf, np.arange(rank * F - hf, rank * F + F + hf + 1))

    ok = True
    checked = 0

    def check(f_lo, f_hi, idx_own, what):
        """sample_check of own points idx_own over the window frames [f_lo, f_hi) (global)"""
        nonlocal ok, checked
        a = wfo[max(f_lo - (rank * F - hf), 0)]
        b = wfo[min(f_hi - (rank * F - hf), len(wfo) - 1)]
        idx = idx_own + off - a
        assert (idx >= 0).all() and (idx < b - a).all()
        xy = np.column_stack([wx[a:b], wy[a:b]])
        cnt, lo, hi = oracle.sample_check(xy, wf[a:b].astype(np.float32), p.eps_space,
                                          p.eps_time, idx, wcore[a:b], wlab[a:b])
        c, l_ = wcore[a:b][idx], wlab[a:b][idx]
        good = bool(np.array_equal(c, (cnt >= p.min_samples).astype(np.uint8)))
        cm = c == 1
        good &= bool(np.array_equal(lo[cm], l_[cm]) and np.array_equal(hi[cm], l_[cm]))
        good &= bool(np.array_equal(l_[~cm], lo[~cm]))
        if not good:
            print(f"[dist_check] rank {rank} MISMATCH in {what}: core "
                  f"{int((c != (cnt >= p.min_samples)).sum())} wrong, labels "
                  f"{int((lo[cm] != l_[cm]).sum() + (hi[cm] != l_[cm]).sum())} / "
                  f"{int((l_[~cm] != lo[~cm]).sum())} wrong", flush=True)
        ok &= good
        checked += len(idx)

    g0 = rank * F
    check(g0 - hf, g0 + 2 * hf, np.arange(0, fo[hf]), "head frames")
    check(g0 + F - 2 * hf, g0 + F + hf, np.arange(fo[F - hf], n), "tail frames")
    rng = np.random.default_rng(100 + rank)
    for f in rng.choice(np.arange(hf, F - hf), 5, replace=False):
        a, b = fo[f], fo[f + 1]
        s = np.sort(rng.choice(np.arange(a, b), min(10_000, b - a), replace=False))
        check(g0 + f - hf, g0 + f + hf + 1, s, f"frame {g0 + f}")
    edge = int(fo[hf] + n - fo[F - hf])
    print(f"[dist_check] rank {rank}: {n} own points, {edge} edge-frame points + "
          f"{checked - edge} random checked ({len(halo_p)} / {len(halo_n)} halo points) ok={ok}",
          flush=True)

    # global numbering: labels by first core point, rank by rank
    cl = lab[pts["core"] == 1].astype(np.int64)
    u, first = np.unique(cl, return_index=True)
    firsts = u[np.argsort(first)]
    ok &= bool((cl >= 0).all() and (lab >= -1).all())
    allf = comm.all_gather_var(torch.from_numpy(firsts))
    if rank == 0:
        seen, order = set(), []
        for t in allf:
            for v in t.cpu().numpy().tolist():
                if v not in seen:
                    seen.add(v)
                    order.append(v)
        num_ok = order == list(range(res.n_clusters))
        if not num_ok:
            print(f"[dist_check] cluster numbering wrong: {len(order)} ids, "
                  f"{res.n_clusters} clusters, first {order[:10]}", flush=True)
        ok &= num_ok
        # K9 rows of rank 0's frames against its points
        seg = res.seg
        sel = seg["frame"] < F
        m = lab >= 0
        key = pf[m] << 32 | lab[m].astype(np.int64)
        uk, uc = np.unique(key, return_counts=True)
        sk = seg["frame"][sel].astype(np.int64) << 32 | seg["label"][sel].astype(np.int64)
        o = np.argsort(sk)
        k9_ok = bool(np.array_equal(sk[o], uk) and np.array_equal(seg["count"][sel][o], uc))
        xy = np.column_stack([pts["x"], pts["y"]])
        ids = np.nonzero(sel)[0]
        pick = np.unique(np.concatenate([[ids[int(np.argmax(seg["count"][sel]))]],
                                         rng.choice(ids, min(40, len(ids)), replace=False)]))
        for s_ in pick:
            f, lb = int(seg["frame"][s_]), int(seg["label"][s_])
            a, b = fo[f], fo[f + 1]
            w = lab[a:b] == lb
            cxy = np.mean(xy[a:b][w], axis=0)
            k9_ok &= (seg["cx"][s_], seg["cy"][s_]) == (cxy[0], cxy[1])
            k9_ok &= seg["mi"][s_] == np.float32(np.mean(pts["v"][a:b][w]))
        ok &= k9_ok
        print(f"[dist_check] sample-check world={world} frames/rank={F} dense={args.dense} "
              f"points={res.n_points_global} clusters={res.n_clusters} segments={res.n_segments} "
              f"numbering={num_ok} k9_rank0={k9_ok} host_merge={args.force_host_merge}",
              flush=True)
    flag = comm.all_reduce(torch.tensor([1 if ok else 0], dtype=torch.int32), dist.ReduceOp.MIN)
    if rank == 0:
        print(f"[dist_check] ok={bool(int(flag.item()) == 1)}", flush=True)
    dist.destroy_process_group()
    return 0 if int(flag.item()) == 1 else 1


def _config(args, n_frames, frame0=0):
    from rpt.synth import SynthConfig, dense_config

    if args.dense:
        return dense_config(n_frames=n_frames, rows=args.rows, frame0=frame0)
    return SynthConfig(n_frames=n_frames, rows=args.rows, frame0=frame0)


_ORACLE = {}


def check_oracle(res, labels, world, args, dev):
    """Rank 0: the sharded run against the oracle's run_path over the whole stack (land filter,
    union-find ST-DBSCAN, per-frame clusters, tracker): labels, per-frame cluster rows in the
    reference order, tracked objects."""
    import oracle
    from oracle import path as op
    from rpt.synth import DeviceSynth

    sys.path.insert(0, str(ROOT / "tests"))
    from _stack_check import oracle_stack

    key = (args.frames * world, args.dense)
    if key not in _ORACLE:   # once per stack (every lane's last run is checked)
        full = _config(args, args.frames * world)
        dsf = DeviceSynth(full, dev)
        frames = oracle_stack(dsf.echo().cpu().numpy(), full, dsf.geo)
        _ORACLE[key] = op.run_path(frames, dbscan=oracle.stdbscan_uf)
    o_frames, o_labels, o_clusters, o_trk = _ORACLE[key]
    got = torch.cat([l.cpu() for l in labels]).numpy()
    ok = bool(np.array_equal(got, o_labels.astype(np.int64)))
    fo, order, seg = res.frame_order_offsets, res.frame_order, res.seg
    rows = [(f, int(seg["label"][s]), int(seg["count"][s]), seg["cx"][s], seg["cy"][s],
             float(seg["mi"][s])) for f in range(len(fo) - 1) for s in order[fo[f]:fo[f + 1]]]
    exp = [(fid, c[0], c[1], c[2][0], c[2][1], c[3]) for fid, _, _ in o_frames
           for c in o_clusters.get(fid, [])]
    rows_ok = rows == exp
    a, b = list(o_trk.objects.values()), res.tracker.objects()
    trk_ok = [x.object_id for x in a] == [x.object_id for x in b] and all(
        np.array_equal(np.vstack(x.positions), np.vstack(y.positions)) and
        x.frames_seen == y.frames_seen for x, y in zip(a, b))
    ok &= rows_ok and trk_ok
    print(f"[dist_check] oracle world={world} dense={args.dense} points={res.n_points_global} "
          f"clusters={res.n_clusters} (oracle {int(o_labels.max()) + 1}) segments="
          f"{res.n_segments} objects={len(b)} labels_equal={np.array_equal(got, o_labels)} "
          f"rows_equal={rows_ok} tracks_equal={trk_ok} lanes={args.lanes} ok={ok}", flush=True)
    return ok


def check(res, labels, rank, world, args, dev):
    """Rank 0: the sharded run against the single-GPU pipeline over the whole stack."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    F = args.frames
    ok = True
    if rank == 0 and args.oracle:
        ok = check_oracle(res, labels, world, args, dev)
        if args.dense:   # (the dense stacks: the oracle only)
            return ok
    if rank == 0:
        full = _config(args, F * world)
        dsf = DeviceSynth(full, dev)
        single = FrameStackPipeline(full.gains, full.rows, full.bins, PathParams(), dev)
        single.set_geometry(np.full(full.rows, full.scale, np.float32), dsf.geo.cos_t,
                            dsf.geo.sin_t, full.n_frames * 3)
        ref = single.run(dsf.echo(), keep_points=True)
        got = torch.cat([l.cpu() for l in labels]).numpy()
        exp = ref.labels.cpu().numpy().astype(np.int64)
        ok &= bool(np.array_equal(got, exp))
        rows = lambda r: [(f, int(r.seg["label"][s]), int(r.seg["count"][s]), float(r.seg["cx"][s]),  # noqa: E731
                           float(r.seg["cy"][s]), float(r.seg["mi"][s]))
                          for f in range(len(r.frame_order_offsets) - 1)
                          for s in r.frame_order[r.frame_order_offsets[f]:r.frame_order_offsets[f + 1]]]
        ok &= rows(res) == rows(ref)
        a, b = res.tracker.objects(), ref.tracker.objects()
        ok &= [o.object_id for o in a] == [o.object_id for o in b]
        ok &= all(np.array_equal(np.vstack(x.positions), np.vstack(y.positions)) for x, y in zip(a, b))
        print(f"[dist_check] world={world} backend={args.backend} impl={args.impl} points={res.n_points_global} "
              f"clusters={res.n_clusters} segments={res.n_segments} objects={len(a)} "
              f"labels_equal={np.array_equal(got, exp)} lanes={args.lanes} ok={ok}", flush=True)
    return ok


if __name__ == "__main__":
    main()
