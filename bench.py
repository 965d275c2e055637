#!/usr/bin/env python3
"""Benchmark: Mpoints/s clustered+tracked on synthetic 1024-echo frames (BASELINE.json metric).

One step = the reference's per-frame path (4_temporal_object_tracker.py run_pipeline :941-991)
over a frame stack whose u8 echo is already resident in HBM: K1 polar scatter + 3-gain fusion,
land filter (> 10 frames), ST-DBSCAN over the stack, per-frame cluster summaries, reference
cluster order and the Hungarian tracker on the host — ending with final tracker state on the
host.  value = points produced by K1 over the stack ("Total points", :950-951) / step time.

Workload at N=1: configs[2] of BASELINE.json — 100-frame 3-gain fused stack, ST-DBSCAN +
tracking (configs[1], one 50k-point frame, is launch-latency bound and is a parity case).
Multi-GPU: every rank owns `--frames` contiguous frames of one global stack (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (str(ROOT / "radar-point-cloud-tracking_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
K5_BYTES_PER_POINT = 17.0  # SURVEY.md §8(d) compulsory model of the neighbour-search kernel


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(echo_host: np.ndarray, cfg, geo, max_seconds: float = 30.0):
    """Oracle (the pinned CPU restatement, 1 thread) on the first frames of the same workload."""
    import oracle
    from oracle import path as op

    F, G, R, B = echo_host.shape
    t0 = time.perf_counter()
    per_frame = []
    for f in range(F):
        per_frame.append({gain: op.polar_scatter(echo_host[f, k], np.full(R, cfg.scale, np.float32),
                                                 geo.cos_t, geo.sin_t)
                          for k, gain in enumerate(cfg.gains)})
        if time.perf_counter() - t0 > max_seconds:
            break
    frames = op.build_frames(per_frame)
    npts = sum(len(p) for _, p, _ in frames)
    op.run_path(frames)
    dt = time.perf_counter() - t0
    del oracle
    return npts, len(frames), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=100, help="frames per GPU")
    ap.add_argument("--cpu-frames", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-stage hipEvent timing")
    ap.add_argument("--sharded", action="store_true",
                    help="run the frame-sharded (multi-GPU) pipeline even with one rank")
    ap.add_argument("--lanes", type=int, default=1,
                    help="single GPU: stacks in flight at once (native handles on separate "
                         "streams, FrameStackPipeline.submit)")
    ap.add_argument("--sync-host", action="store_true",
                    help="run each step's host stage (order + tracker) inline instead of "
                         "overlapping it with the next step's device work")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --sharded: the frame-sharded multi-GPU path even at one rank (measures its per-rank cost)
    dist = world > 1 or args.sharded
    if dist and "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from rpt import _abi
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    _abi.load()
    F = args.frames
    cfg = SynthConfig(n_frames=F, frame0=rank * F)
    ds = DeviceSynth(cfg, dev)
    echo = ds.echo()
    torch.cuda.synchronize(dev)
    timing = not args.no_timing
    if dist:
        # frame-sharded global stack: rank r owns frames [r*F, (r+1)*F) (rpt/dist.py)
        from rpt.dist import Comm, ShardedStackPipeline
        from rpt.stages import HipOps

        ops = HipOps(dev, timing=timing)
        # rank 0's host stage (order + tracker over N*F frames, ~6.7 us/frame) of consecutive
        # steps runs on 4 worker threads: the steps are independent stacks
        pipe = ShardedStackPipeline(ops, Comm(dev), cfg.gains, cfg.rows, cfg.bins, PathParams(),
                                    timing=timing, async_host=not args.sync_host,
                                    host_workers=4)
        G = len(cfg.gains)
        pipe.set_geometry(
            tuple(torch.from_numpy(np.tile(a, F * G)).to(dev) for a in
                  (np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t)),
            torch.tensor(list(cfg.gains) * F, dtype=torch.int32, device=dev))
        run = lambda: pipe.run(echo, _abi.ECHO_U8, rank * F)  # noqa: E731
    else:
        pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev, timing=timing,
                                  async_host=not args.sync_host, lanes=args.lanes)
        pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                          cfg.n_frames * len(cfg.gains))
        run = lambda: pipe.submit(echo)  # noqa: E731

    def resolve(r):
        return r.result() if hasattr(r, "result") else r

    for _ in range(args.warmup):
        resolve(run()).finish()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    stage_acc = {}
    k5_ms = []
    res = None
    results = []
    for _ in range(args.steps):
        res = run()
        results.append(res)
        if timing and dist:
            k5_ms.append(ops.last_core_ms())
    results = [resolve(r) for r in results]
    if timing and not dist:
        k5_ms = [r.stage_ms["dbscan_core"] for r in results]
    res = results[-1]
    for r in results:  # host stages (order + tracker) of the last runs, in order
        r.finish()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    for r in results:
        for k, v in r.stage_ms.items():
            stage_acc[k] = stage_acc.get(k, 0.0) + v
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t[0])
        pts = float(res.n_points_global)        # K1 points of the whole global stack
        n_core_in = ops.core_points             # [halo | own | halo] points of this rank
        summary = {"points_clustered_rank0": res.n_clustered_local, "clusters": res.n_clusters,
                   "segments": res.n_segments, "objects": len(res.tracker)
                   if res.tracker is not None else None}
    else:
        pts = float(res.n_points)
        n_core_in = res.n_clustered_input
        summary = {"points_clustered_rank0": res.n_clustered_input, "clusters": res.n_clusters,
                   "segments": res.n_segments, "objects": len(res.tracker)}
    value = pts * args.steps / dt / 1e6
    ms_step = dt / args.steps * 1e3

    traffic = None
    tfile = ROOT / "profiles" / "r1" / "k5_traffic.json"
    if tfile.exists() and not dist and args.frames == 100:
        # PMC-measured HBM bytes per K5 launch of this same workload (tools/pmc.sh: separate
        # FETCH_SIZE / WRITE_SIZE passes, gfx950 read correction); committed under profiles/
        traffic = json.loads(tfile.read_text()).get("bytes_per_launch")
    roof = None
    if k5_ms:
        k5 = float(np.mean(k5_ms))
        n_in = n_core_in
        achieved = K5_BYTES_PER_POINT * n_in / (k5 * 1e-3) / 1e9
        roof = {"kernel": "K5 = k_core_cells_oct + k_core_fill + k_core_slow (core flags)",
                "bound": "hbm",
                "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else int(traffic),
                "traffic_unit": "bytes per launch (PMC, profiles/r1/k5_traffic.json)",
                "bytes_model": "17 B/point x points entering ST-DBSCAN (SURVEY.md 8d)",
                "avg_ms": round(k5, 4), "points": n_in}
    stage = {k: round(v / args.steps, 3) for k, v in stage_acc.items()}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and not dist:
        cf = min(args.cpu_frames, args.frames)
        eh = echo[:cf].cpu().numpy()
        npts, nfr, cdt = cpu_baseline(eh, cfg, ds.geo)
        cpu = {"value": round(npts / cdt / 1e6, 5), "unit": "Mpoints/s", "cores": 1,
               "kind": "port",
               "sample": f"first {nfr} frames of the same stack ({npts} points): oracle numpy "
                         f"polar scatter + C BFS ST-DBSCAN + numpy/scipy tracker, 1 thread, "
                         f"{cdt:.1f} s"}
    if rank == 0:
        out = {
            "metric": "Mpoints/s clustered+tracked, 1024-echo synthetic frames; 1/2/4/8-GPU scaling",
            "value": round(value, 3), "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8 echo / f32 geometry / f64 distance",
            "data": "synthetic (device-generated, seeded)",
            "config": {"workload": f"{args.frames}-frame 3-gain fused stack per GPU "
                                   f"(4096 az x 1024 echo u8), land filter + ST-DBSCAN eps 8 / "
                                   f"eps_t 2 / min 15 + Hungarian tracking (BASELINE configs[2])",
                       "frames_per_gpu": args.frames, "points_per_step": int(pts),
                       **summary,
                       "parallelism": f"frame-sharded x{world}" if dist else "single GPU",
                       "stacks_in_flight": 1 if dist else args.lanes,
                       "host_stage": "inline" if args.sync_host else
                       "overlapped: step k's order+tracker runs on a host thread during step "
                       "k+1's device work; the timed region ends after the last one"},
            "roofline": roof, "cpu_baseline": cpu, "stage_ms": stage,
        }
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
