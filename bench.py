#!/usr/bin/env python3
"""Benchmark: Mpoints/s clustered+tracked on synthetic 1024-echo frames (BASELINE.json metric).

One step = the reference's per-frame path (4_temporal_object_tracker.py run_pipeline :941-991)
over a frame stack whose u8 echo is already resident in HBM: K1 polar scatter + 3-gain fusion,
land filter (> 10 frames), ST-DBSCAN over the stack, per-frame cluster summaries, reference
cluster order and the Hungarian tracker on the host — ending with final tracker state on the
host.  value = points produced by K1 over the stack ("Total points", :950-951) / step time.

Default workload: the north-star stack of BASELINE.json configs[3] — ONE 1000-frame 3-gain
fused stack (12.6 GB of u8 echo, ~50 M points), land filter + ST-DBSCAN + tracking — strong
scaling: at N GPUs every rank owns 1000/N contiguous frames of that same stack (rpt/dist.py), so
the driver's N=1,2,4,8 values measure the "6x at 8 GPUs on a 1000-frame stack" target directly.
At N=1 the whole stack runs on one MI355X (it fits: 288 GB HBM).
Two differently seeded stacks of that shape (seed 0 / targets 123 and seed 1 / targets 124 --
tests/golden/bigstack_std{0,1}.json hold the oracle's digests of both) alternate over the steps,
so no step replays the previous step's input on its lane (the K1 capacity and K9 label-bit /
segment-count guesses from the previous run are exercised inside the timed region).
  --frames F     weak scaling instead: F frames per GPU (F=100 is configs[2], round 1's line)
  --dense        configs[4]'s density (~500k points per frame, rpt.synth.dense_config)
  --h2d-steps K  also time K steps that first copy the echo from pinned host memory (reported
                 as `h2d_inclusive`, never as `value`)
100 timed steps by default: with stacks in flight the timed region holds the pipeline's fill and
drain (about one stack time per lane in flight), so short runs report less (1000 frames, same box:
6.12 Gpoints/s at 20 steps, 6.47 at 40, 6.9 at 100); `steady_state` gives the rate without them.
At N=1 five stacks are in flight by default (`--lanes 5`: native handles on five streams;
step k+1's device work runs while step k's host stage and readbacks finish, and the stacks'
latency-bound kernels share the CUs; interleaved same-box runs with every lane set up, 40 steps:
2 lanes 8.4 ms per step, 3 lanes 7.9-8.3, 4 lanes 8.1, 5 lanes 7.95, 6 lanes 7.9-8.2; 100 steps:
3 lanes 7.34-7.67, 5 lanes 7.35-7.43, steady state 7.06-7.38 against 6.77-6.92).  Every lane runs
one untimed stack before the warm-up steps (its buffers are allocated on first use: a lane left
cold cost ~80 ms inside the timed region); `one_stack_in_flight` repeats the steps strictly one after
another, and K5's roofline is taken from that leg (K5 alone on the GPU).
At N>1 (the frame-sharded path) four stacks are in flight per rank by default, their
collectives through ONE communicator in a fixed software-pipeline order (rpt.dist.CommSequencer
with NativeShardPipeline.SLOT_OFFSETS: every rank issues the same collectives in the same order;
validated with gloo at 8 ranks and on RCCL at one rank with every collective forced through it
-- RPT_COMM_FORCE_COLLECTIVES=1: 1.41 ms per 125-frame step at 4 lanes, 2.01 with 1,
profiles/r6/rccl_lanes/); `--lanes 1` runs one stack at a time.  With one rank (`--sharded`,
the 125-frame per-rank share of 8 GPUs) the default is 4 as well (identity collectives).  The
process group has a finite timeout (RPT_PG_TIMEOUT_S, default 240 s) and a hang guard
(RPT_HANG_S, default 180 s without a step submitted or finished) dumps every thread's Python
stack -- the lane threads name the collective slot they wait in -- and exits non-zero, so a
cross-GPU ordering fault ends the run instead of hanging it.
After the timed region (N=1, timing on), K5 is also timed on the per-GPU shares at 8 GPUs, where
SURVEY.md §8(d) sets the 0.40 roofline target: `roofline_c4_share` (125 standard frames, the
configs[3] stack's share) and `roofline_configs4_share` (125 dense frames, configs[4]'s), one
stack in flight (`--no-dense-k5` skips both).
`cpu_baseline`: oracle/refpath.py -- the reference's own algorithmic structure (whole-stack
sklearn BallTree, per-neighbour time filter, seed-set expansion; calibrated against the
reference in the build container by tools/time_reference.py --calibrate-refpath,
profiles/r4/refpath_calibration.json) -- on the first frame
of the same stack, one thread, on this node's host.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--total-frames T | --frames F] [--dense]
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

# Eight hardware queues per process before HIP initialises (HIP's default is four): the five
# stacks in flight (three lanes per rank sharded) each get a queue of their own instead of two
# lanes sharing one -- same box, interleaved: 6.91 / 6.87 against 6.51 / 6.80 Gpoints/s, steady
# state 6.27 / 6.50 against 6.94 / 6.77 ms (profiles/r5/bench_hwq/).  An explicit setting wins.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
K5_BYTES_PER_POINT = 17.0  # SURVEY.md §8(d) compulsory model of the neighbour-search kernel


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(echo_host: np.ndarray, cfg, geo, structure: bool = True):
    """The per-frame path on the host, 1 thread, on the first frames of the same workload:
    polar scatter + fusion (numpy), st_dbscan and the tracker.  structure=True: st_dbscan with
    the reference's algorithmic structure (oracle/refpath.py); False: the oracle's grid-indexed C
    BFS.  Returns (points, frames, seconds, labels-equal-to-the-oracle, index name)."""
    import oracle
    from oracle import path as op
    from oracle.refpath import stdbscan_structure
    from oracle.tracker import Tracker

    F, G, R, B = echo_host.shape
    t0 = time.perf_counter()
    per_frame = [{gain: op.polar_scatter(echo_host[f, k], np.full(R, cfg.scale, np.float32),
                                         geo.cos_t, geo.sin_t)
                  for k, gain in enumerate(cfg.gains)} for f in range(F)]
    frames = op.build_frames(per_frame)
    npts = sum(len(p) for _, p, _ in frames)
    if len(frames) > 10:
        frames = op.land_filter(frames)[0]
    xy, t = op.stack_coords(frames)
    index = "oracle grid BFS (C)"
    if structure:
        labels, index = stdbscan_structure(xy, t, 8.0, 2.0, 15)
    else:
        labels = oracle.stdbscan(xy, t, 8.0, 2.0, 15)
    clusters = op.frame_clusters(frames, labels)
    trk = Tracker()
    for fid, _, _ in frames:
        trk.update([(c[2], fid) for c in clusters.get(fid, [])], fid)
    dt = time.perf_counter() - t0
    same = bool(np.array_equal(labels, oracle.stdbscan(xy, t, 8.0, 2.0, 15))) if structure \
        else True
    return npts, len(frames), dt, same, index


def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _reference_measured():
    """The reference's own sklearn/scipy path, timed in the build container by
    tools/time_reference.py (the reference cannot travel to this box): committed numbers."""
    f = ROOT / "profiles" / "r2" / "reference_cpu.json"
    if not f.exists():
        return None
    d = json.loads(f.read_text())
    legs = {k: {kk: v[kk] for kk in ("points", "frames", "total_s", "mpoints_per_s") if kk in v}
            for k, v in d.get("legs", {}).items() if isinstance(v, dict)}
    return {"source": "profiles/r2/reference_cpu.json (tools/time_reference.py)",
            "cpu_model": d.get("cpu_model"), "threads": d.get("threads_used"), "legs": legs,
            "note": "the reference builds one BallTree over all frames: rates fall ~1/k with k "
                    "frames and do not extrapolate to 100-1000 frames"}


def _traffic(name):
    """PMC-measured HBM bytes per launch committed for a workload (tools/pmc.sh: separate
    FETCH_SIZE / WRITE_SIZE passes, gfx950 read correction), newest round first."""
    for rd in ("r6", "r5", "r4", "r3", "r2"):
        f = ROOT / "profiles" / rd / name
        if f.exists():
            d = json.loads(f.read_text())
            return int(d["bytes_per_launch"]), str(f.relative_to(ROOT))
    return None, None


def _pmc_stack_bytes(wkey):
    """PMC-measured HBM bytes of ALL kernels of one stack (committed tools/pmc.sh summary,
    one stack in flight; the synthetic echo generator excluded): per kernel bytes per launch x
    launches, over the runs of the profiled command (launches of the K1 count pass)."""
    import csv

    for rd in ("r6", "r5", "r4"):
        f = ROOT / "profiles" / rd / f"pmc_traffic_by_kernel_{wkey}.csv"
        if not f.exists():
            continue
        rows = list(csv.DictReader(f.open()))
        runs = sum(int(r["launches"]) for r in rows if "k_group_count_u8" in r["kernel"])
        if runs <= 0:
            continue
        tot = sum(float(r["hbm_bytes_per_launch_corrected"]) * int(r["launches"])
                  for r in rows if "k_synth" not in r["kernel"])
        return tot / runs, str(f.relative_to(ROOT))
    return None, None


def _e2e_roof(echo_bytes_step: float, ms_step: float, world: int, wkey: str):
    """End-to-end rate of the bench line against the HBM roofline of the GPUs used
    (Mpoints/s also as a fraction of the HBM roofline): the u8 echo every step must
    read, and (N = 1) the PMC-measured bytes all kernels of one stack move, each / ms_per_step."""
    peak = HBM_PEAK_GBS * world
    t = ms_step * 1e-3
    out = {"bound": "hbm", "peak": peak, "unit": "GB/s", "ms_per_step": round(ms_step, 4),
           "echo_bytes_per_step": int(echo_bytes_step),
           "achieved_echo": round(echo_bytes_step / t / 1e9, 2),
           "frac_echo": round(echo_bytes_step / t / 1e9 / peak, 4),
           "note": "frac_echo: the compulsory echo read of every step (u8, 1 B per sample of all "
                   "ranks) over the driver's step time; frac_pmc: every kernel's PMC-measured HBM "
                   "bytes of one stack (tools/pmc.sh, FETCH x2 + WRITE) over the same time"}
    b, src = (None, None) if world > 1 else _pmc_stack_bytes(wkey)
    if b is not None:
        out.update(pmc_bytes_per_stack=int(b), pmc_source=src,
                   achieved_pmc=round(b / t / 1e9, 2), frac_pmc=round(b / t / 1e9 / peak, 4))
    return out


def best_cpu(echo_host: np.ndarray, cfg, geo):
    """The oracle's fastest host path on every core this process may use (labelled, not the
    reference): numpy polar scatter + fusion, land filter, the OpenMP union-find ST-DBSCAN
    (oracle/stdbscan_oracle.c) and the tracker, over the first frames of the same stack.
    Returns (points, frames, seconds)."""
    import oracle
    from oracle import path as op

    t0 = time.perf_counter()
    frames = _oracle_frames(echo_host, cfg, geo)
    npts = sum(len(p) for _, p, _ in frames)
    op.run_path(frames, dbscan=oracle.stdbscan_uf)
    return npts, len(frames), time.perf_counter() - t0


def _oracle_frames(echo_host, cfg, geo):
    from oracle import path as op

    F, G, R, B = echo_host.shape
    per_frame = [{gain: op.polar_scatter(echo_host[f, k], np.full(R, cfg.scale, np.float32),
                                         geo.cos_t, geo.sin_t)
                  for k, gain in enumerate(cfg.gains)} for f in range(F)]
    return op.build_frames(per_frame)


def _k5_roof(n_points: float, k5_ms: float, traffic, tsrc):
    """K5's roofline fields.  The algorithmic bytes are SURVEY 8(d)'s 17 B/pt compulsory model;
    where the PMC-measured HBM bytes of the same workload are BELOW the model (K5 decides whole
    cells without reading their points, so the model's per-point reads are not all compulsory
    there), achieved and frac are taken from the measured bytes instead and the model rate is
    kept as a labelled second field -- a bandwidth figure never exceeds what the kernel moved."""
    model = K5_BYTES_PER_POINT * n_points
    t = k5_ms * 1e-3
    model_gbs = model / t / 1e9
    out = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "avg_ms": round(k5_ms, 4),
           "points": int(n_points), "traffic": traffic,
           "traffic_unit": f"bytes per launch (PMC, {tsrc})" if tsrc else None,
           "bytes_model": "17 B/point x points entering ST-DBSCAN (SURVEY.md 8d)",
           "achieved_model": round(model_gbs, 2),
           "frac_model": round(model_gbs / HBM_PEAK_GBS, 4)}
    if traffic is not None and traffic < model:
        ach = traffic / t / 1e9
        out.update(achieved=round(ach, 2), frac=round(ach / HBM_PEAK_GBS, 4),
                   basis="pmc_traffic",
                   note=(f"the PMC-measured HBM bytes ({traffic / 1e6:.0f} MB per launch) are "
                         f"below the 17 B/pt model ({model / 1e6:.0f} MB): cells decided whole "
                         f"are never read point by point, so achieved / frac use the measured "
                         f"bytes; achieved_model / frac_model are the model's figures, not "
                         f"bandwidth"))
    else:
        out.update(achieved=round(model_gbs, 2), frac=round(model_gbs / HBM_PEAK_GBS, 4),
                   basis="model",
                   note=None if traffic is None else
                   (f"PMC-measured HBM bytes {traffic / 1e6:.0f} MB per launch = "
                    f"{traffic / model:.2f}x the 17 B/pt model ({model / 1e6:.0f} MB): re-reads "
                    f"the model does not count"))
    return out


def _k5_share(dev, cfg, label, wkey):
    """K5 (hipEvents around the core-flag pass) on one per-GPU share, one stack in flight: one
    warm-up run, then three timed runs."""
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth

    ds = DeviceSynth(cfg, dev)
    echo = ds.echo()
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev, timing=True)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      cfg.n_frames * len(cfg.gains))
    res = [pipe.run(echo).finish() for _ in range(4)][1:]
    k5 = float(np.mean([r.stage_ms["dbscan_core"] for r in res]))
    n = res[-1].n_clustered_input
    tr, src = _traffic(f"k5_traffic_{wkey}.json")
    out = {"workload": label, **_k5_roof(n, k5, tr, src), "runs": len(res),
           "stage_ms": {k: round(float(np.mean([r.stage_ms[k] for r in res])), 3)
                        for k in res[0].stage_ms}}
    del pipe, echo, ds
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--total-frames", type=int, default=1000,
                    help="frames of the one global stack, split over the ranks (strong scaling)")
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per GPU instead (weak scaling)")
    ap.add_argument("--dense", action="store_true", help="configs[4] density (~500k pts/frame)")
    ap.add_argument("--single-seed", action="store_true",
                    help="replay ONE stack every step (round-2 behaviour) instead of alternating "
                         "two differently seeded stacks")
    ap.add_argument("--h2d-steps", type=int, default=2,
                    help="extra steps timed with the echo's H2D copy from pinned host memory "
                         "(0 = skip)")
    ap.add_argument("--cpu-frames", type=int, default=1,
                    help="frames of the stack the CPU baseline runs (reference structure)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--best-cpu-frames", type=int, default=12,
                    help="frames of the all-cores OpenMP oracle line (cpu_baseline.best_cpu; "
                         "0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-stage hipEvent timing")
    ap.add_argument("--no-dense-k5", action="store_true",
                    help="skip the K5 roofline legs at the 8-GPU per-GPU shares")
    ap.add_argument("--sharded", action="store_true",
                    help="run the frame-sharded (multi-GPU) pipeline even with one rank")
    ap.add_argument("--python-shard", action="store_true",
                    help="sharded runs: ShardedStackPipeline (HipOps stages composed in Python) "
                         "instead of the native shard driver")
    ap.add_argument("--lanes", type=int, default=None,
                    help="stacks in flight at once (default 5 at one rank: native handles on "
                         "separate streams; 4 with --sharded and at N>1 ranks, where a lane is a "
                         "NativeShardPipeline with its own stream and thread, all lanes on ONE "
                         "process group in rpt.dist.CommSequencer's order); 1 = strictly one "
                         "after another")
    ap.add_argument("--sequenced", action="store_true",
                    help="sharded runs at one rank: keep the CommSequencer's slot order although "
                         "every collective is the identity (what the ordering costs)")
    ap.add_argument("--host-workers", type=int, default=8,
                    help="threads for the host stages (cluster order + tracker; rank 0's on the "
                         "sharded path) of consecutive steps")
    ap.add_argument("--no-one-stack", action="store_true",
                    help="skip the one-stack-in-flight leg (and so K5's roofline)")
    ap.add_argument("--k1-gate", action="store_true",
                    help="the lanes' K1 passes take turns (rpt_k1_gate; default: they overlap "
                         "freely: over 20 steps the turns cost more than they save, "
                         "profiles/r6/ab_k1_gate/)")
    ap.add_argument("--sync-host", action="store_true",
                    help="run each step's host stage (order + tracker) inline instead of "
                         "overlapping it with the next step's device work")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.lanes is None:
        # N > 1: four stacks in flight per rank, their collectives through ONE communicator in
        # CommSequencer's order -- every rank issues the same collectives in the same order, at
        # most one thread inside a collective at a time (validated on gloo up to 8 ranks and on
        # RCCL at one rank with every collective forced through it); --lanes 1 = one at a time
        args.lanes = (4 if args.sharded else 5) if world == 1 else 4
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --sharded: the frame-sharded multi-GPU path even at one rank (measures its per-rank cost)
    dist = world > 1 or args.sharded
    if dist and "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
    if dist:
        import torch.distributed as tdist

        from datetime import timedelta

        # RCCL errors and timeouts tear the process down (non-zero exit) instead of hanging
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        torch.cuda.set_device(local)
        tdist.init_process_group(
            "nccl", device_id=torch.device("cuda", local),
            timeout=timedelta(seconds=float(os.environ.get("RPT_PG_TIMEOUT_S", "240"))))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from dataclasses import replace as dc_replace

    from rpt import _abi
    from rpt.pipeline import FrameStackPipeline, PathParams
    from rpt.synth import DeviceSynth, SynthConfig

    _abi.load()
    if args.frames is not None:
        F, scaling, total = args.frames, "weak", args.frames * world
    else:
        if args.total_frames % world:
            raise SystemExit(f"--total-frames {args.total_frames} must divide over {world} ranks")
        F, scaling, total = args.total_frames // world, "strong", args.total_frames
    if args.dense:
        from rpt.synth import dense_config
        cfg = dense_config(n_frames=F, frame0=rank * F)
    else:
        cfg = SynthConfig(n_frames=F, frame0=rank * F)
    # the stacks the steps alternate over (same geometry, other data and target seeds)
    cfgs = [cfg] if args.single_seed else [cfg, dc_replace(cfg, seed=1, target_seed=124)]
    dss = [DeviceSynth(c, dev) for c in cfgs]
    echoes = [d.echo() for d in dss]
    ds, E = dss[0], len(echoes)
    torch.cuda.synchronize(dev)
    timing = not args.no_timing
    if dist:
        # frame-sharded global stack: rank r owns frames [r*F, (r+1)*F) (rpt/dist.py); every
        # per-rank stage in librpt's shard driver (--python-shard: the HipOps-composed variant)
        from rpt.dist import Comm, NativeShardPipeline, ShardedStackPipeline

        # rank 0's host stage (order + tracker over N*F frames, ~6 us/frame) of consecutive
        # steps runs on --host-workers threads (default 8): the steps are independent stacks
        if args.python_shard:
            from rpt.stages import HipOps

            ops = HipOps(dev, timing=timing)
            pipe = ShardedStackPipeline(ops, Comm(dev), cfg.gains, cfg.rows, cfg.bins,
                                        PathParams(), timing=timing,
                                        async_host=not args.sync_host, host_workers=4)
            G = len(cfg.gains)
            pipe.set_geometry(
                tuple(torch.from_numpy(np.tile(a, F * G)).to(dev) for a in
                      (np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t)),
                torch.tensor(list(cfg.gains) * F, dtype=torch.int32, device=dev))
            run = lambda e: pipe.run(e, _abi.ECHO_U8, rank * F)  # noqa: E731
        elif args.lanes > 1:
            # several stacks in flight (rpt.dist.ShardLanes: per lane a process group, stream and
            # thread); K5 and the stage times come from the one-stack-in-flight leg below
            from rpt.dist import ShardLanes

            lanes_ = ShardLanes(dev, args.lanes, cfg.gains, cfg.rows, cfg.bins, PathParams(),
                                timing=timing, async_host=not args.sync_host,
                                host_workers=args.host_workers,
                                sequenced=True if args.sequenced else None)
            lanes_.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t,
                                ds.geo.sin_t, cfg.n_frames * len(cfg.gains))
            ops = lanes_.pipes[0]
            run = lambda e: lanes_.submit(e, rank * F)  # noqa: E731
        else:
            ops = pipe = NativeShardPipeline(Comm(dev), cfg.gains, cfg.rows, cfg.bins,
                                             PathParams(), timing=timing,
                                             async_host=not args.sync_host,
                                             host_workers=args.host_workers)
            pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t,
                              ds.geo.sin_t, cfg.n_frames * len(cfg.gains))
            run = lambda e: pipe.run(e, rank * F)  # noqa: E731
    else:
        # host stages of consecutive stacks are independent (one tracker per stack): with fewer
        # workers than lanes, the stacks that finish together at the end of the timed region
        # queue their host stages (~6 ms each at 1000 frames) behind one another
        pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev, timing=timing,
                                  async_host=not args.sync_host, lanes=args.lanes,
                                  host_workers=args.host_workers, k1_gate=args.k1_gate)
        pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                          cfg.n_frames * len(cfg.gains))
        run = lambda e: pipe.submit(e)  # noqa: E731

    import faulthandler

    hang_s = float(os.environ.get("RPT_HANG_S", "180"))

    def alive():
        # hang guard (sharded runs): no step submitted or finished for hang_s seconds -> every
        # thread's stack to stderr (a lane thread shows the CommSequencer slot it waits in) and
        # exit 1, instead of waiting for the driver's limit
        if dist and hang_s > 0:
            faulthandler.dump_traceback_later(hang_s, exit=True)

    def resolve(r):
        alive()
        out = r.result() if hasattr(r, "result") else r
        alive()
        return out

    def points_of(r):  # K1 points of the whole (global) stack of a run
        return float(r.n_points_global if dist else r.n_points)

    if args.lanes > 1 and not args.python_shard:
        # lane setup (untimed, before the warm-up steps): one stack per lane allocates that lane's
        # buffers, whatever --warmup is (free lanes are taken in FIFO order: consecutive steps
        # waited for one at a time visit every lane)
        for k in range(args.lanes):
            resolve(run(echoes[k % E])).finish()
    for k in range(args.warmup):
        resolve(run(echoes[k % E])).finish()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    sharded_lanes = dist and not args.python_shard and args.lanes > 1
    if sharded_lanes:  # slot waits of the timed steps only
        lanes_.seq.wait_s = [0.0] * lanes_.seq.P
        lanes_.seq.wait_n = [0] * lanes_.seq.P
    t0 = time.perf_counter()
    stage_acc = {}
    k5 = []      # (K5 ms, points entering ST-DBSCAN) per timed run
    results = []
    for k in range(args.steps):
        alive()
        results.append(run(echoes[k % E]))
        if timing and dist and not sharded_lanes:
            k5.append((ops.last_core_ms(), ops.core_points))
    results = [resolve(r) for r in results]
    if timing and not dist:
        k5 = [(r.stage_ms["dbscan_core"], r.n_clustered_input) for r in results]
    for r in results:  # host stages (order + tracker) of the last runs, in order
        r.finish()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    slot_wait = None
    if sharded_lanes:
        slot_wait = {"ms_per_step_by_phase": [round(w / args.steps * 1e3, 4)
                                              for w in lanes_.seq.wait_s],
                     "entered_by_phase": list(lanes_.seq.wait_n),
                     "note": "time a lane thread waited for its CommSequencer turn, per "
                             "collective slot (0 info, 1 land, 2 halo, 3 flags, 4 comp ids, "
                             "5 pairs, 6 results, 7 redo), summed over lanes, per timed step"}
    for r in results:
        for key, v in r.stage_ms.items():
            stage_acc[key] = stage_acc.get(key, 0.0) + v
    pts_total = sum(points_of(r) for r in results)
    res = results[-1]
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t[0])
        summary = {"points_clustered_rank0": res.n_clustered_local, "clusters": res.n_clusters,
                   "segments": res.n_segments, "objects": len(res.tracker)
                   if res.tracker is not None else None}
    else:
        summary = {"points_clustered_rank0": res.n_clustered_input, "clusters": res.n_clusters,
                   "segments": res.n_segments, "objects": len(res.tracker)}
    summary["points_per_stack"] = sorted({int(points_of(r)) for r in results})
    value = pts_total / dt / 1e6
    ms_step = dt / args.steps * 1e3
    # steady state: the steps after the pipeline has filled (the first `lanes` steps) up to the
    # last step's device completion (the last host stage -- the drain -- excluded); max over ranks
    steady = None
    L_ = 1 if args.python_shard else args.lanes
    if args.steps > L_ + 1:
        # completion times in order: a run takes whichever lane is free, so runs can finish out
        # of submission order
        td = sorted(r.t_done for r in results)
        span = td[-1] - td[L_ - 1]
        if dist:
            t = torch.tensor([span], dtype=torch.float64, device=dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            span = float(t[0])
        pts_ss = sum(points_of(r) for r in results[L_:])
        steady = {"value": round(pts_ss / span / 1e6, 3), "unit": "Mpoints/s",
                  "ms_per_step": round(span / (args.steps - L_) * 1e3, 3),
                  "steps": args.steps - L_,
                  "done_ms": [round((x - t0) * 1e3, 2) for x in td],
                  "note": f"steps {L_}..{args.steps - 1}: from step {L_ - 1}'s device completion "
                          f"to the last step's (pipeline fill and the last host stage excluded); "
                          f"done_ms: every run's device completion after the timed region's start"}

    # one stack in flight (lanes = 1): the same steps strictly one after another.  K5's roofline
    # is taken here, where its kernels have the GPU to themselves (with several stacks in flight
    # the other stacks' kernels share the CUs and stretch every event-timed stage)
    seq = None
    if sharded_lanes:  # every rank: lane 0's pipeline, one stack at a time
        for k in range(max(args.warmup, 1)):
            ops.run(echoes[k % E], rank * F).finish()
        torch.cuda.synchronize(dev)
        tdist.barrier()
        ts0 = time.perf_counter()
        sres = []
        k5 = []
        for k in range(args.steps):
            sres.append(ops.run(echoes[k % E], rank * F))
            if timing:
                k5.append((ops.last_core_ms(), ops.core_points))
        for r in sres:
            r.finish()
        torch.cuda.synchronize(dev)
        tdist.barrier()
        t = torch.tensor([time.perf_counter() - ts0], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dts = float(t[0])
        seq = {"value": round(sum(points_of(r) for r in sres) / dts / 1e6, 3),
               "unit": "Mpoints/s", "ms_per_step": round(dts / args.steps * 1e3, 3),
               "steps": args.steps, "note": "same workload, one stack in flight per rank"}
        if timing:
            stage_acc = {}
            for r in sres:
                for key, v in r.stage_ms.items():
                    stage_acc[key] = stage_acc.get(key, 0.0) + v
    if not dist and args.lanes > 1 and not args.no_one_stack:
        spipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev, timing=timing,
                                   async_host=not args.sync_host, lanes=1)
        spipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t,
                           ds.geo.sin_t, cfg.n_frames * len(cfg.gains))
        for k in range(max(args.warmup, 1)):
            resolve(spipe.submit(echoes[k % E])).finish()
        torch.cuda.synchronize(dev)
        ts0 = time.perf_counter()
        sres = [resolve(spipe.submit(echoes[k % E])) for k in range(args.steps)]
        for r in sres:
            r.finish()
        torch.cuda.synchronize(dev)
        dts = time.perf_counter() - ts0
        seq = {"value": round(sum(points_of(r) for r in sres) / dts / 1e6, 3),
               "unit": "Mpoints/s", "ms_per_step": round(dts / args.steps * 1e3, 3),
               "steps": args.steps, "note": "same workload, one stack in flight (lanes=1)"}
        if timing:
            k5 = [(r.stage_ms["dbscan_core"], r.n_clustered_input) for r in sres]
            # per-stage times from this leg too: with several stacks in flight every event-timed
            # stage also contains the other stacks' interleaved kernels
            stage_acc = {}
            for r in sres:
                for key, v in r.stage_ms.items():
                    stage_acc[key] = stage_acc.get(key, 0.0) + v
        del spipe

    # optional leg: steps with the echo's H2D copy from pinned host memory inside (stack 0)
    h2d = None
    if args.h2d_steps > 0:
        echo = echoes[0]
        host = torch.empty(echo.shape, dtype=echo.dtype, pin_memory=True)
        host.copy_(echo)
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
        th0 = time.perf_counter()
        hres = []
        for _ in range(args.h2d_steps):
            echo.copy_(host, non_blocking=True)
            hres.append(run(echo))
        hres = [resolve(r) for r in hres]
        for r in hres:
            r.finish()
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
        dth = time.perf_counter() - th0
        if dist:
            t = torch.tensor([dth], dtype=torch.float64, device=dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            dth = float(t[0])
        h2d = {"value": round(sum(points_of(r) for r in hres) / dth / 1e6, 3),
               "unit": "Mpoints/s", "ms_per_step": round(dth / args.h2d_steps * 1e3, 3),
               "steps": args.h2d_steps,
               "echo_bytes_per_rank": int(echo.numel() * echo.element_size()),
               "note": "each step first copies the u8 echo of stack 0 from pinned host memory "
                       "(PCIe), then runs the same path; not the headline value"}
        del host

    wkey = f"{'dense' if args.dense else 'std'}_{F}f"
    traffic, tsrc = (None, None) if dist else _traffic(f"k5_traffic_{wkey}.json")
    roof = None
    k5 = [(a, b) for a, b in k5 if a is not None]
    if k5:
        k5_ms = float(np.mean([a for a, _ in k5]))
        n_in = float(np.mean([b for _, b in k5]))
        roof = {"kernel": "K5 = k_core_cells_oct<FUSED> (cell decisions, point flags, queue) + "
                          "k_core_slow (core flags)",
                "measured_in": "one-stack-in-flight leg" if seq is not None else "timed steps",
                **_k5_roof(n_in, k5_ms, traffic, tsrc), "runs": len(k5)}
    stage = {k: round(v / args.steps, 3) for k, v in stage_acc.items()}
    e0 = echoes[0]
    roof_e2e = _e2e_roof(float(e0.numel() * e0.element_size()) * world, ms_step, world,
                         f"{'dense' if args.dense else 'std'}_{F}f")
    # the largest stage, K1 (count + scan + write): echo read once + 16 B per emitted point
    # (x, y, intensity, frame slot; no per-point gain without keep_points) + 12 B of row geometry
    # per row, over its event time
    roof_k1 = None
    if stage.get("polar") and not dist:
        e0 = echoes[0]
        k1_bytes = int(e0.numel() * e0.element_size()) + 16 * int(pts_total / args.steps) + \
            12 * int(e0.shape[0]) * int(e0.shape[1]) * int(e0.shape[2])
        k1_ach = k1_bytes / (stage["polar"] * 1e-3) / 1e9
        roof_k1 = {"kernel": "K1 stage = k_group_count_u8 + scans + k_group_starts + "
                             "k_expand_write (+ unstaged groups)",
                   "bound": "hbm", "achieved": round(k1_ach, 2), "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": round(k1_ach / HBM_PEAK_GBS, 4),
                   "avg_ms": stage["polar"], "bytes_model": "1 B per echo sample + 16 B per "
                   "point written + 12 B per row (SURVEY 8d's K1 terms for u8 echo)",
                   "bytes": k1_bytes, "traffic": None}
        t1, src1 = _traffic(f"k1_traffic_{wkey}.json")
        if t1 is not None:  # PMC-measured HBM bytes of the K1 kernels, same workload
            roof_k1["traffic"] = t1
            roof_k1["traffic_unit"] = f"bytes per run (PMC, {src1})"

    # K5 again at the per-GPU shares where SURVEY 8(d) sets its 0.40 target (8 GPUs): the
    # configs[3] stack's 125 standard frames and configs[4]'s 125 dense frames
    roof_c4 = roof_c4d = None
    if rank == 0 and not dist and not args.dense and timing and not args.no_dense_k5:
        from rpt.synth import dense_config

        roof_c4 = _k5_share(dev, SynthConfig(n_frames=125),
                            "configs[3] per-GPU share at 8 GPUs: 125 standard frames",
                            "std_125f")
        roof_c4d = _k5_share(dev, dense_config(n_frames=125),
                             "configs[4] per-GPU share at 8 GPUs: 125 dense frames "
                             "(~490k pts/frame)", "dense_125f")

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and not dist:
        cf = min(args.cpu_frames, F)
        eh = echoes[0][:cf].cpu().numpy()
        npts, nfr, cdt, same, index = cpu_baseline(eh, cfg, ds.geo, structure=True)
        gp, gf, gdt, _, _ = cpu_baseline(echoes[0][:8].cpu().numpy(), cfg, ds.geo,
                                         structure=False)
        cpu = {"value": round(npts / cdt / 1e6, 6), "unit": "Mpoints/s", "cores": 1,
               "kind": "port",
               "what": "the reference's algorithmic structure restated (oracle/refpath.py: "
                       "whole-stack sklearn BallTree query, per-neighbour float32 time filter "
                       "in Python, seed-set expansion; calibrated to 1.05-1.12x the reference's "
                       "own time in the build container by tools/time_reference.py "
                       "--calibrate-refpath, profiles/r4/refpath_calibration.json) "
                       "+ numpy polar scatter + oracle tracker, 1 thread on this node",
               "index": index, "labels_equal_oracle": same,
               "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
               "sample": f"first {nfr} frame(s) of the same stack ({npts} points), {cdt:.1f} s; "
                         f"the reference's cost per point grows with the frames in its one "
                         f"BallTree, so the rate does not extrapolate to 1000 frames",
               "grid_bfs_port": {"value": round(gp / gdt / 1e6, 5), "unit": "Mpoints/s",
                                 "sample": f"first {gf} frames ({gp} points), {gdt:.1f} s",
                                 "what": "oracle/ grid-indexed C BFS (not the reference's "
                                         "structure), 1 thread"},
               "reference_measured": _reference_measured()}
        if args.best_cpu_frames > 0:
            bf = min(args.best_cpu_frames, F)
            bp, bfr, bdt = best_cpu(echoes[0][:bf].cpu().numpy(), cfg, ds.geo)
            cpu["best_cpu"] = {
                "value": round(bp / bdt / 1e6, 5), "unit": "Mpoints/s",
                "cores": int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1),
                "kind": "port",
                "sample": f"first {bfr} frames of the same stack ({bp} points), {bdt:.1f} s",
                "what": "oracle's OpenMP union-find ST-DBSCAN (oracle/stdbscan_oracle.c) + numpy "
                        "polar scatter / land filter + oracle tracker on all cores the process "
                        "may use (OMP_NUM_THREADS): the fastest CPU path here, not the "
                        "reference's structure"}
    if rank == 0:
        what = "dense (configs[4] density, ~500k pts/frame)" if args.dense else \
            "3-gain fused"
        if scaling == "strong":
            wl = (f"ONE {total}-frame {what} stack (4096 az x 1024 echo u8) split over {world} "
                  f"GPU(s), {F} frames each; land filter + ST-DBSCAN eps 8 / eps_t 2 / min 15 + "
                  f"Hungarian tracking (BASELINE configs[3]"
                  f"{' / configs[4]' if args.dense else ''}, strong scaling)")
        else:
            wl = (f"{F}-frame {what} stack per GPU (4096 az x 1024 echo u8), land filter + "
                  f"ST-DBSCAN eps 8 / eps_t 2 / min 15 + Hungarian tracking "
                  f"(BASELINE configs[2] at F=100, weak scaling)")
        out = {
            "metric": "Mpoints/s clustered+tracked, 1024-echo synthetic frames; 1/2/4/8-GPU scaling",
            "value": round(value, 3), "unit": "Mpoints/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None,
            "dtype": "u8 echo / f32 geometry / f64 distance",
            "data": "synthetic (device-generated, seeded): "
                    + ("one stack replayed" if E == 1 else
                       "two stacks (seed 0 / 1) alternating over the steps"),
            "config": {"workload": wl, "total_frames": total, "frames_per_gpu": F,
                       "points_per_step": int(round(pts_total / args.steps)), **summary,
                       "parallelism": (f"frame-sharded x{world}"
                                       f"{' (python stages)' if args.python_shard else ''}")
                       if dist else "single GPU",
                       "stacks_in_flight": 1 if args.python_shard else args.lanes,
                       "host_stage": "inline" if args.sync_host else
                       "overlapped: step k's order+tracker runs on a host thread during step "
                       "k+1's device work; the timed region ends after the last one"},
            "steady_state": steady,
            "slot_wait": slot_wait,
            "one_stack_in_flight": seq,
            "roofline": roof, "roofline_c4_share": roof_c4, "roofline_configs4_share": roof_c4d,
            "roofline_k1": roof_k1,
            "roofline_e2e": roof_e2e,
            "cpu_baseline": cpu,
            "h2d_inclusive": h2d, "stage_ms": stage,
            "stage_ms_from": "one_stack_in_flight" if seq is not None else "timed steps",
        }
        print(json.dumps(out), flush=True)
    faulthandler.cancel_dump_traceback_later()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
