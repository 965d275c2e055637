"""Time the stack's host stage (cluster order + tracker) on a dumped input
(tools/dump_host_input.py): the two-step form (rpt_order_clusters, numpy gather,
rpt_tracker_run) against the fused rpt_order_and_track, best of --reps, and check both give the
same order and tracker state.

    python tools/host_stage_bench.py gpurun_out/host_input.npz [--reps 20]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "radar-point-cloud-tracking_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from rpt import stages
    from rpt.pipeline import PathParams

    d = np.load(a.npz)
    F = int(d["n_frames"])
    seg = {k[4:]: d[k] for k in d.files if k.startswith("seg_")}
    noise, built = d["first_noise"], d["built"]
    p = PathParams()
    S = len(seg["frame"])
    print(f"{a.npz}: {F} frames, {len(built)} built, {S} segments "
          f"({S / max(len(built), 1):.1f} per built frame)")

    def best(fn):
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = fn()
            ts.append(time.perf_counter() - t0)
        return min(ts) * 1e3, float(np.median(ts)) * 1e3, out

    o_ms, o_med, (fo, order) = best(lambda: stages.order_frames(F, seg, noise))
    t_ms, t_med, trk1 = best(lambda: stages.track_ordered(built, fo, order, seg, p))
    f_ms, f_med, (fo2, order2, trk2) = best(
        lambda: stages.order_and_track(F, built, seg, noise, p))
    assert np.array_equal(fo, fo2) and np.array_equal(order, order2)
    assert len(trk1) == len(trk2)
    for x, y in zip(trk1.objects(), trk2.objects()):
        assert x.object_id == y.object_id and x.frames_seen == y.frames_seen
        assert np.array_equal(np.vstack(x.positions), np.vstack(y.positions))
    print(f"order {o_ms:.2f} ms (median {o_med:.2f}), gather + tracker {t_ms:.2f} "
          f"(median {t_med:.2f}), two-step {o_ms + t_ms:.2f}; fused {f_ms:.2f} "
          f"(median {f_med:.2f}); {len(trk2)} objects at the end")


if __name__ == "__main__":
    main()
