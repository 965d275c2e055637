#!/usr/bin/env python3
"""Dump the bench workload's per-segment summaries (host arrays fed to the tracker) to
gpurun_out/seg.npz, for profiling the host stage off the GPU box."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "radar-point-cloud-tracking_amd"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rpt.pipeline import FrameStackPipeline, PathParams  # noqa: E402
from rpt.synth import DeviceSynth, SynthConfig  # noqa: E402

dev = torch.device("cuda", 0)
cfg = SynthConfig(n_frames=int(sys.argv[1]) if len(sys.argv) > 1 else 100)
ds = DeviceSynth(cfg, dev)
echo = ds.echo()
pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev)
pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                  cfg.n_frames * 3)
res = pipe.run(echo, keep_points=True)
out = ROOT / "gpurun_out"
out.mkdir(exist_ok=True)
lab = res.labels.cpu().numpy()
pf = res.points["frame"].cpu().numpy()
np.savez(out / "seg.npz", built=res.frame_ids, **{"seg_" + k: v for k, v in res.seg.items()},
         n_frames=cfg.n_frames, first_noise=res.first_noise)
print("segments", res.n_segments, "max count", int(res.seg["count"].max()),
      "top5", np.sort(res.seg["count"])[-5:].tolist(), "noise", int((lab < 0).sum()))
