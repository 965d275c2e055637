#!/usr/bin/env python3
"""Host time per step around rpt_stack_run (one stack in flight): wall per step, time inside the
native call, and the Python before / after it.  Usage: python tools/host_gap.py FRAMES
[async | nohost] (nohost: async with the order + tracker stage replaced by a no-op)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "radar-point-cloud-tracking_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rpt.pipeline import FrameStackPipeline, PathParams  # noqa: E402
from rpt.synth import DeviceSynth, SynthConfig  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 125
async_host = len(sys.argv) > 2 and sys.argv[2] in ("async", "nohost")
if len(sys.argv) > 2 and sys.argv[2] == "nohost":  # host stage replaced by a no-op (GIL probe)
    import rpt.pipeline as _pl
    _pl.order_and_track = lambda *a, **k: (None, None, None)
dev = torch.device("cuda", 0)
cfg = SynthConfig(n_frames=F, rows=4096)
ds = DeviceSynth(cfg, dev)
echo = ds.echo()
pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev, async_host=async_host)
pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t, F * 3)
lib = pipe.lib
inner = []
orig = lib.rpt_stack_run


class Wrap:
    def __getattr__(self, k):
        return getattr(lib, k)

    def rpt_stack_run(self, *a):
        t0 = time.perf_counter()
        r = orig(*a)
        inner.append(time.perf_counter() - t0)
        return r


pipe.lib = Wrap()
for _ in range(3):
    pipe.run(echo).finish()
torch.cuda.synchronize()
inner.clear()
walls = []
res = []
for _ in range(20):
    t0 = time.perf_counter()
    res.append(pipe.run(echo))
    walls.append(time.perf_counter() - t0)
for r in res:
    r.finish()
w, i = np.median(walls) * 1e3, np.median(inner) * 1e3
print(f"frames={F} async={async_host} wall/step {w:.3f} ms, inside rpt_stack_run {i:.3f} ms, "
      f"python around it {w - i:.3f} ms")
