#!/usr/bin/env python3
"""K1 timing on the bench's synthetic stack: hipEvent time of the staged count pass (count
kernel + group scan + file offsets) and of the staged write pass, each repeated, for every
library given (default: the in-tree build; RPT_LIB paths as extra arguments, interleaved so they
share the box).  Usage: python tools/k1_time.py FRAMES [lib.so ...]"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "radar-point-cloud-tracking_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rpt import _abi  # noqa: E402
from rpt._device import stream_handle  # noqa: E402
from rpt.pipeline import PathParams  # noqa: E402
from rpt.synth import DeviceSynth, SynthConfig  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
libs = sys.argv[2:] or [str(_abi._LIB_PATH)]
dev = torch.device("cuda", 0)
cfg = SynthConfig(n_frames=F, rows=4096)
ds = DeviceSynth(cfg, dev)
echo = ds.echo()
nf, rows, bins = F * 3, cfg.rows, cfg.bins
p = PathParams()
sc = torch.full((nf * rows,), cfg.scale, dtype=torch.float32, device=dev)
cd = torch.from_numpy(np.tile(ds.geo.cos_t, nf)).to(dev)
sd = torch.from_numpy(np.tile(ds.geo.sin_t, nf)).to(dev)
gd = torch.tensor(list(cfg.gains) * F, dtype=torch.int32, device=dev)
st = stream_handle(dev)
loaded = [C.CDLL(lp) for lp in libs]
lib0 = _abi.load()
words = int(lib0.rpt_polar_stage_words(nf, rows))
mk = torch.zeros(words, dtype=torch.int32, device=dev)  # zero: diagnostic builds may skip it
rp = torch.empty(nf * ((rows + 3) // 4) + 1, dtype=torch.int64, device=dev)
fo = torch.empty(nf + 1, dtype=torch.int64, device=dev)
tot = C.c_int64(0)
thr = float(np.float32(p.threshold))
res = {lp: ([], []) for lp in libs}
out = None
for rep in range(6):
    for lp, L in zip(libs, loaded):
        fn_c = L.rpt_polar_count_staged
        fn_c.restype = C.c_int32
        fn_c.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_float,
                         C.c_int32, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.c_void_p,
                         C.c_void_p]
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        e0.record()
        s = fn_c(echo.data_ptr(), _abi.ECHO_U8, nf, rows, bins, thr, int(p.stride),
                 rp.data_ptr(), fo.data_ptr(), C.byref(tot), mk.data_ptr(), st)
        assert s == 0, s
        e1.record()
        n = tot.value
        if out is None or out[0].numel() < n:
            out = [torch.empty(max(n, 1), dtype=torch.float32, device=dev) for _ in range(3)] + \
                  [torch.empty(max(n, 1), dtype=torch.int32, device=dev) for _ in range(2)]
        fn_w = L.rpt_polar_write_staged
        fn_w.restype = C.c_int32
        e1b = torch.cuda.Event(enable_timing=True)
        e1b.record()
        s = fn_w(C.c_void_p(echo.data_ptr()), C.c_int32(_abi.ECHO_U8), C.c_int64(nf),
                 C.c_int32(rows), C.c_int32(bins), C.c_void_p(sc.data_ptr()),
                 C.c_void_p(cd.data_ptr()), C.c_void_p(sd.data_ptr()), C.c_void_p(gd.data_ptr()),
                 C.c_float(thr), C.c_int32(int(p.stride)), C.c_void_p(rp.data_ptr()),
                 C.c_void_p(fo.data_ptr()), C.c_int32(3), *[C.c_void_p(o.data_ptr()) for o in out],
                 C.c_void_p(mk.data_ptr()), C.c_void_p(st))
        assert s == 0, s
        e2.record()
        torch.cuda.synchronize()
        if rep:
            res[lp][0].append(e0.elapsed_time(e1))
            res[lp][1].append(e1b.elapsed_time(e2))
for lp in libs:
    c, w = res[lp]
    print(f"{os.path.basename(lp)} frames={F} points={tot.value} count_ms={np.median(c):.3f} "
          f"(min {min(c):.3f}) write_ms={np.median(w):.3f} (min {min(w):.3f}) "
          f"echo_GBps={nf * rows * bins / np.median(c) / 1e6:.0f}")
