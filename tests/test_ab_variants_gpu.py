"""Every kernel form the A/B build keeps selectable (librpt_ab.so, the only build that reads the
RPT_* switches; tools/ab_*.sh measure with it) must give the shipped library's results: three child
processes, each with a set of switches at non-default values, run the same 14-frame stack (land
filter on) and return labels, per-(frame, label) rows, K1 points and tracks, compared bit for bit
with librpt.so's run in this process.  Together the sets flip every switch the A/B build reads."""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

COMBOS = [
    {"RPT_K1_STAGE": "0", "RPT_LAND_U8": "0", "RPT_K4_BUCKET": "0", "RPT_UNION_LIST": "0",
     "RPT_UF_COMPRESS": "1", "RPT_CELL_ROOTS": "0", "RPT_K7_W": "64", "RPT_K9_RADIX": "1",
     "RPT_UNION_PAIR": "0"},
    {"RPT_K1_EXPAND": "0", "RPT_SLAB_CHUNKS": "3", "RPT_K5_MODE": "2", "RPT_F32_SCREEN": "0",
     "RPT_UF_FLAGS": "0"},
    {"RPT_K5_TILES": "1", "RPT_K7_TILES": "1", "RPT_CELL_SIDE": "0.5"},
    # round-5 paths forced on a stack their default rules would not take them for (and off):
    # small cells one lane each, the inverse permutation with original-order core labels, no
    # root snapshot before the listed union pass, k_union over every point
    {"RPT_CELL_BOX_MIXED": "2", "RPT_LABEL_ORIG": "2", "RPT_UNION_SNAP": "0",
     "RPT_UNION_NM": "0"},
]

RUN = r'''
import numpy as np, torch
from rpt.pipeline import FrameStackPipeline, PathParams
from rpt.synth import DeviceSynth, SynthConfig

def run_stack():
    dev = torch.device("cuda", 0)
    cfg = SynthConfig(n_frames=14, rows=1024, n_targets=14, clutter_density=0.01)
    ds = DeviceSynth(cfg, dev)
    pipe = FrameStackPipeline(cfg.gains, cfg.rows, cfg.bins, PathParams(), dev)
    pipe.set_geometry(np.full(cfg.rows, cfg.scale, np.float32), ds.geo.cos_t, ds.geo.sin_t,
                      cfg.n_frames * 3)
    res = pipe.run(ds.echo(), keep_points=True).finish()
    out = {"labels": res.labels.cpu().numpy()}
    for k in ("x", "y", "v", "gain", "frame"):
        out["p_" + k] = res.points[k].cpu().numpy()
    seg = {k: np.asarray(v) for k, v in res.seg.items()}
    key = np.lexsort((seg["label"], seg["frame"]))  # K9's radix form is label-major
    for k, v in seg.items():
        out["s_" + k] = v[key]
    fo, order = res.frame_order_offsets, res.frame_order  # rows in reference order
    out["rows"] = np.array([(f, seg["label"][s], seg["count"][s], seg["cx"][s], seg["cy"][s],
                             seg["mi"][s]) for f in range(len(fo) - 1)
                            for s in order[fo[f]:fo[f + 1]]], np.float64).reshape(-1, 6)
    objs = res.tracker.objects()
    out["obj_id"] = np.array([o.object_id for o in objs])
    out["obj_pos"] = (np.vstack([np.vstack(o.positions) for o in objs]) if objs
                      else np.zeros((0, 2)))
    return out
'''


def _run_here():
    ns = {}
    exec(RUN, ns)  # noqa: S102 (the same code the children run)
    return ns["run_stack"]()


@pytest.mark.parametrize("combo", range(len(COMBOS)))
def test_ab_kernel_forms_match_shipped_library(gpu, combo):
    from rpt import _build

    from rpt import _abi

    assert _build.LIB_AB.exists(), "librpt_ab.so missing: run __graft_entry__.build()"
    assert _abi.load()._name.endswith("librpt.so")
    ref = _run_here()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.npz")
        code = (f"import sys\nsys.path[:0] = {sys.path!r}\n" + RUN +
                "from rpt import _abi\nassert _abi.load()._name.endswith('librpt_ab.so')\n"
                f"import numpy as np\nnp.savez({out!r}, **run_stack())\n")
        env = dict(os.environ, RPT_LIB=str(_build.LIB_AB), **COMBOS[combo])
        subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=240)
        got = np.load(out)
        assert sorted(got.files) == sorted(ref)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} with {COMBOS[combo]}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("combo", range(len(COMBOS)))
def test_ab_kernel_forms_sharded_match_single(gpu, combo):
    """The frame-sharded path (2 gloo ranks on cuda:0, librpt's rpt_shard_* driver; the sharded
    labelling step reads the cell roots the switches change) on librpt_ab.so with each switch set:
    rank 0 checks it against the single-GPU stack of the same build and switches, which the test
    above ties to the shipped library (tools/dist_check.py, as tests/test_dist_gpu.py)."""
    from pathlib import Path

    from rpt import _build
    from test_dist_gpu import _free_port

    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, RPT_LIB=str(_build.LIB_AB), **COMBOS[combo])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           str(root / "tools" / "dist_check.py"), "--backend", "gloo", "--frames", "14",
           "--impl", "native", "--lanes", "1"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ok=True" in out, out[-4000:]
