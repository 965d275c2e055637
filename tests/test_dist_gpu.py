"""Frame-sharded path on the GPU: 2 or 3 ranks (gloo, sharing cuda:0 on a one-GPU box) run
rpt.dist.NativeShardPipeline (librpt's rpt_shard_* driver) or ShardedStackPipeline over librpt; rank 0 compares with the oracle's
run_path over the whole stack and with the single-GPU FrameStackPipeline (labels, per-frame
cluster rows in reference order, tracked objects).
The ranks are started by torch.distributed.run as child processes (tools/dist_check.py)."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, frames, impl, lanes, extra, timeout=600, backend="gloo"):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", str(ROOT / "tools" / "dist_check.py"),
           "--backend", backend, "--frames", str(frames), "--impl", impl, "--lanes", str(lanes),
           *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ok=True" in out, out[-4000:]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("world,frames,impl,lanes", [(2, 14, "native", 1), (3, 6, "native", 1),
                                                     (2, 14, "python", 1), (2, 8, "native", 2),
                                                     (3, 6, "native", 3),
                                                     (3, 6, "native-tinycaps", 1),
                                                     (4, 4, "native-tinycaps", 2),
                                                     (3, 6, "native-hostmerge", 1),
                                                     (2, 8, "native-hostmerge", 2)])
def test_sharded_gpu_matches_single_gpu(world, frames, impl, lanes):
    """lanes = 2 / 3: stacks in flight (rpt.dist.ShardLanes: a stream and thread per lane, every
    lane's collectives through the ONE process group in the CommSequencer's software-pipeline
    order); each lane's last run is checked.  native-tinycaps: one-pair / 16-word capacities for
    the pair and packed-result gathers, so every step is finished again with grown capacities
    (the redo slot).  native-hostmerge: device merge limit 0, so every step's equivalence pairs
    are merged on the host (rpt_merge_equivalences, rpt/dist.py's flag-2 branch of the redo
    slot: the path a merge of more than 8192 ids takes) and the step finished again with them."""
    extra = []
    if impl == "native-tinycaps":
        impl, extra = "native", ["--tiny-caps"]
    elif impl == "native-hostmerge":
        impl, extra = "native", ["--force-host-merge"]
    # rank 0 checks every run against the oracle's run_path over the whole stack as well
    # (labels, per-frame cluster rows in reference order, tracked objects), not only against
    # the single-GPU pipeline
    out = _run(world, frames, impl, lanes, extra + ["--oracle"])
    assert "labels_equal=True rows_equal=True tracks_equal=True" in out, out[-4000:]


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,frames,lanes", [(8, 2, 1), (4, 4, 2)])
def test_sharded_dense_giant_component_matches_oracle(world, frames, lanes):
    """configs[4]'s density split over ranks of 2 and 4 frames: one giant component crosses
    every rank boundary (its halo ids pair up along the whole chain), ~490k points per frame;
    rank 0 compares labels, the per-frame cluster rows in reference order and the tracked objects
    with the oracle's run_path (union-find ST-DBSCAN) over the whole stack
    (4_temporal_object_tracker.py:466-506, 508-536, 984-991)."""
    _run(world, frames, "native", lanes, ["--dense", "--oracle"], timeout=840)


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("redo", ["--tiny-caps", "--force-host-merge"])
def test_sharded_dense_redo_slot_matches_oracle(redo):
    """The redo slot on DENSE slabs: there the grid build leaves the inverse permutation in the
    slab buffer and the global label pass reads it once before overwriting it with the core
    labels (k_label_global_orig, then k_label_global_core), so a step finished a second time
    (pair / result capacities exceeded, or the equivalences merged on the host) must take the
    sorted-order form on its second call.  2 ranks x 2 dense frames, every step finished again,
    against the oracle's run_path over the whole stack (4_temporal_object_tracker.py:466-506)."""
    _run(2, 2, "native", 1, ["--dense", "--oracle", redo], timeout=840)


@pytest.mark.gpu
@pytest.mark.timeout(1000)
def test_sharded_config4_full_share_sample_check():
    """BASELINE configs[4] at its real per-rank shape: 8 gloo ranks sharing the GPU, each with
    125 dense frames (~490k points per frame, ~61 M points per rank, ~490 M in all, one component
    chaining the whole stack) through NativeShardPipeline.  No whole-stack reference fits, so
    every rank checks its core flags and labels against oracle.sample_check's exact
    neighbourhoods on every point of its first and last floor(eps_t) = 2 frames (the halo, the
    cross-rank merge and the global numbering all meet there) plus 50,000 random points; rank 0
    checks the global cluster numbering and its frames' K9 rows (tools/dist_check.py
    run_sample_check; 4_temporal_object_tracker.py:466-506, 527-531)."""
    out = _run(8, 125, "native", 1, ["--dense", "--sample-check"], timeout=960)
    assert out.count("edge-frame points") == 8, out[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 2])
def test_rccl_world1_forced_collectives_match_single_gpu(lanes):
    """The RCCL (nccl backend) branch of rpt.dist.Comm on one GPU: world 1 with the identity
    shortcut off, so the land-grid all_reduce, the info all_gather, the device-resident pair and
    result gathers (all_gather_into_tensor on the lane's stream) and, at lanes = 2, the
    CommSequencer all run through RCCL; the result must equal the single-GPU pipeline's."""
    out = _run(1, 10, "native", lanes, ["--force-collectives"], backend="nccl", timeout=300)
    assert "backend=nccl" in out, out[-4000:]
