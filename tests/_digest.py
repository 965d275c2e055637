"""Compact digests of a stack result (tests only).

The headline workload (BASELINE configs[3]: ONE 1000-frame fused stack, ~50 M points) is too
large for the oracle to run inside the GPU suite (the union-find oracle alone takes minutes), so
``tests/golden/make_bigstack.py`` runs ``oracle.run_path`` on the same seeded input in the build
container (numpy restatement of the device generator, pinned equal by
``test_path_gpu.py::test_synth_echo_bit_identical``) and commits these digests; the GPU test
computes the same digests from the device result.  Per-frame digests (labels, cluster rows in
reference order) and per-object digests localise a mismatch to a frame / a track.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Sequence

import numpy as np

ROW_DTYPE = np.dtype([("label", "<i4"), ("count", "<i8"), ("cx", "<f4"), ("cy", "<f4"),
                      ("mi", "<f4")])


def _h(*parts: bytes) -> str:
    h = hashlib.blake2b(digest_size=8)
    for p in parts:
        h.update(p)
    return h.hexdigest()


def label_digests(labels: np.ndarray, counts: Sequence[int]) -> List[str]:
    """One digest per built frame of its (land-filtered) points' labels, in stack order."""
    labels = np.ascontiguousarray(labels, dtype="<i4")
    out, off = [], 0
    for c in counts:
        out.append(_h(labels[off:off + c].tobytes()))
        off += c
    assert off == len(labels)
    return out


def rows_digest(rows) -> str:
    """rows: [(label, count, cx, cy, mean_intensity)] of one frame in reference order."""
    a = np.array([(int(l), int(n), np.float32(x), np.float32(y), np.float32(m))
                  for l, n, x, y, m in rows], dtype=ROW_DTYPE)
    return _h(a.tobytes())


def object_digest(oid: int, otype: str, positions, frames_seen) -> str:
    pos = np.vstack(positions).astype(np.float64) if len(positions) else np.zeros((0, 2))
    return _h(np.int64(oid).tobytes(), otype.encode(), pos.tobytes(),
              np.asarray(frames_seen, dtype="<i8").tobytes())


def oracle_digest(frames_in, o_frames, o_labels, o_clusters, o_trk, land_cells: int) -> Dict:
    """Digest of oracle.run_path's outputs (frames_in: the built frames before the land filter)."""
    return {
        "n_points": int(sum(len(p) for _, p, _ in frames_in)),
        "n_clustered_input": int(len(o_labels)),
        "n_land_cells": int(land_cells),
        "n_clusters": int(o_labels.max()) + 1 if len(o_labels) else 0,
        "frame_ids": [int(f) for f, _, _ in o_frames],
        "frame_counts": [int(len(p)) for _, p, _ in o_frames],
        "labels": label_digests(o_labels, [len(p) for _, p, _ in o_frames]),
        "rows": [rows_digest([(c[0], c[1], c[2][0], c[2][1], c[3])
                              for c in o_clusters.get(fid, [])]) for fid, _, _ in o_frames],
        "objects": [object_digest(o.object_id, o.object_type, o.positions, o.frames_seen)
                    for o in o_trk.objects.values()],
    }


def device_digest(res) -> Dict:
    """The same digest from a device StackResult run with keep_points=True (host stage done)."""
    lab = res.labels.cpu().numpy()
    pf = res.points["frame"].cpu().numpy()
    fids = [int(f) for f in res.frame_ids]
    counts = np.bincount(pf, minlength=max(fids) + 1 if fids else 0) if len(pf) else \
        np.zeros(max(fids) + 1 if fids else 0, np.int64)
    fo, order, seg = res.frame_order_offsets, res.frame_order, res.seg
    rows = []
    for f in fids:
        rows.append(rows_digest([(seg["label"][s], seg["count"][s], seg["cx"][s], seg["cy"][s],
                                  seg["mi"][s]) for s in order[fo[f]:fo[f + 1]]]))
    return {
        "n_points": int(res.n_points),
        "n_clustered_input": int(res.n_clustered_input),
        "n_land_cells": int(res.n_land_cells),
        "n_clusters": int(res.n_clusters),
        "frame_ids": fids,
        "frame_counts": [int(counts[f]) for f in fids],
        "labels": label_digests(lab, [int(counts[f]) for f in fids]),
        "rows": rows,
        "objects": [object_digest(o.object_id, o.object_type, o.positions, o.frames_seen)
                    for o in res.tracker.objects()],
    }


def shard_digest(res, labels: np.ndarray, frame_counts: np.ndarray) -> Dict:
    """The digest from rank 0's ShardResult of the frame-sharded path (rpt.dist; host stage
    done), every rank's labels concatenated in rank order and the kept points per global frame
    slot (the land-cell count is not reported by the sharded path: None)."""
    fids = [int(f) for f in res.built_global]
    fo, order, seg = res.frame_order_offsets, res.frame_order, res.seg
    rows = [rows_digest([(seg["label"][s], seg["count"][s], seg["cx"][s], seg["cy"][s],
                          seg["mi"][s]) for s in order[fo[f]:fo[f + 1]]]) for f in fids]
    return {
        "n_points": int(res.n_points_global),
        "n_clustered_input": int(len(labels)),
        "n_land_cells": None,
        "n_clusters": int(res.n_clusters),
        "frame_ids": fids,
        "frame_counts": [int(frame_counts[f]) for f in fids],
        "labels": label_digests(labels, [int(frame_counts[f]) for f in fids]),
        "rows": rows,
        "objects": [object_digest(o.object_id, o.object_type, o.positions, o.frames_seen)
                    for o in res.tracker.objects()],
    }


def compare(got: Dict, exp: Dict, what: str = ""):
    """Assert equality with the first differing frame / object named (a None in `got` = not
    reported by that path)."""
    for k in ("n_points", "n_clustered_input", "n_land_cells", "n_clusters", "frame_ids",
              "frame_counts"):
        if got[k] is None:
            continue
        assert got[k] == exp[k], f"{what}: {k} differs: {got[k]!r:.200} vs {exp[k]!r:.200}"
    for k in ("labels", "rows"):
        bad = [exp["frame_ids"][i] for i, (a, b) in enumerate(zip(got[k], exp[k])) if a != b]
        assert not bad, f"{what}: {k} differ in {len(bad)} frames, first {bad[:5]}"
    assert len(got["objects"]) == len(exp["objects"]), \
        f"{what}: {len(got['objects'])} tracked objects vs {len(exp['objects'])}"
    bad = [i for i, (a, b) in enumerate(zip(got["objects"], exp["objects"])) if a != b]
    assert not bad, f"{what}: tracked objects differ at positions {bad[:5]}"
