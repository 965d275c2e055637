"""ctypes binding of librpt.so (the C-ABI declared in include/rpt.h).

The library is the product: every numeric entry point of ``rpt`` goes through it.  There is no
CPU fallback; when the library or a GPU is missing the call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parent / "librpt.so"

RPT_OK = 0
RPT_EINVAL = 1
RPT_ENOMEM = 2
RPT_EHIP = 3
RPT_EEMPTY = 4
RPT_ENOTSUP = 5
RPT_ENONFINITE = 6

ECHO_F32 = 0
ECHO_U8 = 1

c_f32p = C.POINTER(C.c_float)
c_f64p = C.POINTER(C.c_double)
c_i32p = C.POINTER(C.c_int32)
c_i64p = C.POINTER(C.c_int64)
c_u8p = C.POINTER(C.c_uint8)
c_u32p = C.POINTER(C.c_uint32)
vp = C.c_void_p


class StdbscanStats(C.Structure):
    _fields_ = [
        ("n_points", C.c_int64),
        ("n_core", C.c_int64),
        ("n_clusters", C.c_int32),
        ("grid_dims", C.c_int32 * 4),
        ("grid_cells", C.c_int64),
        ("ms_bounds", C.c_double),
        ("ms_grid", C.c_double),
        ("ms_core", C.c_double),
        ("ms_union", C.c_double),
        ("ms_label", C.c_double),
        ("timing", C.c_int32),
    ]


class TrackerParams(C.Structure):
    _fields_ = [
        ("max_association_distance", C.c_double),
        ("max_missed_frames", C.c_int32),
        ("motion_history_frames", C.c_int32),
        ("stationary_velocity_threshold", C.c_double),
    ]


class ObjectInfo(C.Structure):
    _fields_ = [
        ("object_id", C.c_int64),
        ("object_type", C.c_int32),
        ("n_positions", C.c_int32),
        ("n_velocities", C.c_int32),
        ("last_seen_frame", C.c_int64),
        ("average_velocity", C.c_double),
        ("average_velocity_is_f32", C.c_int32),
        ("color", C.c_int32 * 3),
    ]


class SynthParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("rows", C.c_int32),
        ("bins", C.c_int32),
        ("n_gains", C.c_int32),
        ("n_targets", C.c_int32),
        ("scale", C.c_float),
        ("target_fill_u8", C.c_uint32),
        ("land_fill_u8", C.c_uint32),
        ("land_row0", C.c_int32),
        ("land_row1", C.c_int32),
        ("land_bin0", C.c_int32),
    ]


class StackParams(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32),
        ("files_per_frame", C.c_int32),
        ("rows", C.c_int32),
        ("bins", C.c_int32),
        ("echo_dtype", C.c_int32),
        ("threshold", C.c_float),
        ("stride", C.c_int32),
        ("land_filter", C.c_int32),
        ("land_resolution", C.c_double),
        ("land_persistence", C.c_double),
        ("land_min_intensity", C.c_double),
        ("eps_space", C.c_double),
        ("eps_time", C.c_double),
        ("min_samples", C.c_int32),
        ("timing", C.c_int32),
    ]


class StackResult(C.Structure):
    _fields_ = [
        ("n_points", C.c_int64),
        ("n_clustered", C.c_int64),
        ("n_land_cells", C.c_int64),
        ("n_segments", C.c_int64),
        ("n_built", C.c_int32),
        ("n_clusters", C.c_int32),
        ("ms_polar", C.c_double),
        ("ms_land", C.c_double),
        ("ms_stdbscan", C.c_double),
        ("ms_summaries", C.c_double),
        ("dbscan", StdbscanStats),
    ]


class ShardInfo(C.Structure):
    _fields_ = [
        ("n_points", C.c_int64),
        ("n_built", C.c_int32),
        ("halo_frames", C.c_int32),
        ("bounds", C.c_float * 4),
        ("n_head_k1", C.c_int64),
        ("n_tail_k1", C.c_int64),
        ("n_kept", C.c_int64),
        ("n_head", C.c_int64),
        ("n_tail", C.c_int64),
        ("n_prev", C.c_int64),
        ("n_next", C.c_int64),
        ("n_land_cells", C.c_int64),
    ]


# (name, restype, argtypes)
_SIGS = [
    ("rpt_version", C.c_int32, []),
    ("rpt_last_error", C.c_char_p, []),
    ("rpt_device_count", C.c_int32, []),
    ("rpt_set_device", C.c_int32, [C.c_int32]),
    ("rpt_release_scratch", None, []),
    ("rpt_exclusive_scan", C.c_int32, [vp, C.c_int32, C.c_int64, vp, C.c_int32, C.c_int32, vp]),
    ("rpt_polar_count", C.c_int32,
     [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_float, C.c_int32, vp, vp, c_i64p, vp]),
    ("rpt_polar_write", C.c_int32,
     [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp, vp, C.c_float, C.c_int32, vp,
      vp, C.c_int32, vp, vp, vp, vp, vp, vp]),
    ("rpt_polar_stage_words", C.c_int64, [C.c_int64, C.c_int32]),
    ("rpt_polar_count_staged", C.c_int32,
     [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_float, C.c_int32, vp, vp, c_i64p, vp,
      vp]),
    ("rpt_polar_write_staged", C.c_int32,
     [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp, vp, C.c_float, C.c_int32, vp,
      vp, C.c_int32, vp, vp, vp, vp, vp, vp, vp]),
    ("rpt_frame_times", C.c_int32, [vp, C.c_int64, vp, vp, vp]),
    ("rpt_sweep_to_points", C.c_int32,
     [vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_float, C.c_int32, vp, vp, vp, C.c_int64, c_i64p,
      vp]),
    ("rpt_polar_to_cartesian", C.c_int32, [vp, vp, vp, C.c_int64, C.c_int64, vp, vp, vp]),
    ("rpt_bounds_xy", C.c_int32, [vp, vp, C.c_int64, c_f32p, vp]),
    ("rpt_land_grid", C.c_int32,
     [vp, vp, vp, C.c_int64, vp, C.c_int32, vp, C.c_int32, vp, vp, vp]),
    ("rpt_land_mask", C.c_int32,
     [vp, vp, C.c_int64, C.c_int64, C.c_double, C.c_double, vp, c_i64p, vp]),
    ("rpt_land_filter", C.c_int32,
     [vp, vp, vp, vp, vp, C.c_int64, vp, C.c_int32, vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp,
      vp, vp, vp, c_i64p, vp]),
    ("rpt_stdbscan", C.c_int32,
     [vp, vp, vp, C.c_int64, vp, C.c_int64, C.c_double, C.c_double, C.c_int32, vp,
      C.POINTER(StdbscanStats), vp]),
    ("rpt_label_means", C.c_int32,
     [vp, vp, vp, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp]),
    ("rpt_stdbscan_denoise", C.c_int32,
     [vp, vp, vp, C.c_int64, C.c_double, C.c_double, C.c_int32, C.c_int32, vp,
      C.POINTER(StdbscanStats), vp]),
    ("rpt_infer_time_from_colors", C.c_int32, [vp, C.c_int64, vp, C.c_int32, vp, vp]),
    ("rpt_dbscan_create", vp, []),
    ("rpt_dbscan_destroy", None, [vp]),
    ("rpt_dbscan_build", C.c_int32,
     [vp, vp, vp, vp, C.c_int64, vp, C.c_int64, C.c_double, C.c_double, C.c_int32, vp]),
    ("rpt_dbscan_core", C.c_int32, [vp, vp, vp]),
    ("rpt_dbscan_set_core", C.c_int32, [vp, vp, vp]),
    ("rpt_dbscan_components", C.c_int32, [vp, vp, vp]),
    ("rpt_dbscan_labels_global", C.c_int32, [vp, vp, vp, C.c_int64, vp, vp]),
    ("rpt_remap_components", C.c_int32, [vp, C.c_int64, C.c_int64, vp, vp, C.c_int64, vp, vp]),
    ("rpt_select_roots", C.c_int32, [vp, C.c_int64, C.c_int64, C.c_int64, vp, c_i64p, vp]),
    ("rpt_cluster_summaries", C.c_int32,
     [vp, vp, vp, vp, vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, vp, vp,
      c_i64p, vp]),
    ("rpt_arange_edges", C.c_int32, [C.c_float, C.c_float, C.c_double, c_f64p, C.c_int32]),
    ("rpt_stack_create", vp, []),
    ("rpt_stack_destroy", None, [vp]),
    ("rpt_stack_run", C.c_int32, [vp, C.POINTER(StackParams), vp, vp, vp, vp, vp,
                                  C.POINTER(StackResult), vp]),
    ("rpt_stack_frame_offsets", C.c_int32, [vp, C.c_int32, c_i64p]),
    ("rpt_stack_segments", C.c_int32, [vp, c_i32p, c_i32p, c_i64p, c_i64p, c_f32p, c_f32p, c_f32p,
                                       c_i64p]),
    ("rpt_stack_points", C.c_int32, [vp, vp, vp, vp, vp, vp, vp, vp]),
    ("rpt_stack_core_flags", C.c_int32, [vp, vp, vp]),
    ("rpt_shard_create", vp, []),
    ("rpt_shard_destroy", None, [vp]),
    ("rpt_shard_polar", C.c_int32, [vp, C.POINTER(StackParams), vp, vp, vp, vp, vp,
                                    C.POINTER(ShardInfo), vp]),
    ("rpt_shard_land_cells", C.c_int64, [c_f32p, C.c_double]),
    ("rpt_shard_land_grid", C.c_int32, [vp, c_f32p, vp, C.c_int64, vp]),
    ("rpt_shard_halo", C.c_int32, [vp, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int64, vp, vp,
                                   C.c_int64, C.c_int64, vp]),
    ("rpt_shard_window", C.c_int32, [vp, vp, C.c_int64, vp, C.c_int64, vp, vp,
                                     C.POINTER(ShardInfo), vp]),
    ("rpt_shard_core_ms", C.c_double, [vp]),
    ("rpt_shard_link", C.c_int32, [vp, vp, vp, vp, vp, vp]),
    ("rpt_shard_pairs", C.c_int32, [vp, vp, vp, vp, C.c_int64, vp]),
    ("rpt_merge_equivalences", C.c_int64, [c_i64p, C.c_int64, c_i64p, c_i64p, C.c_int64]),
    ("rpt_shard_finish", C.c_int32, [vp, vp, C.c_int32, C.c_int64, vp, c_i64p, c_i64p,
                                     C.c_int64, C.c_int32, vp, C.c_int64, vp]),
    ("rpt_shard_labels", C.c_int32, [vp, vp, C.c_int64, vp, vp]),
    ("rpt_shard_frame_offsets", C.c_int32, [vp, C.c_int32, c_i64p]),
    ("rpt_shard_set_merge_limit", C.c_int32, [vp, C.c_int32]),
    ("rpt_shard_points", C.c_int32, [vp, vp, vp, vp, vp, vp, vp]),
    ("rpt_shard_gathered_sizes", C.c_int32, [c_i64p, C.c_int32, C.c_int64, c_i64p]),
    ("rpt_shard_host_stage", C.c_int32, [c_i64p, C.c_int32, C.c_int64, vp, c_i32p, c_i32p,
                                         c_i64p, c_i64p, c_f32p, c_f32p, c_f32p, c_i64p, c_i64p,
                                         c_i64p, c_i32p, C.c_int32]),
    ("rpt_order_clusters", C.c_int32, [C.c_int32, C.c_int64, c_i32p, c_i32p, c_i64p, c_i64p,
                                        c_i64p, c_i64p]),
    ("rpt_k1_gate_create", vp, []),
    ("rpt_k1_gate_destroy", None, [vp]),
    ("rpt_stack_set_k1_gate", C.c_int32, [vp, vp]),
    ("rpt_order_and_track", C.c_int32, [C.c_int32, C.c_int64, c_i32p, c_i32p, c_i64p, c_i64p,
                                         c_f32p, c_f32p, C.c_int32, c_i64p, c_i64p, vp, c_i64p,
                                         c_i64p]),
    ("rpt_set_order", C.c_int32, [c_i32p, C.c_int32, c_i32p]),
    ("rpt_lsap", C.c_int32, [c_f64p, C.c_int32, C.c_int32, c_i64p, c_i64p]),
    ("rpt_tracker_new", vp, [C.POINTER(TrackerParams)]),
    ("rpt_tracker_free", None, [vp]),
    ("rpt_tracker_update", C.c_int32, [vp, C.c_int64, C.c_int32, c_f32p, c_f32p, c_i64p]),
    ("rpt_tracker_run", C.c_int32, [vp, C.c_int32, c_i64p, c_i64p, c_f32p, c_f32p]),
    ("rpt_tracker_num_objects", C.c_int32, [vp]),
    ("rpt_tracker_object_info", C.c_int32, [vp, C.c_int32, C.POINTER(ObjectInfo)]),
    ("rpt_tracker_object_history", C.c_int32, [vp, C.c_int32, c_f32p, c_f32p, c_i64p, c_f64p,
                                                c_f64p]),
    ("rpt_fuse_gains_max", C.c_int32,
     [vp, vp, vp, C.c_int64, C.c_double, vp, vp, vp, c_i64p, vp]),
    ("rpt_csv_count_rows", C.c_int32, [C.POINTER(C.c_char_p), C.c_int32, c_i64p, C.c_int32]),
    ("rpt_csv_parse_sweeps", C.c_int32,
     [C.POINTER(C.c_char_p), C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, c_f32p, c_f32p,
      c_f32p, c_i32p, c_i64p, C.c_int32, C.c_int32]),
    ("rpt_synth_echo", C.c_int32,
     [C.POINTER(SynthParams), C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp]),
]

EXPORTED = [s[0] for s in _SIGS]

_lib = None


class RptError(RuntimeError):
    pass


def lib_path() -> Path:
    return Path(os.environ.get("RPT_LIB", str(_LIB_PATH)))


def load(require: bool = True):
    """Load librpt.so (cached).  Raises ImportError when it is missing: there is no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    p = lib_path()
    if not p.exists():
        if not require:
            return None
        raise ImportError(
            f"librpt.so not found at {p}; build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950). The rpt device path has no CPU fallback.")
    lib = C.CDLL(str(p))
    missing = []
    for name, res, args in _SIGS:
        fn = getattr(lib, name, None)
        if fn is None:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    lib.rpt_missing_symbols = missing  # tests/test_abi.py requires this to be empty
    _lib = lib
    return lib


def last_error() -> str:
    return load().rpt_last_error().decode("utf-8", "replace")


def check(status: int, what: str = "") -> None:
    if status == RPT_OK:
        return
    msg = last_error() or f"status {status}"
    if what:
        msg = f"{what}: {msg}"
    if status in (RPT_EINVAL, RPT_EEMPTY, RPT_ENONFINITE):
        raise ValueError(msg)
    if status == RPT_ENOTSUP:
        raise NotImplementedError(msg)
    if status == RPT_ENOMEM:
        raise MemoryError(msg)
    raise RptError(msg)
