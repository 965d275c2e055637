"""Radar CSV sweeps -> echo batches through librpt's native parser (rpt_csv_count_rows /
rpt_csv_parse_sweeps, csrc/csv.cpp): the file half of load_radar_csv
(PointCloudWork/4_temporal_object_tracker.py:189-211, radar_pipeline/core/loaders.py:46-101)
without pandas, multithreaded, written straight into the [file][row][bin] layout the device
stack takes (u8 when every echo value is an integer in 0..255, else float32)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path
from typing import List, Sequence, Union

import numpy as np

from .. import _abi

STATUS_OK, STATUS_UNREADABLE, STATUS_EMPTY, STATUS_NOT_U8, STATUS_NON_NUMERIC = 0, 1, 2, 3, 4


@dataclass
class SweepBatch:
    echo: np.ndarray     # [n_files][rows][bins] uint8 or float32 (rows past a file's end: 0)
    scale: np.ndarray    # float32 [n_files][rows]
    angle: np.ndarray    # float32 [n_files][rows] (Angle column, radar units)
    gain: np.ndarray     # float32 [n_files]: the file's Gain value (NaN if rows disagree)
    rows: np.ndarray     # int64 [n_files]: data rows per file (-1 unreadable)
    status: np.ndarray   # int32 [n_files]: STATUS_*


def _paths(paths: Sequence[Union[str, Path]]):
    enc = [str(p).encode() for p in paths]
    arr = (C.c_char_p * max(len(enc), 1))(*enc)
    return arr, enc


def read_sweeps(paths: Sequence[Union[str, Path]], bins: int = 1024, threads: int = 0,
                out_echo: np.ndarray = None) -> SweepBatch:
    """Parse radar CSVs.  out_echo (optional): a preallocated (e.g. pinned) uint8 buffer of at
    least n_files*rows*bins bytes, used when every file holds u8 samples."""
    lib = _abi.load()
    n = len(paths)
    arr, _keep = _paths(paths)
    rows = np.zeros(max(n, 1), np.int64)
    _abi.check(lib.rpt_csv_count_rows(arr, n, rows.ctypes.data_as(_abi.c_i64p), threads),
               "rpt_csv_count_rows")
    rows = rows[:n]
    cap = int(max(rows.max(initial=0), 0))
    status = np.zeros(max(n, 1), np.int32)
    scale = np.zeros((n, cap), np.float32)
    angle = np.zeros((n, cap), np.float32)
    gain = np.zeros(max(n, 1), np.float32)

    def parse(dtype, code, buf=None):
        if buf is None:
            echo = np.empty((n, cap, bins), dtype)
        else:
            echo = buf.reshape(-1)[:n * cap * bins].view(dtype).reshape(n, cap, bins)
        _abi.check(lib.rpt_csv_parse_sweeps(
            arr, n, cap, bins, code, echo.ctypes.data, scale.ctypes.data_as(_abi.c_f32p),
            angle.ctypes.data_as(_abi.c_f32p), gain.ctypes.data_as(_abi.c_f32p),
            status.ctypes.data_as(_abi.c_i32p), threads), "rpt_csv_parse_sweeps")
        return echo

    echo = parse(np.uint8, _abi.ECHO_U8, out_echo)
    if (status[:n] == STATUS_NOT_U8).any():   # non-integer or out-of-range samples: float32
        echo = parse(np.float32, _abi.ECHO_F32)
    return SweepBatch(echo=echo, scale=scale, angle=angle, gain=gain[:n], rows=rows,
                      status=status[:n].copy())
