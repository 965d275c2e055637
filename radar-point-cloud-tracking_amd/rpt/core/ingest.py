"""Radar CSV sweeps -> echo batches through librpt's native parser (rpt_csv_count_rows /
rpt_csv_parse_sweeps, csrc/csv.cpp): the file half of load_radar_csv
(PointCloudWork/4_temporal_object_tracker.py:189-211, radar_pipeline/core/loaders.py:46-101)
without pandas, multithreaded, written straight into the [file][row][bin] layout the device
stack takes (u8 when every echo value is an integer in 0..255, else float32).

Where read_csv raises, ``SweepBatch.errors`` holds the text of its exception (the reference
prints ``Error loading {path}: {e}``, 4_temporal_object_tracker.py:193-194): the I/O error of an
unreadable file (``[Errno 13] Permission denied: '<path>'``) or the C tokenizer's
``Error tokenizing data. C error: Expected E fields in line L, saw S`` + newline.  Not reproduced:
quoted fields, comment characters and read_csv's UnicodeDecodeError on non-UTF-8 bytes (such a
byte is a non-numeric value here: ValueError)."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional, Sequence, Union

import numpy as np

from .. import _abi

STATUS_OK, STATUS_UNREADABLE, STATUS_EMPTY, STATUS_NOT_U8, STATUS_NON_NUMERIC = 0, 1, 2, 3, 4
STATUS_UNSUPPORTED = 6          # mode "genfromtxt": a field count other than 5 + bins
MODE_READ_CSV, MODE_GENFROMTXT = 0, 1
GAIN_FIRST_NAN, GAIN_DISAGREE = 1, 2   # SweepBatch.gain_flags bits


@dataclass
class SweepBatch:
    echo: np.ndarray     # [n_files][rows][bins] uint8 or float32 (rows past a file's end: 0)
    scale: np.ndarray    # float32 [n_files][rows]
    angle: np.ndarray    # float32 [n_files][rows] (Angle column, radar units)
    gain: np.ndarray     # float32 [n_files]: the file's Gain value (NaN if rows disagree)
    rows: np.ndarray     # int64 [n_files]: data rows per file (-1 unreadable)
    status: np.ndarray   # int32 [n_files]: STATUS_*
    errors: List[Optional[str]]  # the loader's exception text where it raises, else None
    gain_flags: np.ndarray       # int64 [n_files]: GAIN_FIRST_NAN | GAIN_DISAGREE bits
    detail_kind: np.ndarray      # int64 [n_files]: 0 none, 1 I/O, 2 tokenizer, 3 non-numeric,
                                 # 5 genfromtxt rows of < 5 fields (rpt_csv_parse_sweeps)
    n_fields: Optional[np.ndarray] = None  # int64 [n_files]: fields per row of the files
                                           # with STATUS_UNSUPPORTED (0 for the others)


def read_csv_error(path, detail) -> Optional[str]:
    """str(e) of the exception the reference's loader raises for this file (None when it does
    not): read_csv's I/O and tokenizer errors, to_numpy(float32)'s non-numeric value, the
    genfromtxt array's data[:, 4] IndexError."""
    kind = int(detail[0])
    if kind == 1:
        err = int(detail[1])
        return f"[Errno {err}] {os.strerror(err)}: {str(path)!r}"
    if kind == 2:
        return (f"Error tokenizing data. C error: Expected {int(detail[1])} fields in line "
                f"{int(detail[2])}, saw {int(detail[3])}\n")
    if kind == 3:
        tok = _field(path, int(detail[2]), int(detail[1]))
        return f"could not convert string to float: {tok!r}"
    if kind == 5:
        return f"index 4 is out of bounds for axis 1 with size {int(detail[1])}"
    return None


def _field(path, line: int, col: int) -> str:
    """Field col of physical line `line` (1-based) as pandas' C tokenizer holds it."""
    with open(path, "rb") as fh:
        for k, raw in enumerate(fh, 1):
            if k == line:
                text = raw.decode("utf-8", "replace").rstrip("\n").rstrip("\r")
                parts = text.split(",")
                return parts[col] if col < len(parts) else ""
    return ""


def _paths(paths: Sequence[Union[str, Path]]):
    enc = [str(p).encode() for p in paths]
    arr = (C.c_char_p * max(len(enc), 1))(*enc)
    return arr, enc


def read_sweeps(paths: Sequence[Union[str, Path]], bins: int = 1024, threads: int = 0,
                out_echo: np.ndarray = None, mode: int = MODE_READ_CSV) -> SweepBatch:
    """Parse radar CSVs.  out_echo (optional): a preallocated (e.g. pinned) uint8 buffer of at
    least n_files*rows*bins bytes, used when every file holds u8 samples.  mode: MODE_READ_CSV
    (pd.read_csv, the tracker's loader) or MODE_GENFROMTXT (np.genfromtxt first, read_csv when
    it raises: the denoise loader)."""
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
    detail = np.zeros((max(n, 1), 5), np.int64)

    def parse(dtype, code, buf=None):
        if buf is None:
            echo = np.empty((n, cap, bins), dtype)
        else:
            echo = buf.reshape(-1)[:n * cap * bins].view(dtype).reshape(n, cap, bins)
        _abi.check(lib.rpt_csv_parse_sweeps(
            arr, n, cap, bins, code, echo.ctypes.data, scale.ctypes.data_as(_abi.c_f32p),
            angle.ctypes.data_as(_abi.c_f32p), gain.ctypes.data_as(_abi.c_f32p),
            status.ctypes.data_as(_abi.c_i32p), detail.ctypes.data_as(_abi.c_i64p), int(mode),
            threads),
            "rpt_csv_parse_sweeps")
        return echo

    echo = parse(np.uint8, _abi.ECHO_U8, out_echo)
    if (status[:n] == STATUS_NOT_U8).any():   # non-integer or out-of-range samples: float32
        echo = parse(np.float32, _abi.ECHO_F32)
    return SweepBatch(echo=echo, scale=scale, angle=angle, gain=gain[:n], rows=rows,
                      status=status[:n].copy(),
                      errors=[read_csv_error(p, detail[i]) for i, p in enumerate(paths)],
                      gain_flags=detail[:n, 4].copy(), detail_kind=detail[:n, 0].copy(),
                      n_fields=np.where(status[:n] == STATUS_UNSUPPORTED, detail[:n, 1], 0))
