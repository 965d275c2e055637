"""Native radar-CSV ingest (csrc/csv.cpp) against pandas' read_csv
exactly as load_radar_csv calls it (PointCloudWork/4_temporal_object_tracker.py:189-211):
values, NaN handling, the empty / error outcomes, u8 vs float32 selection.  CPU only."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pandas as pd
import pytest

from rpt.core.ingest import (STATUS_EMPTY, STATUS_NON_NUMERIC, STATUS_OK, STATUS_UNREADABLE,
                             read_sweeps)

B = 16
COLS = ["Status", "Scale", "Range", "Gain", "Angle"] + [f"Echo_{i}" for i in range(B)]
HDR = ",".join(COLS) + "\n"


def _pandas(path, bins=B):
    """The reference's read (:191-211): pandas C parser, fillna(0), float32."""
    cols = ["Status", "Scale", "Range", "Gain", "Angle"] + [f"Echo_{i}" for i in range(bins)]
    try:
        df = pd.read_csv(path, header=None, names=cols, skiprows=1, engine="c")
    except Exception:
        return "error", None
    if df.empty:
        return "empty", None
    try:
        return "ok", (df.iloc[:, 5:].fillna(0).to_numpy(np.float32),
                      df["Scale"].to_numpy(np.float32), df["Angle"].to_numpy(np.float32))
    except (ValueError, TypeError):
        return "nonnum", None


def _row(vals, scale="231.5", angle="5", gain="40"):
    return f"1,{scale},0,{gain},{angle}," + ",".join(str(v) for v in vals)


CASES = {
    "plain": HDR + "\n".join(_row(range(k, k + B)) for k in range(5)) + "\n",
    "blank_and_ws_lines": HDR + _row([3] * B) + "\n\n   \n" + _row([11] * B) + "\n",
    "crlf": (HDR + _row([12] * B) + "\n" + _row([9] * B) + "\n").replace("\n", "\r\n"),
    "spaces_in_fields": HDR + "1, 231.5 ,0,40, 7 , 12 ," + ",".join(["3"] * (B - 1)) + "\n",
    "short_rows": HDR + _row([50] * 3) + "\n" + "1,100.0,0,40\n" + _row([20] * B) + "\n",
    "first_row_extra_fields_is_index": HDR + _row([1] * (B + 1)) + "\n" + _row([2] * B) + "\n",
    "later_row_too_many_fields": HDR + _row([1] * B) + "\n" + _row([2] * (B + 1)) + "\n",
    "trailing_comma_every_row": HDR + "\n".join(_row([k] * B) + "," for k in range(3)) + "\n",
    "header_only": HDR,
    "header_no_newline": HDR.strip(),
    "empty_file": "",
    "nan_spellings": HDR + _row(["nan", "NA", "", "NaN", "null"] + [30] * (B - 5)) + "\n" +
    _row([40] * B, scale="nan", angle="") + "\n",
    "decimals": HDR + _row([12.5, 0.25, 255.0, 256, -3] + [1] * (B - 5), scale="115.75",
                           angle="8195") + "\n",
    "scientific": HDR + _row(["1e1", "2.5E1", "+7", "-0"] + [0] * (B - 4), scale="2.315e2") + "\n",
    "hex_is_not_a_number": HDR + _row([1] * B, scale="0x10") + "\n",
    "text_value": HDR + _row(["abc"] + [1] * (B - 1)) + "\n",
    "no_trailing_newline": HDR + _row([77] * B),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_native_csv_matches_pandas(tmp_path, name):
    p = tmp_path / f"{name}.csv"
    p.write_text(CASES[name])
    kind, ref = _pandas(p)
    b = read_sweeps([p], bins=B)
    st = int(b.status[0])
    if kind == "ok":
        e, sc, an = ref
        R = e.shape[0]
        assert st == STATUS_OK and b.rows[0] == R
        np.testing.assert_array_equal(b.echo[0, :R].astype(np.float32), e)
        np.testing.assert_array_equal(b.scale[0, :R], sc)
        np.testing.assert_array_equal(b.angle[0, :R], an)
        assert b.echo.dtype == (np.uint8 if np.array_equal(e, np.clip(np.round(e), 0, 255))
                                else np.float32)
    elif kind == "empty":
        assert st == STATUS_EMPTY
    elif kind == "error":
        assert st in (STATUS_UNREADABLE, STATUS_EMPTY)  # both give the reference an empty sweep
    else:
        assert st == STATUS_NON_NUMERIC


def test_missing_file_is_unreadable(tmp_path):
    b = read_sweeps([tmp_path / "nope.csv"], bins=B)
    assert b.rows[0] == -1 and int(b.status[0]) == STATUS_UNREADABLE


def test_batch_of_full_sweeps_matches_pandas(tmp_path):
    """Full 4096 x 1029 radar files (the reference's format), several at once, different row
    counts: zero padding past each file's end, u8 layout, threads."""
    rng = np.random.default_rng(9)
    paths, refs = [], []
    for k, rows in enumerate((4096, 4000, 4096, 1)):
        echo = np.where(rng.random((rows, 1024)) < 0.1, rng.integers(0, 256, (rows, 1024)), 0)
        angle = np.sort(rng.choice(8196, rows, replace=False))
        scale = rng.choice([231.5, 463.0, 115.75], rows)
        lines = [",".join(["Status", "Scale", "Range", "Gain", "Angle"] +
                          [f"Echo_{i}" for i in range(1024)])]
        for r in range(rows):
            lines.append(f"1,{scale[r]:g},0,{40 + k},{angle[r]}," + ",".join(map(str, echo[r])))
        p = tmp_path / f"f{k}.csv"
        p.write_text("\n".join(lines) + "\n")
        paths.append(p)
        refs.append(_pandas(p, bins=1024)[1])
    b = read_sweeps(paths, bins=1024, threads=3)
    assert b.echo.dtype == np.uint8 and b.echo.shape == (4, 4096, 1024)
    for k, (e, sc, an) in enumerate(refs):
        R = e.shape[0]
        np.testing.assert_array_equal(b.echo[k, :R].astype(np.float32), e)
        assert not b.echo[k, R:].any()
        np.testing.assert_array_equal(b.scale[k, :R], sc)
        np.testing.assert_array_equal(b.angle[k, :R], an)
        assert b.gain[k] == 40 + k


def test_package_load_radar_csv_matches_reference(tmp_path, golden):
    """rpt.core.loaders.load_radar_csv (native parser) against radar_pipeline's load_radar_csv
    output recorded in g1 (angles_rad, ranges) on the same CSV content."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    from make_golden import write_csv

    from rpt.core.loaders import load_radar_csv

    g = golden("g1_polar.npz")
    for k in range(3):
        p = tmp_path / f"f{k}.csv"
        write_csv(p, 1, g[f"f{k}_scale"].astype(np.float64), 0, int(g[f"f{k}_gain"]),
                  g[f"f{k}_angle"].astype(np.int64), g[f"f{k}_echo"].astype(np.int64))
        sw = load_radar_csv(p)
        np.testing.assert_array_equal(sw.angles_rad, g[f"f{k}_pkg_angles"])
        np.testing.assert_array_equal(sw.ranges, g[f"f{k}_pkg_ranges"])
        np.testing.assert_array_equal(sw.intensities, g[f"f{k}_echo"].astype(np.float32))
        assert sw.gain == int(g[f"f{k}_gain"])
    e = tmp_path / "empty.csv"
    e.write_text(HDR)
    with pytest.raises(ValueError):
        load_radar_csv(e)


def test_discover_and_group_frames(tmp_path):
    """discover_files (:235-267) + group_files_by_frame (:270-309): gain-dir regex, unsupported
    gains and unparsable names skipped, 2000 ms runs from each run's first file, first file per
    gain wins inside a run."""
    from rpt.core.discovery import discover_files, group_files_by_frame, parse_timestamp

    def touch(d, name):
        (tmp_path / d).mkdir(exist_ok=True)
        (tmp_path / d / name).write_text("x\n")

    touch("gain_40", "20250813_142600_000.csv")
    touch("gain_40", "20250813_142601_900.csv")   # same run as :00.000 (1900 ms): dropped
    touch("gain_40", "20250813_142603_000.csv")
    touch("Gain-50", "20250813_142600_500.csv")
    touch("Gain-50", "20250813_142602_100.csv")   # 2100 ms after the run start: new run
    touch("gain75", "20250813_142603_400.csv")
    touch("gain75", "notes.csv")                   # unparsable name
    touch("gain_60", "20250813_142600_000.csv")    # unsupported gain
    touch("other", "20250813_142600_000.csv")      # not a gain dir
    fb = discover_files(tmp_path)
    assert sorted(fb) == [40, 50, 75]
    assert [p.name for p in fb[40]] == ["20250813_142600_000.csv", "20250813_142601_900.csv",
                                        "20250813_142603_000.csv"]
    frames = group_files_by_frame(fb)
    got = [{g: p.name for g, p in f.items()} for f in frames]
    assert got == [{40: "20250813_142600_000.csv", 50: "20250813_142600_500.csv"},
                   {50: "20250813_142602_100.csv", 40: "20250813_142603_000.csv",
                    75: "20250813_142603_400.csv"}]
    assert parse_timestamp("20250813_142602_181.csv")[1] % 1000 == 181
    with pytest.raises(ValueError):
        parse_timestamp("x.csv")


# ------------------------------------------------------------ exception texts (stdout parity)
def _pandas_error_text(path, bins=B):
    """str(e) of what the reference's read (:191-198, + to_numpy :203-207) raises, else None."""
    cols = ["Status", "Scale", "Range", "Gain", "Angle"] + [f"Echo_{i}" for i in range(bins)]
    try:
        df = pd.read_csv(path, header=None, names=cols, skiprows=1, engine="c")
    except Exception as e:  # the reference prints f"Error loading {path}: {e}"
        return str(e)
    try:
        df.to_numpy(dtype=np.float32)
    except ValueError as e:
        return str(e)
    return None


ERROR_CASES = {
    "later_row_too_many_fields": CASES["later_row_too_many_fields"],
    "too_many_after_blank_lines": HDR + _row([1] * B) + "\n\n\n" + _row([2] * (B + 3)) + "\n",
    "index_then_too_many": HDR + _row([1] * (B + 1)) + "\n" + _row([2] * (B + 2)) + "\n",
    "crlf_too_many": CASES["later_row_too_many_fields"].replace("\n", "\r\n"),
    "text_value": CASES["text_value"],
    "text_in_two_columns": HDR + _row([1] * B) + "\n" + _row(["zz"] + [1] * (B - 1)) + "\n" +
    _row([1, "yy"] + [1] * (B - 2)) + "\n" + _row(["xx"] * B) + "\n",
    "text_with_space": HDR + _row([1, " ab c"] + [1] * (B - 2)) + "\n",
}


@pytest.mark.parametrize("name", sorted(ERROR_CASES))
def test_error_text_matches_pandas(tmp_path, name):
    """The "Error loading {path}: {e}" text (:194) and the non-numeric ValueError text: the
    tokenizer's expected fields, physical line and fields seen; the leftmost bad column's first
    bad value as numpy's column-block conversion names it."""
    p = tmp_path / f"{name}.csv"
    p.write_text(ERROR_CASES[name])
    exp = _pandas_error_text(p)
    assert exp is not None
    b = read_sweeps([p], bins=B)
    assert b.errors[0] == exp


def test_missing_file_error_text(tmp_path):
    p = tmp_path / "nope.csv"
    with pytest.raises(FileNotFoundError) as ei:
        pd.read_csv(p, header=None, names=COLS, skiprows=1, engine="c")
    assert read_sweeps([p], bins=B).errors[0] == str(ei.value)


def test_gain_first_row_and_unique(tmp_path):
    """int(df["Gain"].iloc[0]) (:200) and radar_pipeline's unique() rule (loaders.py:88-92):
    all-NaN raises like int(nan), rows that disagree give None, one value gives it."""
    from rpt.core.ingest import GAIN_DISAGREE, GAIN_FIRST_NAN
    from rpt.core.loaders import load_radar_csv

    files = {"same": [40, 40, 40], "mixed": [40, 50, 40], "first_nan": ["", 40, 40],
             "all_nan": ["", "nan", ""], "later_nan": [40, "", 40]}
    for name, gains in files.items():
        p = tmp_path / f"{name}.csv"
        p.write_text(HDR + "".join(_row([20] * B, gain=g) + "\n" for g in gains))
        b = read_sweeps([p], bins=B)
        df = pd.read_csv(p, header=None, names=COLS, skiprows=1, engine="c")
        u = df["Gain"].unique()
        assert bool(b.gain_flags[0] & GAIN_FIRST_NAN) == bool(np.isnan(df["Gain"].iloc[0]))
        assert bool(b.gain_flags[0] & GAIN_DISAGREE) == (len(u) > 1), name
        if len(u) == 1 and np.isnan(u[0]):
            with pytest.raises(ValueError):
                load_radar_csv(p, _cfg16())
        else:
            assert load_radar_csv(p, _cfg16()).gain == (int(u[0]) if len(u) == 1 else None)


def _cfg16():
    from rpt.config import RadarConfig

    return RadarConfig(num_echo_columns=B)


# ----------------------------------------------------- the denoise loader (genfromtxt first)
def _genfromtxt_ref(path, bins=B):
    """PointCloudWorkF/stdbscan_denoising_pipeline.py:104-120: genfromtxt, pandas fallback,
    the ndim/size check.  Returns ("raise", text) | ("empty", None) | ("ok", (echo, scale,
    angle))."""
    import warnings

    cols = ["Status", "Scale", "Range", "Gain", "Angle"] + [f"Echo_{i}" for i in range(bins)]
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            data = np.genfromtxt(path, delimiter=",", skip_header=1, dtype=np.float32,
                                 filling_values=0.0)
    except Exception:
        try:
            df = pd.read_csv(path, header=None, names=cols, skiprows=1, engine="c")
            if df.empty:
                return "empty", None
            data = df.to_numpy(dtype=np.float32)
        except Exception as e:
            return "raise", str(e)
    if data.size == 0 or data.ndim != 2:
        return "empty", None
    try:
        return "ok", (data[:, 5:], data[:, 1], data[:, 4])
    except IndexError as e:
        return "raise", str(e)


GF_CASES = {
    "plain": CASES["plain"],
    "single_row": HDR + _row(list(range(20, 20 + B))) + "\n",
    "header_only": HDR,
    "empty_file": "",
    "hash_comment": HDR + _row([30] * B) + "\n" + _row([12, "13#"] + [99] * (B - 2)) + "\n" +
    _row([31] * B) + "\n# a comment line\n",
    "empty_fields_fill_zero": HDR + _row([""] * 3 + [44] * (B - 3), scale="", angle="") + "\n" +
    _row([45] * B) + "\n",
    "nan_inf_text": HDR + _row(["nan", "inf", "NA", "abc", "1_0", " 12 "] + [50] * (B - 6)) +
    "\n" + _row([51] * B, scale="nan") + "\n",
    "ragged_rows_pandas_fallback": HDR + _row([60] * B) + "\n" + _row([61] * (B - 4)) + "\n",
    "ragged_one_row_fallback_keeps_it": HDR + _row([62] * B) + "\n" + "1,2\n",
    "ragged_and_too_many": HDR + _row([1] * B) + "\n" + _row([2] * (B - 1)) + "\n" +
    _row([3] * (B + 2)) + "\n",
    "ragged_text": HDR + _row([1] * B) + "\n" + _row(["q"] * (B - 1)) + "\n",
    "crlf": CASES["crlf"],
    "four_columns": HDR + "1,2,3,4\n1,2,3,4\n",
}


@pytest.mark.parametrize("name", sorted(GF_CASES))
def test_genfromtxt_mode_matches_denoise_loader(tmp_path, name):
    from rpt.core.ingest import MODE_GENFROMTXT

    p = tmp_path / f"{name}.csv"
    p.write_text(GF_CASES[name])
    kind, ref = _genfromtxt_ref(p)
    b = read_sweeps([p], bins=B, mode=MODE_GENFROMTXT)
    st = int(b.status[0])
    if kind == "ok":
        e, sc, an = ref
        R = e.shape[0]
        assert st == STATUS_OK
        got = b.echo[0, :R].astype(np.float32)
        # the echo only matters through `> 10` and its value where kept; NaN (pandas fallback
        # without fillna) and 0 keep nothing alike
        np.testing.assert_array_equal(np.nan_to_num(got, nan=0.0), np.nan_to_num(e, nan=0.0))
        np.testing.assert_array_equal(b.scale[0, :R], sc)
        np.testing.assert_array_equal(b.angle[0, :R], an)
        assert not b.echo[0, R:].any()
    elif kind == "empty":
        assert st == STATUS_EMPTY
    else:
        assert b.errors[0] == ref
