"""The device exclusive scan under every compaction of the path (K1 offsets, land filter, grid
build, summaries), through rpt_exclusive_scan: exact against numpy cumsum at tile boundaries of
both kernel sizes, in place, with and without the grand total, and across an epoch wrap of the
persistent look-back state (65535 launches)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

I32, I64 = 0, 1


def _scan(lib, dev, a, in_dt, out_dt, total, inplace=False):
    from rpt import _abi
    from rpt._device import stream_handle

    t_in = torch.from_numpy(a).to(dev)
    n = len(a)
    if inplace:
        buf = torch.zeros(n + (1 if total else 0), dtype=t_in.dtype, device=dev)
        buf[:n] = t_in
        t_in, out = buf, buf
    else:
        out = torch.full((n + (1 if total else 0),), -7,
                         dtype=torch.int32 if out_dt == I32 else torch.int64, device=dev)
    _abi.check(lib.rpt_exclusive_scan(t_in.data_ptr(), in_dt, n, out.data_ptr(), out_dt,
                                      1 if total else 0, stream_handle(dev)))
    return out.cpu().numpy()


def _expect(a, total):
    c = np.concatenate([[0], np.cumsum(a.astype(np.int64))])
    return c if total else c[:-1]


SIZES = [0, 1, 2, 2047, 2048, 2049, 4095, 4096, 4097, 3 * 4096 + 5, 1 << 20, (1 << 20) + 1,
         16384 * 70 - 1, 16384 * 70, 16384 * 70 + 1, 5_000_003]


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dts", [(I32, I32), (I32, I64), (I64, I64)])
def test_exclusive_scan_matches_cumsum(gpu, n, dts):
    from rpt import _abi

    lib = _abi.load()
    rng = np.random.default_rng(n + 7 * dts[1])
    a = rng.integers(0, 200, n).astype(np.int32 if dts[0] == I32 else np.int64)
    for total in (False, True):
        got = _scan(lib, gpu, a, *dts, total)
        np.testing.assert_array_equal(got.astype(np.int64), _expect(a, total))
    if dts[0] == dts[1]:
        got = _scan(lib, gpu, a, *dts, True, inplace=True)
        np.testing.assert_array_equal(got.astype(np.int64), _expect(a, True))


@pytest.mark.parametrize("n", [5000, 300_001])
def test_exclusive_scan_unaligned(gpu, n):
    """Pointers off the 16-B grid take the scalar-access kernel."""
    from rpt import _abi
    from rpt._device import stream_handle

    lib = _abi.load()
    rng = np.random.default_rng(n)
    a = rng.integers(0, 100, n).astype(np.int32)
    t_in = torch.zeros(n + 1, dtype=torch.int32, device=gpu)
    t_in[1:] = torch.from_numpy(a).to(gpu)
    out = torch.zeros(n + 3, dtype=torch.int64, device=gpu)
    _abi.check(lib.rpt_exclusive_scan(t_in[1:].data_ptr(), I32, n, out[1:].data_ptr(), I64, 1,
                                      stream_handle(gpu)))
    np.testing.assert_array_equal(out[1:n + 2].cpu().numpy(), _expect(a, True))


def test_exclusive_scan_large_values_i64(gpu):
    """Running totals far beyond 32 bits (up to 2^45) survive the 46-bit status granules."""
    from rpt import _abi

    lib = _abi.load()
    rng = np.random.default_rng(3)
    n = 3_000_001
    a = rng.integers(0, 1 << 23, n).astype(np.int64)
    assert a.sum() < (1 << 46)
    got = _scan(lib, gpu, a, I64, I64, True)
    np.testing.assert_array_equal(got, _expect(a, True))


def test_release_scratch_between_scans(gpu):
    """rpt_release_scratch frees the device's scratch and look-back state; the next scans
    re-create them (zeroed) and stay exact."""
    from rpt import _abi

    lib = _abi.load()
    rng = np.random.default_rng(21)
    a = rng.integers(0, 9, 300_000).astype(np.int32)
    for _ in range(3):
        np.testing.assert_array_equal(_scan(lib, gpu, a, I32, I64, True), _expect(a, True))
        torch.cuda.synchronize(gpu)
        lib.rpt_release_scratch()


def test_exclusive_scan_epoch_wrap(gpu):
    """70000 consecutive multi-tile scans on one stream (the epoch tag wraps at 65535 and the
    state is cleared then): every 5000th result and the last one stay exact."""
    from rpt import _abi
    from rpt._device import stream_handle

    lib = _abi.load()
    st = stream_handle(gpu)
    n = 9000  # three tiles of the 256-thread kernel
    rng = np.random.default_rng(11)
    a = rng.integers(0, 50, n).astype(np.int32)
    exp = _expect(a, True)
    t_in = torch.from_numpy(a).to(gpu)
    out = torch.empty(n + 1, dtype=torch.int64, device=gpu)
    for i in range(70000):
        out.fill_(-1) if i % 5000 == 0 else None
        _abi.check(lib.rpt_exclusive_scan(t_in.data_ptr(), I32, n, out.data_ptr(), I64, 1, st))
        if i % 5000 == 4999 or i == 69999:
            np.testing.assert_array_equal(out.cpu().numpy(), exp)
