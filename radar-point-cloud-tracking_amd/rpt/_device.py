"""Device plumbing: torch-ROCm tensors as HBM buffers, the current HIP stream as the ABI stream.

PyTorch is used only for allocation, host<->device copies, streams and torch.distributed; all
arithmetic of the hot path runs in librpt's HIP kernels.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _abi


def require_gpu(device: int | torch.device | None = None) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "rpt requires a ROCm GPU (torch.cuda.is_available() is False); "
            "there is no CPU fallback for the device path")
    _abi.load()
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device) if not isinstance(device, torch.device) else device
    if d.type != "cuda":
        raise ValueError(f"rpt device path needs a cuda (HIP) device, got {d}")
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def to_device(a, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """numpy array or tensor -> contiguous tensor of `dtype` on `device` (no copy if already)."""
    if isinstance(a, torch.Tensor):
        t = a
        if t.dtype != dtype:
            t = t.to(dtype)
        if t.device != device:
            t = t.to(device, non_blocking=False)
        return t.contiguous()
    arr = np.ascontiguousarray(a)
    t = torch.from_numpy(arr)
    if t.dtype != dtype:
        t = t.to(dtype)
    return t.to(device)


def is_torch(a) -> bool:
    return isinstance(a, torch.Tensor)
