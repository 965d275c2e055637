"""rpt — MI355X-native (gfx950) ST-DBSCAN clustering and multi-object tracking for marine-radar
point clouds.  Drop-in for the ``radar_pipeline`` package API and the
``3_stdbscan_point_clouds.py`` / ``4_temporal_object_tracker.py`` scripts of the reference.

Numerics run in hand-written HIP kernels behind the C-ABI of ``librpt.so`` (include/rpt.h);
PyTorch-ROCm only provides device memory, streams and torch.distributed.
"""
__version__ = "0.1.0"

from . import config  # noqa: F401
