"""Drop-in for ``radar_pipeline.processors`` (hot-path members only)."""
from .clustering import (  # noqa: F401
    cluster_point_cloud,
    infer_time_from_colors,
    process_ply_clustering,
    st_dbscan,
)
