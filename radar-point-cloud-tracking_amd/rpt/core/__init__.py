"""Drop-in for ``radar_pipeline.core`` (hot-path members only)."""
