"""Command-line drop-ins: ``rpt.cli.tracker`` (PointCloudWork/4_temporal_object_tracker.py),
``rpt.cli.stdbscan_ply`` (PointCloudWork/3_stdbscan_point_clouds.py), ``rpt.cli.denoise``
(PointCloudWorkF/stdbscan_denoising_pipeline.py) and ``rpt.cli.main`` (the ``radar-pipeline``
click group's ``cluster`` command)."""
