#!/bin/bash
# Host tracker timing on the GPU box: dump an 800-frame stack's summaries, order them, time the
# C++ tracker through the C-ABI (tools/microbench/tracker_bench.cpp).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/dump_seg.py 800 > gpurun_out/trk_dump.log 2>&1 || exit $?
python tools/trk_dump.py gpurun_out/seg.npz /tmp/trk800.bin || exit $?
g++ -O2 -Iinclude tools/microbench/tracker_bench.cpp -Lradar-point-cloud-tracking_amd/rpt -lrpt \
  -Wl,-rpath,"$R/radar-point-cloud-tracking_amd/rpt" -o /tmp/tracker_bench || exit $?
/tmp/tracker_bench /tmp/trk800.bin 50 | tee gpurun_out/tracker_bench.json
