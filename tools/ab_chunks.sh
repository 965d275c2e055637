#!/bin/bash
# Slab-bucket chunking check: ST-DBSCAN parity suites, then the bench at 1000 / 125 standard
# frames and the dense configs[4] share with the default rule vs RPT_SLAB_CHUNKS=1 (one block per
# slab).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
# RPT_* switches are read only by the A/B build (python -m rpt._build --ab, built on the CPU host)
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so"
[ -f "$RPT_LIB" ] || { echo "build librpt_ab.so first: (cd radar-point-cloud-tracking_amd && python -m rpt._build --ab)"; exit 1; }
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_stdbscan_gpu.py tests/test_path_gpu.py \
  tests/test_fullsize_gpu.py tests/test_dist_gpu.py tests/test_denoise_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_sel.log 2>&1 || { tail -30 gpurun_out/gpu_sel.log; exit 1; }
tail -1 gpurun_out/gpu_sel.log
for args in "--total-frames 1000" "--total-frames 125" "--dense --total-frames 125"; do
  for v in 0 1; do
    RPT_SLAB_CHUNKS=$v timeout -k 10 300 python bench.py $args --steps 10 --warmup 2 \
      --no-cpu-baseline --h2d-steps 0 --no-dense-k5 > gpurun_out/ch.json 2> gpurun_out/ch.err || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/ch.json').read().strip().splitlines()[-1]);print('$args chunks_override=$v', d['value'], d['one_stack_in_flight']['ms_per_step'], d['stage_ms']['dbscan_grid'])"
  done
done
