#!/bin/bash
# Round-end style check on one GPU box: smoke, the whole -m gpu suite, the default bench (with
# the CPU baseline and the H2D leg), a 125-frame bench, then a 1000-frame kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --total-frames 125 --no-cpu-baseline --h2d-steps 0 > gpurun_out/bench_125.json 2> gpurun_out/bench_125.err || exit 1
bash tools/kprof.sh r2e --total-frames 1000 || exit 1
python tools/kstats.py $(find gpurun_out/kprof_r2e -name "*kernel_stats.csv") 4 > gpurun_out/ks_r2e.txt
head -20 gpurun_out/ks_r2e.txt
