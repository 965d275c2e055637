#!/bin/bash
# K9 check on the GPU box: the summaries parity tests, then one-stack kernel traces of the K9
# kernels at 1000 / 125 standard and 125 dense frames.   bash tools/k9_check.sh
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_path_gpu.py tests/test_bigstack_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/k9_tests.log 2>&1 || { tail -30 gpurun_out/k9_tests.log; exit 1; }
tail -1 gpurun_out/k9_tests.log
bash tools/kprof.sh k9a --lanes 1 --total-frames 1000 || exit 1
bash tools/kprof.sh k9b --lanes 1 --total-frames 125 || exit 1
bash tools/kprof.sh k9d --lanes 1 --dense --total-frames 125 || exit 1
for t in k9a k9b k9d; do
  echo "== $t"
  python tools/kstats.py $(ls gpurun_out/kprof_$t/*kernel_stats.csv | head -1) 4 > gpurun_out/ks_$t.txt
  grep "summarize\|runs_lane\|frame_sort" gpurun_out/ks_$t.txt
done
