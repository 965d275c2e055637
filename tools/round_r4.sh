#!/bin/bash
# Round-4 measurement: the default bench line, then the one-stack-in-flight profiles of the three
# roofline workloads (tools/prof_r4.sh).   bash tools/round_r4.sh [keys...]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out profiles/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_sel.log 2>&1 || { tail -40 gpurun_out/gpu_sel.log; exit 1; }
  tail -2 gpurun_out/gpu_sel.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
    || { tail -20 gpurun_out/bench_default.err; exit 1; }
  tail -c 3000 gpurun_out/bench_default.json
fi
for k in ${*:-std_1000f std_125f dense_125f}; do
  case $k in
    std_1000f) a="" ;;
    std_125f) a="--total-frames 125" ;;
    dense_125f) a="--dense --total-frames 125" ;;
  esac
  bash tools/prof_r4.sh $k $a || { echo "prof $k failed"; tail -20 gpurun_out/prof_$k.err; exit 1; }
done
