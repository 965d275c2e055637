#!/bin/bash
# GPU-box check: smoke, -m gpu tests, bench, rocprofv3 kernel-trace summary.
# Usage (from the repo root on the box): bash tools/gpu_check.sh [tag]
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures: keep going; else stop
timeout -k 10 150 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --sync-host --no-cpu-baseline > gpurun_out/bench_sync.json 2>> gpurun_out/bench.err
rc=$?; echo "bench sync rc=$rc" >> gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" \
  -o bench -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-timing \
  > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/prof_$TAG.log
tail -4 gpurun_out/gpu_tests.log; cat gpurun_out/bench.json
exit $rc
