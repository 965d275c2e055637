#!/bin/bash
# Bench with 1, 2 and 3 stacks in flight (lanes), plus the lanes GPU test.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_path_gpu.py -x -q -k "lanes or stack_path" \
  --timeout 200 --timeout-method thread > gpurun_out/lanes_test.log 2>&1
rc=$?; tail -3 gpurun_out/lanes_test.log; [ $rc -eq 0 ] || exit $rc
for L in 1 2 3; do
  timeout -k 10 300 python bench.py --lanes $L --no-cpu-baseline --steps 10 > gpurun_out/bench_l$L.json 2> gpurun_out/bench_l$L.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/bench_l$L.json'));print($L, d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done
