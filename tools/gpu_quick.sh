#!/bin/bash
# GPU-box quick check: the K1/scan/path GPU tests first (fail fast), then tools/gpu_check.sh.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_prims_gpu.py tests/test_path_gpu.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1
rc=$?; tail -5 gpurun_out/quick.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_check.sh "${1:-r1}"
