#!/bin/bash
# GPU check of the denoise mode: its tests, then the rest of the GPU suite.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_denoise_gpu.py > gpurun_out/denoise_tests.log 2>&1 \
  || { tail -60 gpurun_out/denoise_tests.log; exit 1; }
tail -3 gpurun_out/denoise_tests.log
