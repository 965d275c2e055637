#!/bin/bash
# Round-3 GPU check: the new full-size parity tests first, then the whole GPU suite.
#   bash tools/gpu_r3.sh [pytest selection...]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export RPT_HEARTBEAT=gpurun_out/heartbeat.log
SEL=${*:-tests/test_bigstack_gpu.py tests/test_cli_gpu.py tests/test_denoise_gpu.py "tests/test_fullsize_gpu.py::test_dense_stack_12_frames_land"}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 900 --timeout-method thread \
  > gpurun_out/gpu_new.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_new.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$*" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
    > gpurun_out/gpu_all.log 2>&1
  rc=$?
  tail -15 gpurun_out/gpu_all.log
fi
exit $rc
