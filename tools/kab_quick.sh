#!/bin/bash
# Kernel-level A/B only (no bench legs): in-tree librpt vs abl/librpt_base.so at FR frames,
# after the ST-DBSCAN parity tests.   [FR=1000] bash tools/kab_quick.sh
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_stdbscan_gpu.py tests/test_fullsize_gpu.py tests/test_bigstack_gpu.py::test_bench_stacks_lanes3_match_oracle -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/kq_tests.log 2>&1 || { tail -30 gpurun_out/kq_tests.log; exit 1; }
tail -1 gpurun_out/kq_tests.log
TESTS= NOBENCH=1 bash tools/kab_lib.sh
