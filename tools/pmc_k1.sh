#!/bin/bash
# Stall profile of the K1 (polar scatter) and K5 kernels: one rocprofv3 --pmc pass of SQ counters
# (within the 8-SQ-counter limit of one pass), counters only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$R/gpurun_out/pmc_sq" \
  -o pmc -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timing \
  > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc" >> gpurun_out/pmc_sq.log; exit $rc
