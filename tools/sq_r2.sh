#!/bin/bash
# One SQ-counter pass (instruction mix / waits per kernel) of a bench configuration; counters
# only, no traces.  bash tools/sq_r2.sh <tag> [bench args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM \
  SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv \
  -d "$R/gpurun_out/sq_$TAG" -o pmc -- python "$R/bench.py" --steps 2 --warmup 1 \
  --no-cpu-baseline --no-timing --h2d-steps 0 "$@" > "gpurun_out/sq_$TAG.log" 2>&1
