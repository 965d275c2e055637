#!/bin/bash
# rocprofv3 kernel-trace summary of one bench configuration (no counters).  On the GPU box:
#   bash tools/kprof.sh <tag> [bench args...]   -> gpurun_out/kprof_<tag>/..._kernel_stats.csv
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kprof_$TAG" \
  -o bench -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --h2d-steps 0 \
  --no-timing "$@" > "gpurun_out/kprof_$TAG.log" 2>&1
