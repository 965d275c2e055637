#!/bin/bash
# rocprofv3 kernel-trace summary + the two PMC passes (FETCH_SIZE, WRITE_SIZE, separate runs) of
# one bench configuration.  Usage on the GPU box, from the repo root:
#   bash tools/prof_r2.sh <tag> [bench args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --h2d-steps 0 --no-timing $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" \
  -o bench -- python "$R/bench.py" $ARGS > "gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "prof rc=$rc" >> "gpurun_out/prof_$TAG.log"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc \
    -- python "$R/bench.py" $ARGS > "gpurun_out/pmc_${C}_$TAG.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc" >> "gpurun_out/pmc_${C}_$TAG.log"; [ $rc -eq 0 ] || exit $rc
done
