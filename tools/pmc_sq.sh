#!/bin/bash
# One rocprofv3 --pmc pass of SQ (shader sequencer) counters over a short bench run, counters only
# (no traces): per-kernel instruction mix and busy cycles, for telling issue-bound kernels from
# memory-bound ones.  On the GPU box:  bash tools/pmc_sq.sh <tag> [bench args...]
#   -> gpurun_out/pmcsq_<tag>/ and a summary from tools/pmc_sq.py
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmcsq_$TAG" -o pmc \
  -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --h2d-steps 0 --no-timing \
  --no-one-stack --no-dense-k5 "$@" > "gpurun_out/pmcsq_$TAG.log" 2>&1 || exit $?
python tools/pmc_sq.py "gpurun_out/pmcsq_$TAG" | tee "gpurun_out/pmcsq_$TAG.txt"
