#!/bin/bash
# PMC passes for the roofline traffic figure (run on the GPU box from the repo root):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they do not fit one TCC pass), counters
# only (no sys/runtime traces), then tools/pmc_traffic.py writes profiles/<tag>/k5_traffic.json.
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc \
    -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-timing \
    > "gpurun_out/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc" >> "gpurun_out/pmc_$C.log"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py "$TAG" "${2:-k5_traffic.json}" "${3:-bench.py default workload}"
