#!/bin/bash
# HBM traffic per kernel launch at the bench workload (1000 frames, one stack in flight): FETCH_SIZE
# and WRITE_SIZE in separate rocprofv3 --pmc passes (counters only), then tools/pmc_traffic.py
# writes profiles/r2/k5_traffic_std_1000f.json, k1_traffic_std_1000f.json and the per-kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc \
    -- python "$R/bench.py" --steps 2 --warmup 1 --lanes 1 --no-cpu-baseline --no-timing \
    --h2d-steps 0 --no-dense-k5 > "gpurun_out/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc" >> "gpurun_out/pmc_$C.log"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py r2 k5_traffic_std_1000f.json "bench.py --total-frames 1000 (one stack in flight)"
