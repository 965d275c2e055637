#!/bin/bash
# Reproducible roofline evidence for one workload, ONE stack in flight (--lanes 1, no other
# stack's kernels overlap the traced ones):
#   1. bench.py with hipEvent stage timing under rocprofv3 --kernel-trace --stats: the bench line
#      (gpurun_out/prof_<key>.json) and the kernel summary of the SAME command;
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (counters only) ->
#      profiles/$RD/k5_traffic_<key>.json / k1_traffic_<key>.json (tools/pmc_traffic.py);
#   3. the summaries copied to gpurun_out/$RD/ (kernel_stats_<key>.csv, bench_prof_<key>.json,
#      the traffic JSONs): gpurun brings gpurun_out/ back; `cp gpurun_out/$RD/* profiles/$RD/`.
# RD = the round's profile directory (default r5).
# Usage on the GPU box, from the repo root:  [RD=r5] bash tools/prof.sh <key> [bench args...]
#   keys used: std_1000f (default workload), std_125f (--total-frames 125),
#              dense_125f (--dense --total-frames 125)
KEY=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
RD=${RD:-r5}
mkdir -p gpurun_out/$RD
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-6}
ARGS="--lanes 1 --no-one-stack --no-dense-k5 --no-cpu-baseline --h2d-steps 0 --steps $STEPS --warmup 1 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$KEY" \
  -o bench -- python "$R/bench.py" $ARGS > "gpurun_out/prof_$KEY.json" 2> "gpurun_out/prof_$KEY.err"
rc=$?; echo "prof rc=$rc" >> "gpurun_out/prof_$KEY.err"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$R/gpurun_out/pmc_$C"
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o pmc \
    -- python "$R/bench.py" $ARGS --no-timing > "gpurun_out/pmc_${C}_$KEY.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc" >> "gpurun_out/pmc_${C}_$KEY.log"; [ $rc -eq 0 ] || exit $rc
done
RPT_PROFILE_OUT="$R/gpurun_out/$RD" python tools/pmc_traffic.py $RD "k5_traffic_$KEY.json" "bench.py $ARGS (one stack in flight)" \
  > "gpurun_out/pmc_traffic_$KEY.log" || exit 1
ST=$(find "$R/gpurun_out/prof_$KEY" -name '*kernel_stats.csv' | head -1)
cp "$ST" "gpurun_out/$RD/kernel_stats_$KEY.csv"
tail -1 "gpurun_out/prof_$KEY.json" > "gpurun_out/$RD/bench_prof_$KEY.json"
echo "[prof] $KEY done; steps=$STEPS (+1 warm-up) per command"
