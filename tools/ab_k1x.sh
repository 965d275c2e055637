#!/bin/bash
# GPU suite (unless SKIP_TESTS), then same-box A/B of the K1 variants at 1000 frames (default,
# RPT_K1_EXPAND=0: wave-per-group write), then a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
# RPT_* switches are read only by the A/B build (python -m rpt._build --ab, built on the CPU host)
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so"
[ -f "$RPT_LIB" ] || { echo "build librpt_ab.so first: (cd radar-point-cloud-tracking_amd && python -m rpt._build --ab)"; exit 1; }
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
  tail -2 gpurun_out/gpu_all.log
fi
FR=${FR:-1000}
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --total-frames $FR --steps 20 --warmup 3 \
    --no-cpu-baseline --h2d-steps 0 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || return 1
  python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{t}.json").read().strip().splitlines()[-1])
print(t, d["value"], d["ms_per_step"], d.get("one_stack_in_flight", {}).get("ms_per_step"), d["stage_ms"])
PY
}
run base RPT_K1_X=1 || exit 1
run noexp RPT_K1_EXPAND=0 || exit 1
run base2 RPT_K1_X=1 || exit 1
bash tools/kprof.sh x$FR --total-frames $FR
python tools/kstats.py $(find gpurun_out/kprof_x$FR -name "*kernel_stats.csv") 4 > gpurun_out/ks_x.txt; head -14 gpurun_out/ks_x.txt
