#!/bin/bash
# GPU check of the slab-bucket K4: ST-DBSCAN / path / full-size parity, then the GPU suite, then
# bench A/B (RPT_K4_BUCKET=1 / 0) at 125 and 1000 frames and a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
# RPT_* switches are read only by the A/B build (python -m rpt._build --ab, built on the CPU host)
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so"
[ -f "$RPT_LIB" ] || { echo "build librpt_ab.so first: (cd radar-point-cloud-tracking_amd && python -m rpt._build --ab)"; exit 1; }
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
for fr in 125 1000; do
  for b in 1 0; do
    RPT_K4_BUCKET=$b timeout -k 10 200 python bench.py --total-frames $fr --steps 20 --warmup 3 \
      --no-cpu-baseline --h2d-steps 0 > gpurun_out/k4b_b${fr}_$b.json 2> gpurun_out/k4b_b${fr}_$b.err || exit 1
    python - "$fr" "$b" <<'PY'
import json, sys
fr, b = sys.argv[1:]
d = json.loads(open(f"gpurun_out/k4b_b{fr}_{b}.json").read().strip().splitlines()[-1])
print("bucket" if b == "1" else "radix", fr, d["value"], d["ms_per_step"], d["stage_ms"])
PY
  done
done
bash tools/kprof.sh k4b1000 --total-frames 1000
