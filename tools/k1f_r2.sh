#!/bin/bash
# GPU check of the staged K1: its parity tests first, then the whole GPU suite, then the
# single-GPU bench at 125 / 1000 frames with the fused and the two-pass K1, and a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
# RPT_* switches are read only by the A/B build (python -m rpt._build --ab, built on the CPU host)
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so"
[ -f "$RPT_LIB" ] || { echo "build librpt_ab.so first: (cd radar-point-cloud-tracking_amd && python -m rpt._build --ab)"; exit 1; }
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_path_gpu.py -k "k1 or stack_path or speculative" > gpurun_out/k1f_tests.log 2>&1 \
  || { tail -40 gpurun_out/k1f_tests.log; exit 1; }
tail -3 gpurun_out/k1f_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1 || { tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
for fr in 125 1000; do
  for fz in 1 0; do
    RPT_K1_STAGE=$fz timeout -k 10 200 python bench.py --total-frames $fr --steps 20 --warmup 3 \
      --no-cpu-baseline --h2d-steps 0 > gpurun_out/k1f_b${fr}_$fz.json 2> gpurun_out/k1f_b${fr}_$fz.err || exit 1
    python - "$fr" "$fz" <<'PY'
import json, sys
fr, fz = sys.argv[1:]
d = json.loads(open(f"gpurun_out/k1f_b{fr}_{fz}.json").read().strip().splitlines()[-1])
print("staged" if fz == "1" else "2read", fr, d["value"], d["ms_per_step"], d["stage_ms"])
PY
  done
done
bash tools/kprof.sh k1f125 --total-frames 125
