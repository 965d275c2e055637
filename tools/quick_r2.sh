#!/bin/bash
# GPU suite (unless SKIP_TESTS is set), then the single-GPU bench at 125 and 1000 frames, then a 1000-frame kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
  tail -2 gpurun_out/gpu_all.log
fi
for fr in 125 1000; do
  timeout -k 10 200 python bench.py --total-frames $fr --steps 20 --warmup 3 --no-cpu-baseline \
    --h2d-steps 0 > gpurun_out/q_b${fr}.json 2> gpurun_out/q_b${fr}.err || exit 1
  python - "$fr" <<'PY'
import json, sys
fr = sys.argv[1]
d = json.loads(open(f"gpurun_out/q_b{fr}.json").read().strip().splitlines()[-1])
print(fr, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["stage_ms"])
PY
done
bash tools/kprof.sh q1000 --total-frames 1000
