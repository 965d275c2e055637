#!/bin/bash
# Same-box bench of several builds: bash tools/ab_libs.sh lib1.so lib2.so ... (two interleaved
# rounds, FR frames); optional TESTS=... first (in-tree build).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_sel.log 2>&1 || { tail -40 gpurun_out/gpu_sel.log; exit 1; }
  tail -2 gpurun_out/gpu_sel.log
fi
FR=${FR:-1000}
for round in 1 2; do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)_$round
    RPT_LIB=$lib timeout -k 10 240 python bench.py --total-frames $FR --steps 20 --warmup 3 \
      --no-cpu-baseline --h2d-steps 0 --no-dense-k5 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || exit 1
    python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{t}.json").read().strip().splitlines()[-1])
print(t, d["value"], d["ms_per_step"], d.get("one_stack_in_flight", {}).get("ms_per_step"), d["stage_ms"])
PY
  done
done
