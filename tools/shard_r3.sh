#!/bin/bash
# Sharded-path checks and per-rank cost at one rank (identity collectives): the dist parity tests,
# then bench.py --sharded at F frames with 1, 2 and 3 stacks in flight (CommSequencer lanes).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py tests/test_bigstack_gpu.py -k "shard or dist" \
    -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_dist.log 2>&1 \
    || { tail -40 gpurun_out/gpu_dist.log; exit 1; }
  grep -E "PASSED|FAILED" gpurun_out/gpu_dist.log | tail -12
fi
FR=${FR:-125}
for L in ${LANES:-1 2 3}; do
  timeout -k 10 300 python bench.py --sharded --total-frames $FR --lanes $L --steps 20 --warmup 3 \
    --no-cpu-baseline --h2d-steps 0 --no-dense-k5 > gpurun_out/shard_l$L.json 2> gpurun_out/shard_l$L.err \
    || { tail -20 gpurun_out/shard_l$L.err; exit 1; }
  python - $L <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/shard_l{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("lanes", sys.argv[1], d["value"], d["ms_per_step"], (d.get("one_stack_in_flight") or {}).get("ms_per_step"), d["stage_ms"])
PY
done
