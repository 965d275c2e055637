#!/bin/bash
# GPU check of the native shard driver: multi-rank parity (gloo ranks sharing the GPU), then
# 1-rank sharded bench vs the single-GPU stack driver at 125 and 1000 frames.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_dist_gpu.py > gpurun_out/shard_dist.log 2>&1 || { tail -40 gpurun_out/shard_dist.log; exit 1; }
tail -6 gpurun_out/shard_dist.log
for fr in 125 1000; do
  timeout -k 10 200 python bench.py --total-frames $fr --steps 20 --warmup 3 --no-cpu-baseline \
    --h2d-steps 0 --sharded > gpurun_out/shard_b${fr}.json 2> gpurun_out/shard_b${fr}.err || exit 1
  timeout -k 10 200 python bench.py --total-frames $fr --steps 20 --warmup 3 --no-cpu-baseline \
    --h2d-steps 0 > gpurun_out/single_b${fr}.json 2> gpurun_out/single_b${fr}.err || exit 1
  python - "$fr" <<'PY'
import json, sys
fr = sys.argv[1]
for k in ("shard", "single"):
    d = json.loads(open(f"gpurun_out/{k}_b{fr}.json").read().strip().splitlines()[-1])
    print(k, fr, d["value"], d["ms_per_step"], d["roofline"] and d["roofline"]["avg_ms"],
          d["stage_ms"])
PY
done
