#!/bin/bash
# Sharded path at one rank, 125 frames, 1 and 3 stacks in flight (quick A/B of the lane mechanics).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r4lanes
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
COMMON="--total-frames ${FR:-125} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --h2d-steps 0 --no-dense-k5"
for L in ${SLANES:-1 3}; do
  timeout -k 10 240 python bench.py --sharded --lanes $L $COMMON $EXTRA > $O/shard_l$L.json 2> $O/shard_l$L.err \
    || { tail -20 $O/shard_l$L.err; exit 1; }
  python3 tools/benchline.py $O/shard_l$L.json "sharded lanes $L"
done
