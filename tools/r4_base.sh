#!/bin/bash
# Round-4 baseline of the per-rank 125-frame step on one box: the frame-sharded path at one rank
# (identity collectives) with 1, 2 and 3 stacks in flight, and the single-GPU stack driver at 125
# frames with 1 and 3 stacks in flight.  Output: gpurun_out/r4base/*.json
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r4base
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
FR=${FR:-125}
COMMON="--total-frames $FR --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --h2d-steps 0 --no-dense-k5"
for L in ${SLANES:-1 2 3}; do
  timeout -k 10 240 python bench.py --sharded --lanes $L $COMMON > $O/shard_l$L.json 2> $O/shard_l$L.err \
    || { tail -20 $O/shard_l$L.err; exit 1; }
  python3 tools/benchline.py $O/shard_l$L.json "sharded lanes $L"
done
for L in ${LANES:-1 3}; do
  timeout -k 10 240 python bench.py --lanes $L $COMMON > $O/single_l$L.json 2> $O/single_l$L.err \
    || { tail -20 $O/single_l$L.err; exit 1; }
  python3 tools/benchline.py $O/single_l$L.json "single lanes $L"
done
