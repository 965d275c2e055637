#!/bin/bash
# Shard driver v2 on one box: the dist parity tests (gloo ranks sharing the GPU), then
# bench.py --sharded at 125 frames with 1 and 3 stacks in flight (and 3 with the sequencer's
# order kept at one rank).  Output: gpurun_out/r4shard/
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r4shard
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py ${TESTK:+-k "$TESTK"} -m gpu -x -v \
    --timeout 600 --timeout-method thread > $O/test_dist.log 2>&1 \
    || { tail -60 $O/test_dist.log; exit 1; }
  grep -E "PASSED|FAILED" $O/test_dist.log | tail -12
fi
COMMON="--total-frames ${FR:-125} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --h2d-steps 0 --no-dense-k5"
for L in ${SLANES:-1 3}; do
  timeout -k 10 240 python bench.py --sharded --lanes $L $COMMON > $O/shard_l$L.json 2> $O/shard_l$L.err \
    || { tail -30 $O/shard_l$L.err; exit 1; }
  python3 tools/benchline.py $O/shard_l$L.json "sharded lanes $L"
done
if [ -n "$SEQ" ]; then
  timeout -k 10 240 python bench.py --sharded --lanes 3 --sequenced $COMMON > $O/shard_l3s.json 2> $O/shard_l3s.err \
    || { tail -30 $O/shard_l3s.err; exit 1; }
  python3 tools/benchline.py $O/shard_l3s.json "sharded lanes 3 sequenced"
fi
