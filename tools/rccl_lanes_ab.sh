#!/bin/bash
# Same-box A/B of the frame-sharded per-rank step at one rank (the 8-GPU share of the 1000-frame
# stack): identity collectives vs every collective through RCCL (RPT_COMM_FORCE_COLLECTIVES=1),
# 1 and 3 stacks in flight, interleaved.  Output: gpurun_out/rccl_ab/*.json
set -e
O=gpurun_out/rccl_ab
mkdir -p $O
B="python bench.py --sharded --total-frames 125 --steps 40 --warmup 6 --no-cpu-baseline --h2d-steps 0"
for rep in 1 2; do
  for lanes in 1 3; do
    timeout -k 10 150 $B --lanes $lanes > $O/id_l${lanes}_r${rep}.json 2> $O/id_l${lanes}_r${rep}.err
    RPT_COMM_FORCE_COLLECTIVES=1 timeout -k 10 150 $B --lanes $lanes \
      > $O/rccl_l${lanes}_r${rep}.json 2> $O/rccl_l${lanes}_r${rep}.err
    echo "rep $rep lanes $lanes done"
  done
done
