#!/bin/bash
# Same-box kernel A/B in ABBA order (base, new, new, base) of the in-tree librpt against
# abl/librpt_base.so, per workload (WL: std std1000 dense); the first run on a fresh box is
# slower across the board, so a plain new-then-base order biases every kernel.  Output:
# gpurun_out/kab2[_TAG]/<W>_{new,base}.txt (NEWLIB / BASE: other libraries than the in-tree
# build / abl/librpt_base.so; NEWENV: VAR=value switches for the NEWLIB runs only, e.g. the A/B
# build against itself) (per-kernel means over both runs of a variant) + a diff.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/kab2${TAG:+_$TAG}
BASE=${BASE:-$PWD/abl/librpt_base.so}
mkdir -p $O
for W in ${WL:-std1000 dense}; do
  A=(--lanes 1 --total-frames 125); [ $W = dense ] && A+=(--dense)
  [ $W = std1000 ] && A=(--lanes 1 --total-frames 1000)
  for v in base1 new1 new2 base2; do
    K=${TAG:+${TAG}_}${W}_$v
    if [[ $v == base* ]]; then
      RPT_LIB="$BASE" bash tools/kprof.sh $K "${A[@]}" || exit 1
    elif [ -n "$NEWLIB" ]; then
      env $NEWENV RPT_LIB="$NEWLIB" bash tools/kprof.sh $K "${A[@]}" || exit 1
    else
      bash tools/kprof.sh $K "${A[@]}" || exit 1
    fi
    python tools/kstats.py "$(ls gpurun_out/kprof_$K/*kernel_stats.csv | head -1)" 4 \
      > $O/${W}_$v.txt
  done
  python tools/kab_mean.py $O/${W}_new1.txt $O/${W}_new2.txt > $O/${W}_new.txt
  python tools/kab_mean.py $O/${W}_base1.txt $O/${W}_base2.txt > $O/${W}_base.txt
  echo "== $W (new vs base)"
  python tools/kab_diff.py $O/${W}_new.txt $O/${W}_base.txt ${TOP:-8} | tee $O/${W}_diff.txt
done
