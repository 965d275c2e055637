#!/bin/bash
# The whole GPU suite (durations), then a same-box kernel A/B of the in-tree librpt against
# abl/librpt_base.so on the dense 125-frame share and the standard 125-frame share.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4suite
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    --durations=20 ${TESTK:+-k "$TESTK"} > $O/gputest.log 2>&1 || { tail -60 $O/gputest.log; exit 1; }
  tail -28 $O/gputest.log
fi
for W in ${WL:-dense std}; do
  A=(--lanes 1 --total-frames 125); [ $W = dense ] && A+=(--dense)
  [ $W = std1000 ] && A=(--lanes 1 --total-frames 1000)
  bash tools/kprof.sh ${W}_new "${A[@]}" || exit 1
  RPT_LIB="$PWD/abl/librpt_base.so" bash tools/kprof.sh ${W}_base "${A[@]}" || exit 1
  for t in new base; do
    echo "== $W $t"
    python tools/kstats.py "$(ls gpurun_out/kprof_${W}_$t/*kernel_stats.csv | head -1)" 4 > $O/kab_${W}_$t.txt
    head -${TOP:-16} $O/kab_${W}_$t.txt
  done
done
