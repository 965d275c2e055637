#!/bin/bash
# Same-box kernel-level A/B of one RPT_* switch (A/B build), after optional GPU tests:
#   VAR=NAME OFF=value [FR=frames] [TESTS="tests/..."] bash tools/kab.sh
# -> per-kernel us/run of the default (on) and NAME=OFF (off) bench, rocprofv3 kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so" RPT_AB=1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/kab_tests.log 2>&1 || { tail -40 gpurun_out/kab_tests.log; exit 1; }
  tail -2 gpurun_out/kab_tests.log
fi
FR=${FR:-1000}
bash tools/kprof.sh on --lanes 1 --total-frames $FR || exit 1
env $VAR=$OFF bash tools/kprof.sh off --lanes 1 --total-frames $FR || exit 1
for t in on off; do
  echo "== $t"
  python tools/kstats.py "$(ls gpurun_out/kprof_$t/*kernel_stats.csv | head -1)" > gpurun_out/kab_$t.txt
  head -${TOP:-16} gpurun_out/kab_$t.txt
done
