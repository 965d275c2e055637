#!/bin/bash
# Same-box kernel-level A/B of the in-tree librpt against abl/librpt_base.so (a copy of an earlier
# build), after optional GPU tests:   [FR=frames] [TESTS="tests/..."] bash tools/kab_lib.sh
# -> per-kernel us/run of both (rocprofv3 kernel trace, one stack in flight), then the bench line
#    of each (interleaved new, base).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/kab_tests.log 2>&1 || { tail -40 gpurun_out/kab_tests.log; exit 1; }
  tail -2 gpurun_out/kab_tests.log
fi
FR=${FR:-1000}
bash tools/kprof.sh new --lanes 1 --total-frames $FR || exit 1
RPT_LIB="$PWD/abl/librpt_base.so" bash tools/kprof.sh base --lanes 1 --total-frames $FR || exit 1
for t in new base; do
  echo "== $t"
  python tools/kstats.py "$(ls gpurun_out/kprof_$t/*kernel_stats.csv | head -1)" > gpurun_out/kab_$t.txt
  head -${TOP:-24} gpurun_out/kab_$t.txt
done
if [ -z "$NOBENCH" ]; then
  for t in new base; do
    lib=(); [ $t = base ] && lib=(RPT_LIB="$PWD/abl/librpt_base.so")
    env "${lib[@]}" timeout -k 10 240 python bench.py --total-frames $FR --steps 20 --warmup 3 \
      --no-cpu-baseline --h2d-steps 0 --no-dense-k5 > gpurun_out/kab_bench_$t.json 2> gpurun_out/kab_bench_$t.err || exit 1
    python - "$t" <<'PY'
import json, sys
t = sys.argv[1]
d = json.loads(open(f"gpurun_out/kab_bench_{t}.json").read().strip().splitlines()[-1])
print(t, d["value"], d["ms_per_step"], d.get("one_stack_in_flight", {}).get("ms_per_step"), d["stage_ms"])
PY
  done
fi
