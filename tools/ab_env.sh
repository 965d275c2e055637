#!/bin/bash
# A/B a tuning environment variable on the bench: bash tools/ab_env.sh VAR v1 v2 ...
VAR=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
# RPT_* switches are read only by the A/B build (python -m rpt._build --ab, built on the CPU host)
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so"
[ -f "$RPT_LIB" ] || { echo "build librpt_ab.so first: (cd radar-point-cloud-tracking_amd && python -m rpt._build --ab)"; exit 1; }
mkdir -p gpurun_out
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 \
    > "gpurun_out/ab_${VAR}_$v.json" 2>> gpurun_out/ab.err
  rc=$?; [ $rc -eq 0 ] || { echo "ab $VAR=$v rc=$rc"; exit $rc; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_${VAR}_$v.json').read().strip().splitlines()[-1]);print('$VAR=$v',d['value'],d['ms_per_step'],d['stage_ms'])"
done
