#!/bin/bash
# A/B of the K5 / K1 variants (env switches) on the bench at 1000 and 100 frames, after the
# parity tests of the touched kernels; then a kernel-trace profile of the default variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
# RPT_* switches are read only by the A/B build (python -m rpt._build --ab, built on the CPU host)
export RPT_LIB="$PWD/radar-point-cloud-tracking_amd/rpt/librpt_ab.so"
[ -f "$RPT_LIB" ] || { echo "build librpt_ab.so first: (cd radar-point-cloud-tracking_amd && python -m rpt._build --ab)"; exit 1; }
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_stdbscan_gpu.py tests/test_fullsize_gpu.py \
  tests/test_path_gpu.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_ab.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_ab.log; [ $rc -eq 0 ] || exit 1
for cfg in "RPT_K5_MODE=0 RPT_K1_MASKS=0" "RPT_K5_MODE=1 RPT_K1_MASKS=0" "RPT_K5_MODE=2 RPT_K1_MASKS=1" "RPT_K5_MODE=2 RPT_K1_MASKS=0"; do
  tag=$(echo $cfg | tr -d ' =_A-Z')
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --h2d-steps 0 > gpurun_out/ab_1000_$tag.json 2>/dev/null || exit 2
  env $cfg timeout -k 10 120 python bench.py --total-frames 100 --no-cpu-baseline --h2d-steps 0 > gpurun_out/ab_100_$tag.json 2>/dev/null || exit 3
done
export TMPDIR=/tmp
for fr in 1000 100; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_ab$fr" \
    -o bench -- python "$R/bench.py" --total-frames $fr --steps 3 --warmup 1 --no-cpu-baseline \
    --h2d-steps 0 --no-timing > gpurun_out/prof_ab$fr.log 2>&1 || exit 4
done
