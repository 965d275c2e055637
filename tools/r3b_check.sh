set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_stdbscan_gpu.py tests/test_fullsize_gpu.py tests/test_bigstack_gpu.py::test_bench_stacks_lanes3_match_oracle "tests/test_path_gpu.py" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3b_tests.log; [ $rc -eq 0 ] || exit $rc
NOBENCH=1 bash tools/kab_lib.sh || exit 1
timeout -k 10 300 python bench.py --sharded --total-frames 125 --steps 20 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/shard125.json 2> gpurun_out/shard125.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/shard125.json').read().strip().splitlines()[-1]); print('shard125', d['value'], d['ms_per_step'], d.get('stage_ms'), d['config'].get('stacks_in_flight'))"
