set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_path_gpu.py -k "stack_driver_matches or stack_path or regrow or concurrent" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/k1f_tests.log 2>&1
rc=$?; tail -15 gpurun_out/k1f_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/kprof.sh k1f --lanes 1 --total-frames 1000 || exit 1
python tools/kstats.py $(ls gpurun_out/kprof_k1f/*kernel_stats.csv | head -1) 4 > gpurun_out/ks_k1f.txt; head -12 gpurun_out/ks_k1f.txt
