set -o pipefail
for L in 1 2 3; do
  timeout -k 10 200 python bench.py --lanes $L --no-cpu-baseline --h2d-steps 0 > gpurun_out/lanes_$L.json 2>/dev/null || exit 1
done
timeout -k 10 120 python bench.py --total-frames 125 --no-cpu-baseline --h2d-steps 0 > gpurun_out/b125.json 2>/dev/null || exit 2
timeout -k 10 120 python bench.py --sharded --total-frames 125 --no-cpu-baseline --h2d-steps 0 > gpurun_out/b125s.json 2>gpurun_out/b125s.err || exit 3
timeout -k 10 120 python bench.py --sharded --sync-host --total-frames 125 --no-cpu-baseline --h2d-steps 0 > gpurun_out/b125ss.json 2>>gpurun_out/b125s.err || exit 4
