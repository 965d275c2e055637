#!/bin/bash
# Round-6 GPU steps, run on the GPU box from the repo root:  bash tools/gpu_r6.sh <step> [...]
# Every step has its own time limit; the script stops at the first failing step.  Output under
# gpurun_out/r5/ (gpurun brings it back).
#   tests_new     the GPU tests added this round (dense redo slot) + forced-RCCL world 1
#   shard_cmp     sharded 125-frame step 1 / 3 lanes (forced RCCL, slot waits) vs the stack driver
#   tests_all     the whole -m gpu suite
#   shard_trace   kernel trace of the sharded per-rank step at one rank (125 frames, one lane,
#                 every collective forced through RCCL) + the host-side profile (identity)
#   shard_lanes   per-rank step, forced RCCL at one rank: 1 and 3 lanes
#   diag          A/B-build diagnostics (queue sizes, union cells per wave)
#   tests_dist    the sharded-path GPU tests + the A/B-variant tests
#   tests_core    ST-DBSCAN parity tests (after a K5-K8 change)
#   kab           same-box ABBA kernel A/B against abl/librpt_base.so (tools/ab_base.sh)
#   prof          profiles/r6 kernel traces + PMC traffic (tools/prof.sh) for the three workloads
#   bench         the default bench line (driver command)
#   smoke         __graft_entry__.smoke()
#   bench_hwq     the bench line at 4 (default) and 8 hardware queues per process, interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r6
mkdir -p $O
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python -u -m pytest -x -v --timeout-method thread"
BS="python bench.py --sharded --total-frames 125 --no-cpu-baseline --h2d-steps 0"
run() {  # run <name> <seconds> <cmd...>: output to $O/<name>.log
  local name=$1 lim=$2; shift 2
  echo "[gpu_r6] $name ..."
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[gpu_r6] $name rc=$rc"
  tail -3 "$O/$name.log"
  return $rc
}
for step in "$@"; do
  case $step in
    tests_new)
      run tests_new 1000 $PYT --timeout 900 \
        "tests/test_dist_gpu.py::test_sharded_dense_redo_slot_matches_oracle" \
        "tests/test_dist_gpu.py::test_rccl_world1_forced_collectives_match_single_gpu" || exit 1 ;;
    shard_cmp)    # per-rank 125-frame step, forced RCCL, 1 and 3 lanes, beside the stack driver's
                  # 125-frame line at 3 lanes (same box, interleaved)
      for rep in 1 2; do
        RPT_COMM_FORCE_COLLECTIVES=1 run sl1_$rep 200 $BS --lanes 1 --steps 40 --warmup 6 || exit 1
        RPT_COMM_FORCE_COLLECTIVES=1 run sl3_$rep 200 $BS --lanes 3 --steps 40 --warmup 6 || exit 1
        run st3_$rep 200 python bench.py --total-frames 125 --lanes 3 --steps 40 --warmup 6 \
          --no-cpu-baseline --h2d-steps 0 --no-dense-k5 || exit 1
      done
      for f in $O/sl1_*.log $O/sl3_*.log $O/st3_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], (d.get('steady_state') or {}).get('ms_per_step'), (d.get('slot_wait') or {}).get('ms_per_step_by_phase'))" $f
      done ;;
    tests_all)
      run tests_all 1100 $PYT --timeout 990 -m gpu tests/ || exit 1 ;;
    shard_trace)
      RPT_COMM_FORCE_COLLECTIVES=1 run shard_trace 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$R/$O/prof_shard" -o shard -- \
        python bench.py --sharded --total-frames 125 --no-cpu-baseline --h2d-steps 0 \
        --lanes 1 --steps 20 --warmup 3 --no-one-stack || exit 1
      run shard_host 200 python tools/prof_shard.py 125 20 || exit 1
      RPT_COMM_FORCE_COLLECTIVES=1 run shard_l1 200 $BS --lanes 1 --steps 40 --warmup 6 || exit 1 ;;
    shard_lanes)  # per-rank step at one rank, every collective through RCCL: 1 and 3 lanes
                  # (two rounds, interleaved)
      for rep in 1 2; do
        RPT_COMM_FORCE_COLLECTIVES=1 run sl1_$rep 200 $BS --lanes 1 --steps 40 --warmup 6 || exit 1
        RPT_COMM_FORCE_COLLECTIVES=1 run sl3_$rep 200 $BS --lanes 3 --steps 40 --warmup 6 || exit 1
      done ;;
    shard_lanes5) # per-rank step at one rank, every collective through RCCL: 3 vs 5 lanes
      for rep in 1 2; do
        RPT_COMM_FORCE_COLLECTIVES=1 run sl3b_$rep 200 $BS --lanes 3 --steps 40 --warmup 6 || exit 1
        RPT_COMM_FORCE_COLLECTIVES=1 run sl5_$rep 200 $BS --lanes 5 --steps 40 --warmup 6 || exit 1
      done ;;
    diag)         # A/B build: queue / list sizes (RPT_STATS) per workload, union cells per wave
      AB=radar-point-cloud-tracking_amd/rpt/librpt_ab.so
      for w in "125" "1000" "125 --dense"; do
        RPT_LIB=$AB RPT_STATS=1 run "stats_${w// /_}" 200 python bench.py --total-frames $w \
          --lanes 1 --steps 1 --warmup 0 --no-one-stack --no-dense-k5 --no-cpu-baseline \
          --h2d-steps 0 --no-timing || exit 1
        grep "rpt stats" "$O/stats_${w// /_}.log" | sort | uniq -c | head -8
      done
      for c in ${CPWS-4 8 16 32}; do  # (CPWS= : none)
        RPT_LIB=$PWD/$AB RPT_UNION_CPW=$c bash tools/kprof.sh cpw$c --lanes 1 --total-frames 125 \
          || exit 1
        python tools/kstats.py "$(ls gpurun_out/kprof_cpw$c/*kernel_stats.csv | head -1)" 4 \
          | grep -i "union\|label<" | sed "s/^/cpw=$c /"
      done ;;
    k5ab)         # K5 with the cell pass's masks (in-tree default) vs without (RPT_K5_MASK=0),
                  # A/B build, one stack in flight, hipEvent K5 time; 3 workloads, ABBA
      AB=radar-point-cloud-tracking_amd/rpt/librpt_ab.so
      K5B="python bench.py --lanes 1 --steps 12 --warmup 3 --no-cpu-baseline --h2d-steps 0 --no-dense-k5 --no-one-stack"
      for w in "1000" "125" "125 --dense"; do
        i=0
        for m in 1 0 0 1; do
          i=$((i + 1))
          RPT_LIB=$AB RPT_K5_MASK=$m run "k5m${m}_${w// /_}_$i" 300 $K5B --total-frames $w || exit 1
        done
      done
      for f in $O/k5m*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], 'K5 ms', d['roofline']['avg_ms'], 'step ms', d['ms_per_step'])" $f
      done ;;
    seqab)        # sharded 125-frame step, forced RCCL, 3 lanes: CommSequencer orders
      for rep in 1 2; do
        for v in "3:0,1,2,3,4,5,6,7" "4:0,1,2,6,7,8,9,10" "4:0,1,2,4,5,7,9,10" "3:0,1,2,4,5,6,7,8" "2:0,0,1,1,2,3,4,5"; do
          tag=$(echo "$v" | tr ':,' '__')
          RPT_COMM_FORCE_COLLECTIVES=1 RPT_SEQ_STAGGER=${v%%:*} RPT_SEQ_OFFSETS=${v#*:} \
            run "seq_${tag}_$rep" 200 $BS --lanes 3 --steps 40 --warmup 6 || exit 1
        done
      done
      for f in $O/seq_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['steady_state']['ms_per_step'], d['slot_wait']['ms_per_step_by_phase'])" $f
      done ;;
    seqab2)       # sharded 125-frame step, forced RCCL: lanes x CommSequencer orders (SEQV)
      for rep in ${SEQREPS:-1 2}; do
        for v in ${SEQV:-"3:2:0,0,1,1,2,3,4,5" "4:2:0,0,1,1,2,3,4,5" "5:2:0,0,1,1,2,3,4,5" "3:4:0,1,2,2,3,3,4,5" "4:3:0,1,2,4,5,6,7,8" "5:2:0,1,2,3,4,5,6,7"}; do
          IFS=: read -r L D OFF <<< "$v"
          tag="${SEQTAG}L${L}_d${D}_$(echo "$OFF" | tr ',' '_')"
          RPT_COMM_FORCE_COLLECTIVES=1 RPT_SEQ_STAGGER=$D RPT_SEQ_OFFSETS=$OFF \
            run "sq_${tag}_$rep" 200 $BS --lanes $L --steps ${SEQSTEPS:-40} --warmup 6 || exit 1
        done
      done
      for f in $O/sq_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['steady_state']['ms_per_step'], d['slot_wait']['ms_per_step_by_phase'])" $f
      done ;;
    tests_shard)
      run tests_shard 900 $PYT --timeout 600 tests/test_dist_gpu.py \
        "tests/test_bigstack_gpu.py::test_sharded_share_matches_oracle" || exit 1 ;;
    digest8)      # the 8 x 125 sharded digest check with every rank's output kept
      OMP_NUM_THREADS=2 run digest8 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29611 --tee 3 \
        tools/dist_check.py --backend gloo --frames 125 --lanes 1 --digest std0 || exit 1 ;;
    gridcap)      # A/B build: the wave-per-item kernels' grid cap (RPT_WAVE_GRID_CAP), the driver's
                  # bench line (5 stacks in flight, 1000 frames), interleaved
      AB=radar-point-cloud-tracking_amd/rpt/librpt_ab.so
      BB="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 --no-dense-k5 --no-one-stack"
      for rep in 1 2; do
        for c in ${CAPS:-4096 1024 512}; do
          RPT_LIB=$AB RPT_WAVE_GRID_CAP=$c run gcap${c}_$rep 300 $BB || exit 1
        done
      done
      for f in $O/gcap*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['steady_state']['ms_per_step'])" $f
      done ;;
    sldef)        # the default sharded configuration (lanes, sequencer order), forced RCCL, 100 steps
      for rep in 1 2; do
        RPT_COMM_FORCE_COLLECTIVES=1 run sldef${SEQTAG}_$rep 300 $BS --steps 100 --warmup 6 || exit 1
      done
      for f in $O/sldef${SEQTAG}_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['config']['stacks_in_flight'], d['ms_per_step'], d['steady_state']['ms_per_step'], d['slot_wait']['ms_per_step_by_phase'])" $f
      done ;;
    sl1)
      for rep in 1 2; do
        RPT_COMM_FORCE_COLLECTIVES=1 run sl1${SEQTAG}_$rep 200 $BS --lanes 1 --steps 40 --warmup 6 || exit 1
      done ;;
    tests_dist)
      run tests_dist 1000 $PYT --timeout 990 tests/test_dist_gpu.py tests/test_ab_variants_gpu.py \
        || exit 1 ;;
    tests_core)   # ST-DBSCAN parity (g2, full-size configs, 1000-frame digests, dense share)
      run tests_core 900 $PYT --timeout 600 tests/test_stdbscan_gpu.py tests/test_fullsize_gpu.py \
        "tests/test_bigstack_gpu.py::test_bench_stacks_lanes3_match_oracle" \
        "tests/test_bigstack_gpu.py::test_dense_config4_share_invariants" || exit 1 ;;
    kab)          # same-box ABBA kernel traces: in-tree build vs abl/librpt_base.so
      TAG=$KABTAG WL="${KABWL:-std std1000 dense}" run kab 1000 bash tools/kab2.sh || exit 1 ;;
    prof)         # profiles/r6: kernel traces + FETCH/WRITE passes, one stack in flight, per workload
      RD=r6 run prof_std_1000f 900 bash tools/prof.sh std_1000f || exit 1
      RD=r6 run prof_std_125f 600 bash tools/prof.sh std_125f --total-frames 125 || exit 1
      RD=r6 run prof_dense_125f 600 bash tools/prof.sh dense_125f --dense --total-frames 125 \
        || exit 1 ;;
    bench_ab)     # the driver's bench line: host workers 2 (round 4) vs 8, lanes 5 vs 4, interleaved
      BB="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-dense-k5 --h2d-steps 0"
      for rep in 1 2; do
        run bab_hw2_$rep 300 $BB --host-workers 2 || exit 1
        run bab_hw8_$rep 300 $BB || exit 1
        run bab_l4_$rep 300 $BB --lanes 4 || exit 1
      done
      for f in $O/bab_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['steady_state']['ms_per_step'])" $f
      done ;;
    bench)
      run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1 ;;
    bench_nothr)  # the bench line: threaded host ordering (in-tree) vs abl/librpt_nothr.so
      BB="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0"
      for rep in 1 2; do
        run bth_$rep 300 $BB || exit 1
        RPT_LIB=$R/abl/librpt_nothr.so run bnt_$rep 300 $BB || exit 1
      done
      for f in $O/bth_*.log $O/bnt_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['steady_state']['ms_per_step'])" $f
      done ;;
    bench_gate)   # the driver's bench line: K1 turns across lanes (--k1-gate) vs overlapping K1s
      BB="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0"
      for rep in 1 2; do
        run bg1_$rep 300 $BB --k1-gate || exit 1
        run bg0_$rep 300 $BB || exit 1
      done
      for f in $O/bg1_*.log $O/bg0_*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['steady_state']['ms_per_step'])" $f
      done ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench_lanes)  # the driver's bench line at 5 (default), 6 and 8 stacks in flight, interleaved
      BB="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0"
      for rep in 1 2; do
        for l in ${LANESET:-5 6 8}; do run bln${l}_$rep 300 $BB --lanes $l || exit 1; done
      done
      for f in $O/bln*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['steady_state']['ms_per_step'])" $f
      done ;;
    bench_hwq)    # the driver's bench line with the default 4 hardware queues vs 8, interleaved
      BB="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0"
      for rep in 1 2; do
        run bhq4_$rep 300 $BB || exit 1
        GPU_MAX_HW_QUEUES=8 run bhq8_$rep 300 $BB || exit 1
      done
      for f in $O/bhq*.log; do
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['steady_state']['ms_per_step'])" $f
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
