#!/bin/bash
# One parametrised GPU script for gpurun calls (replaces the per-version scratch scripts).
#
#   bash tools/gpu.sh TAG STEP [STEP ...]
#
# Steps (run in order; each under its own time limit; the script stops at the first failure):
#   tests            full GPU test suite          (PYTEST_K="not slow" selects by -k, PYTEST_ARGS adds files)
#   smoke            __graft_entry__.smoke()
#   bench            bench.py $BENCH_ARGS         (default: the headline grid)
#   prof             rocprofv3 --kernel-trace --stats of a short bench.py $BENCH_ARGS
#   pmc              PMC counter passes (one rocprofv3 run per counter group) of one bench step
#   counters         rocprofv3 -L (available PMC counters) -> <TAG>_counter_names.txt
#   configs          bench.py on every BASELINE config that fits one GPU
#   rehearse2        2-rank torchrun bench on one GPU over the shared-memory loopback data plane
#   ab               bench.py once per env setting in AB_ENVS ("A=1 B=2;A=2 B=2")
#   turb             long Re_tau~180 run (tools/turbulence.py $TURB_ARGS)
# Output: gpurun_out/<TAG>_<step>.log (+ rocprofv3 directories).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
shift
BENCH_ARGS=${BENCH_ARGS:-}
fail() { echo "FAILED: $1"; tail -n 40 "$2"; exit 1; }

for step in "$@"; do
  log=gpurun_out/${tag}_${step}.log
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} $PYTEST_ARGS > $log 2>&1 || fail tests $log
      tail -n 2 $log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || fail smoke $log
      tail -n 1 $log ;;
    bench)
      timeout -k 10 400 python bench.py $BENCH_ARGS > $log 2>&1 || fail bench $log
      tail -n 1 $log ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
        -- python3 bench.py --steps 3 --warmup 1 $BENCH_ARGS > $log 2>&1 || fail prof $log
      python3 tools/kstats.py "$(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' | head -n 1)" 10 ;;
    pmc)
      i=0
      for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
                 "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                 "WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
                 "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INST_CYCLES_VMEM" \
                 ${PMC_EXTRA:+"$PMC_EXTRA"}; do
        i=$((i + 1))
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/${tag}_pmc$i -o run --output-format csv \
          -- python3 bench.py --steps 1 --warmup 1 $BENCH_ARGS > gpurun_out/${tag}_pmc$i.log 2>&1 \
          || fail "pmc pass $i" gpurun_out/${tag}_pmc$i.log
      done
      python3 tools/pmc_summary.py gpurun_out/${tag}_pmc* > $log 2>&1 || fail pmc_summary $log
      echo "pmc: $i passes -> $log" ;;
    counters)
      timeout -s KILL 120 rocprofv3 -L > $log 2>&1 || fail counters $log
      grep -o -E '\b(SQ|TCC|TCP|TA|TD|GRBM)_[A-Z0-9_]+' $log | sort -u > gpurun_out/${tag}_counter_names.txt || true
      wc -l < gpurun_out/${tag}_counter_names.txt ;;
    configs)
      run_cfg() {
        name=$1; tl=$2; shift 2
        timeout -k 10 $tl python bench.py "$@" > gpurun_out/${tag}_cfg_${name}.log 2>&1 \
          || fail "config $name" gpurun_out/${tag}_cfg_${name}.log
        echo "$name $(tail -n 1 gpurun_out/${tag}_cfg_${name}.log | cut -c1-400)"
      }
      run_cfg retau180_fp64 180 --grid 128x129x128 --re 3130 --precision fp64 --steps 50 --warmup 5
      run_cfg retau180_fp32 180 --grid 128x129x128 --re 3130 --precision fp32 --steps 50 --warmup 5
      run_cfg retau550_fp32 180 --grid 512x257x512 --re 11150 --precision fp32 --steps 20 --warmup 3
      run_cfg retau950_fp64 240 --grid 1024x385x1024 --re 20700 --precision fp64 --steps 5 --warmup 2
      run_cfg retau2000_fp32 400 --grid 2048x633x2048 --re 48300 --precision fp32 --steps 3 --warmup 1 ;;
    rehearse2)
      CHANNEL_COMM=shm CHANNEL_SHM_SLOT_MB=64 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --grid 256x129x256 \
        --re 3250 --steps 3 --warmup 1 > $log 2>&1 || fail rehearse2 $log
      tail -n 1 $log ;;
    ab)
      IFS=';' read -ra settings <<< "$AB_ENVS"
      i=0
      for envs in "${settings[@]}"; do
        i=$((i + 1))
        env $envs timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/${tag}_ab$i.log 2>&1 \
          || fail "ab [$envs]" gpurun_out/${tag}_ab$i.log
        echo "[$envs] $(tail -n 1 gpurun_out/${tag}_ab$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')"
      done ;;
    turb)
      timeout -k 10 ${TURB_TL:-1000} python -u tools/turbulence.py $TURB_ARGS > $log 2>&1 || fail turb $log
      tail -n 5 $log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
