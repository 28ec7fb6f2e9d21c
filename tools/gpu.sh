#!/bin/bash
# One parametrised GPU script for gpurun calls (replaces the per-version scratch scripts).
#
#   bash tools/gpu.sh TAG STEP [STEP ...]
#
# Steps (run in order; each under its own time limit; the script stops at the first failure):
#   tests            full GPU test suite          (PYTEST_K="not slow" selects by -k, PYTEST_ARGS adds files)
#   smoke            __graft_entry__.smoke()
#   bench            bench.py $BENCH_ARGS         (default: the headline grid)
#   prof             rocprofv3 --kernel-trace --stats of a short bench.py $BENCH_ARGS (+ gaps, graph dot)
#   fcprof           the same with CHANNEL_FORCE_COMM=1 (the P > 1 per-rank pipeline on one GPU)
#   pmc              PMC counter passes (one rocprofv3 run per counter group) of one bench step
#   counters         rocprofv3 -L (available PMC counters) -> <TAG>_counter_names.txt
#   configs          bench.py on every BASELINE config that fits one GPU
#   rehearse2        2-rank torchrun bench on one GPU over the shared-memory loopback data plane
#   rehearse8        8-rank bench.py --gpus 8 (slab, pencil 4x2 (auto), pencil 2x4) over the loopback, headline grid
#   rehearse24       2- and 4-rank bench.py (slab, kx sub-block overlap) over the loopback, headline grid
#   ab               bench.py once per env setting in AB_ENVS ("A=1 B=2;A=2 B=2")
#   probe            transform stage alone (tools/xform_probe.py $PROBE_ARGS) per env setting in PROBE_ENVS
#   kprobe           rocprofv3 kernel stats of the transform stage on one stream (env: $KPROBE_ENV)
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
      CHANNEL_GRAPH_DOT=gpurun_out/${tag}_graph timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof \
        -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 $BENCH_ARGS > $log 2>&1 || fail prof $log
      python3 tools/kstats.py "$(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' | head -n 1)" 10
      python3 tools/trace_gaps.py "$(find gpurun_out/${tag}_prof -name '*kernel_trace.csv' | head -n 1)" > gpurun_out/${tag}_gaps.txt
      tail -n 1 gpurun_out/${tag}_gaps.txt ;;
    fcprof)
      # the P > 1 per-rank pipeline on a 1-rank RCCL communicator: kernel trace, inter-kernel gaps,
      # step-graph topology (dot) next to the P = 1 one
      CHANNEL_FORCE_COMM=1 CHANNEL_GRAPH_DOT=gpurun_out/${tag}_graph_fc timeout -k 10 400 rocprofv3 --kernel-trace --stats \
        -d gpurun_out/${tag}_fcprof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 $BENCH_ARGS \
        > $log 2>&1 || fail fcprof $log
      python3 tools/kstats.py "$(find gpurun_out/${tag}_fcprof -name '*kernel_stats.csv' | head -n 1)" 10
      python3 tools/trace_gaps.py "$(find gpurun_out/${tag}_fcprof -name '*kernel_trace.csv' | head -n 1)" > gpurun_out/${tag}_fc_gaps.txt
      tail -n 1 gpurun_out/${tag}_fc_gaps.txt ;;
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
    rehearse8)
      # 8 ranks on the one GPU over the shared-memory loopback at the headline shape (bench.py
      # self-launches torch.distributed.run): slab, the automatic pencil (4 x 2) and the 2 x 4 pencil
      for dec in ${REHEARSE_DECS:-slab pencil pencil2x4}; do
        extra=""
        [ $dec = pencil2x4 ] && extra="--decomposition pencil --pr 2" || extra="--decomposition $dec"
        CHANNEL_COMM=shm timeout -k 10 600 python bench.py --gpus 8 $extra --steps 2 --warmup 1 \
          $BENCH_ARGS > gpurun_out/${tag}_rehearse8_$dec.log 2>&1 || fail "rehearse8 $dec" gpurun_out/${tag}_rehearse8_$dec.log
        tail -n 1 gpurun_out/${tag}_rehearse8_$dec.log
      done ;;
    rehearse24)
      # 2 and 4 ranks (slab: 4 and 2 kx sub-blocks, the K-SPEC / exchange overlap) on the one GPU
      # over the shared-memory loopback at the headline shape
      for n in 2 4; do
        CHANNEL_COMM=shm CHANNEL_SHM_SLOT_MB=64 timeout -k 10 600 python bench.py --gpus $n --steps 2 --warmup 1 \
          $BENCH_ARGS > gpurun_out/${tag}_rehearse$n.log 2>&1 || fail "rehearse $n" gpurun_out/${tag}_rehearse$n.log
        tail -n 1 gpurun_out/${tag}_rehearse$n.log
      done ;;
    ab)
      IFS=';' read -ra settings <<< "$AB_ENVS"
      i=0
      for envs in "${settings[@]}"; do
        i=$((i + 1))
        env $envs timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/${tag}_ab$i.log 2>&1 \
          || fail "ab [$envs]" gpurun_out/${tag}_ab$i.log
        echo "[$envs] $(tail -n 1 gpurun_out/${tag}_ab$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')"
      done ;;
    probe)
      # transform stage alone, once per env setting in PROBE_ENVS ("A=1;A=2 B=3"); "-" = defaults
      IFS=';' read -ra settings <<< "${PROBE_ENVS:--}"
      : > $log
      for envs in "${settings[@]}"; do
        [ "$envs" = "-" ] && envs=""
        env $envs timeout -k 10 200 python tools/xform_probe.py $PROBE_ARGS >> $log 2>&1 \
          || fail "probe [$envs]" $log
      done
      cat $log ;;
    kprobe)
      # isolated kernel times of the transform stage (one stream) under a rocprofv3 kernel trace
      env CHANNEL_YSTREAMS=1 $KPROBE_ENV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_kprobe -o run \
        --output-format csv -- python3 tools/xform_probe.py --reps 5 $PROBE_ARGS > $log 2>&1 || fail kprobe $log
      python3 tools/kstats.py "$(find gpurun_out/${tag}_kprobe -name '*kernel_stats.csv' | head -n 1)" 10 ;;
    pmcprobe)
      # PMC passes over the transform stage alone (one stream): issue/latency/LDS/TA/TLB/MALL groups
      i=0
      for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                 "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE" \
                 "FETCH_SIZE TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
                 "WRITE_SIZE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
                 ${PMC_EXTRA:+"$PMC_EXTRA"}; do
        i=$((i + 1))
        env CHANNEL_YSTREAMS=1 $KPROBE_ENV timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/${tag}_pmcp$i \
          -o run --output-format csv -- python3 ${PMC_PROG:-tools/xform_probe.py --reps 2 --warmup 1 $PROBE_ARGS} \
          > gpurun_out/${tag}_pmcp$i.log 2>&1
        st=$?
        if [ $st -ne 0 ]; then
          echo "pmc pass $i [$grp] exit $st"; tail -n 5 gpurun_out/${tag}_pmcp$i.log
          case $st in 124|134|137|139) exit 1 ;; esac
        fi
      done
      python3 tools/pmc_summary.py gpurun_out/${tag}_pmcp* > $log 2>&1 || fail pmc_summary $log
      echo "pmcprobe: $i passes -> $log" ;;
    turb)
      timeout -k 10 ${TURB_TL:-1000} python -u tools/turbulence.py $TURB_ARGS > $log 2>&1 || fail turb $log
      tail -n 5 $log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
