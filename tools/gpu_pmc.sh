#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, kernel-trace only) on one RK3 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-pmc}
shift
ARGS="$@"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/${tag}_p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 $ARGS > gpurun_out/${tag}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${tag}_p$i.log; exit 1; }
done
echo done
