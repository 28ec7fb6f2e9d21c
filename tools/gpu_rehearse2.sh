#!/bin/bash
# Rehearse the multi-rank bench path (torchrun + gloo control plane + ShmComm data plane; RCCL
# refuses two ranks on one device) with 2 ranks sharing the single GPU of a
# gpurun box: small grid, short run.  Each step is time-limited; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CHANNEL_COMM=shm CHANNEL_SHM_SLOT_MB=64 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --grid 256x129x256 --re 3250 --steps 3 --warmup 1 \
  > gpurun_out/rccl2_bench.log 2>&1
rc=$?
tail -30 gpurun_out/rccl2_bench.log
exit $rc
