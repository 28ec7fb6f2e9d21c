#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t_gpu_$tag.log 2>&1
rc=$?
tail -n 15 gpurun_out/t_gpu_$tag.log
exit $rc
