#!/bin/bash
# GPU test subset: bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-x}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/t_$tag.log 2>&1
rc=$?
tail -n 25 gpurun_out/t_$tag.log
exit $rc
