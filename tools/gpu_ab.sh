#!/bin/bash
# A/B: kernel tests, then bench + kernel stats for each env setting given as args ("A=1 B=2" strings)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_solver_gpu.py > gpurun_out/ab_${tag}_tests.log 2>&1 || { tail -30 gpurun_out/ab_${tag}_tests.log; exit 1; }
tail -2 gpurun_out/ab_${tag}_tests.log
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/ab_${tag}_$i.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_$i.log; exit 1; }
  echo "[$envs] $(tail -1 gpurun_out/ab_${tag}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), "ms/step")')"
done
