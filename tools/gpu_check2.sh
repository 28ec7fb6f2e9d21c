#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-x}
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_solver_gpu.py -x -q -m gpu > gpurun_out/t_all_$tag.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$tag.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_$tag.log 2>&1
rc=$?
tail -n 2 gpurun_out/t_all_$tag.log; cat gpurun_out/bench_$tag.log | grep metric
exit $rc
