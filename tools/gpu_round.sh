#!/bin/bash
# One GPU call: GPU tests, 1-GPU bench, rocprofv3 kernel stats of a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_gpu_$tag.log 2>&1 \
  || { tail -n 30 gpurun_out/t_gpu_$tag.log; exit 1; }
tail -n 3 gpurun_out/t_gpu_$tag.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -n 1 gpurun_out/bench_$tag.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1 | xargs head -8
