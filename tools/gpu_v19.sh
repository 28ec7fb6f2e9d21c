#!/bin/bash
# v19: large-NY oracle tests, full GPU suite, then 2048 bench + kernel stats and the headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_solver_gpu.py -k large_ny -x -v --timeout 120 --timeout-method thread > gpurun_out/v19_large.log 2>&1 || { tail -40 gpurun_out/v19_large.log; exit 1; }
tail -5 gpurun_out/v19_large.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v19_tests.log 2>&1 || { tail -40 gpurun_out/v19_tests.log; exit 1; }
tail -2 gpurun_out/v19_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v19_prof2048 -o run --output-format csv -- python3 bench.py --grid 2048x633x2048 --re 48300 --steps 2 --warmup 1 > gpurun_out/v19_prof2048.log 2>&1 || { tail -20 gpurun_out/v19_prof2048.log; exit 1; }
timeout -k 10 300 python bench.py --grid 2048x633x2048 --re 48300 --steps 3 --warmup 1 > gpurun_out/v19_2048.log 2>&1 || { tail -20 gpurun_out/v19_2048.log; exit 1; }
tail -1 gpurun_out/v19_2048.log
timeout -k 10 200 python bench.py > gpurun_out/v19_bench.log 2>&1 || { tail -20 gpurun_out/v19_bench.log; exit 1; }
tail -1 gpurun_out/v19_bench.log
