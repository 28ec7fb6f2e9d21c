#!/bin/bash
# v21: fp64 K-SPEC with address-only prefetch slots (R >= 3): solver/kernel tests, fp64 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_solver_gpu.py tests/test_kernels_gpu.py tests/test_physics_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v21_tests.log 2>&1 || { tail -40 gpurun_out/v21_tests.log; exit 1; }
tail -2 gpurun_out/v21_tests.log
timeout -k 10 200 python bench.py --grid 1024x385x1024 --precision fp64 --steps 5 --warmup 2 > gpurun_out/v21_f64.log 2>&1 || { tail -20 gpurun_out/v21_f64.log; exit 1; }
tail -1 gpurun_out/v21_f64.log | cut -c1-260
timeout -k 10 200 python bench.py --grid 128x129x128 --re 3130 --precision fp64 --steps 50 --warmup 5 > gpurun_out/v21_180.log 2>&1 || { tail -20 gpurun_out/v21_180.log; exit 1; }
tail -1 gpurun_out/v21_180.log | cut -c1-260
