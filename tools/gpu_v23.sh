#!/bin/bash
# v23: fp32 K-SPEC address-only slots at R = 3, 4: solver tests and the 128x129x128 fp32 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_solver_gpu.py tests/test_kernels_gpu.py tests/test_physics_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v23_tests.log 2>&1 || { tail -40 gpurun_out/v23_tests.log; exit 1; }
tail -2 gpurun_out/v23_tests.log
timeout -k 10 200 python bench.py --grid 128x129x128 --re 3130 --precision fp32 --steps 50 --warmup 5 > gpurun_out/v23_180.log 2>&1 || { tail -20 gpurun_out/v23_180.log; exit 1; }
tail -1 gpurun_out/v23_180.log | cut -c1-260
