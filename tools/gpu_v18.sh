#!/bin/bash
# v18: default-chunk bench on the headline grid and the 512/2048 grids, plus kernel stats at 2048.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/v18_bench.log 2>&1 || { tail -20 gpurun_out/v18_bench.log; exit 1; }
tail -1 gpurun_out/v18_bench.log
timeout -k 10 200 python bench.py --grid 512x257x512 --re 11150 --steps 20 --warmup 3 > gpurun_out/v18_512.log 2>&1 || { tail -20 gpurun_out/v18_512.log; exit 1; }
tail -1 gpurun_out/v18_512.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v18_prof2048 -o run --output-format csv -- python3 bench.py --grid 2048x633x2048 --re 48300 --steps 2 --warmup 1 > gpurun_out/v18_prof2048.log 2>&1 || { tail -20 gpurun_out/v18_prof2048.log; exit 1; }
tail -1 gpurun_out/v18_prof2048.log
