#!/bin/bash
# Sweep the x->z->x y-chunk size (CHANNEL_YCHUNK) on the large grids; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
one() {
  tag=$1; yc=$2; shift 2
  CHANNEL_YCHUNK=$yc timeout -k 10 240 python bench.py "$@" > gpurun_out/yc_${tag}_${yc}.log 2>&1 || { echo "FAILED $tag $yc"; tail -20 gpurun_out/yc_${tag}_${yc}.log; exit 1; }
  echo "$tag ychunk=$yc $(tail -1 gpurun_out/yc_${tag}_${yc}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), "ms/step")')"
}
for yc in ${YCS_2048:-1 2 4}; do one g2048 $yc --grid 2048x633x2048 --re 48300 --steps 3 --warmup 1 || exit 1; done
for yc in ${YCS_F64:-2 4 8}; do one f64 $yc --grid 1024x385x1024 --precision fp64 --steps 5 --warmup 2 || exit 1; done
for yc in ${YCS_550:-8 16 32}; do one g512 $yc --grid 512x257x512 --re 11150 --steps 20 --warmup 3 || exit 1; done
