#!/bin/bash
# Measure every BASELINE.json config that fits one MI355X (single-GPU numbers; the 2/4/8-GPU runs
# are the driver's).  One bench.py per config, each under its own time limit; stop at the first
# failure.  JSON lines land in gpurun_out/cfg_<name>.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 "$TL" python bench.py "$@" > gpurun_out/cfg_${name}.log 2>&1 || { echo "FAILED $name"; tail -20 gpurun_out/cfg_${name}.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/cfg_${name}.log)"
}
TL=180 run retau180_fp64 --grid 128x129x128 --re 3130 --precision fp64 --steps 50 --warmup 5
TL=180 run retau180_fp32 --grid 128x129x128 --re 3130 --precision fp32 --steps 50 --warmup 5
TL=180 run retau550_fp32 --grid 512x257x512 --re 11150 --precision fp32 --steps 20 --warmup 3
TL=240 run retau950_fp64 --grid 1024x385x1024 --re 20700 --precision fp64 --steps 5 --warmup 2
TL=400 run retau2000_fp32 --grid 2048x633x2048 --re 48300 --precision fp32 --steps 3 --warmup 1
