#!/bin/bash
# kernel stats (rocprofv3 --stats) of a short bench for each env setting: bash tools/gpu_prof_ab.sh TAG "ENV=.." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pab_${tag}_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pab_${tag}_$i.log 2>&1 || { tail -20 gpurun_out/pab_${tag}_$i.log; exit 1; }
  echo "== [$envs]"
  python3 - "gpurun_out/pab_${tag}_$i" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if float(r["Percentage"]) > 0.5:
        print(f'{float(r["AverageNs"])/1e6:8.3f} ms  x{r["Calls"]:>3}  {r["Name"][:90]}')
PY
done
