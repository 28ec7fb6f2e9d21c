#!/bin/bash
# GPU validation pass (each GPU step bounded; stop at the first failure)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_solver_gpu.py -x -q -m gpu > gpurun_out/t_solver.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof1.log 2>&1
rc=$?
for f in gpurun_out/*.log; do echo "== $f"; tail -n 3 $f; done
exit $rc
