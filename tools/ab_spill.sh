# Same-box A/B of the current tree against a baseline commit built in a worktree at ./ab_base
# (git worktree add -f ab_base <commit> && (cd ab_base && python tools/build.py)); GPU tests first.
# Used for profiles/r03s3/kspec_zero_spill.txt.  Remove the worktree afterwards (it travels with gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { tail -n 30 gpurun_out/sp_tests.log; exit 1; }
tail -n 2 gpurun_out/sp_tests.log
for i in 1 2; do
  for v in new old; do
    d=.; [ $v = old ] && d=ab_base
    (cd $d && timeout -k 10 300 python bench.py --phases) > gpurun_out/sp_h_${v}$i.log 2>&1 || { tail -n 20 gpurun_out/sp_h_${v}$i.log; exit 1; }
    echo "headline $v: $(tail -n 1 gpurun_out/sp_h_${v}$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d.get("phase_ms_per_step",{}).get("kspec"))')"
  done
done
for v in new old; do
  d=.; [ $v = old ] && d=ab_base
  (cd $d && timeout -k 10 400 python bench.py --grid 2048x633x2048 --re 48300 --precision fp32 --steps 3 --warmup 1 --phases) > gpurun_out/sp_2k_${v}.log 2>&1 || { tail -n 20 gpurun_out/sp_2k_${v}.log; exit 1; }
  echo "retau2000 $v: $(tail -n 1 gpurun_out/sp_2k_${v}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d.get("phase_ms_per_step",{}).get("kspec"))')"
done
