#!/bin/bash
# same-box A/B of the 1-GPU bench: A = $A_ENV (+ RT1_HIP_SO=$A_SO), B = $B_ENV, ABAB order; optional pytest first
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$PYTEST_SEL" ]; then
  timeout -k 10 300 python -u -m pytest $PYTEST_SEL -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab2_pytest.log; exit 1; }
  tail -1 gpurun_out/ab2_pytest.log
fi
for r in 1 2; do
  env $A_ENV ${A_SO:+RT1_HIP_SO=$A_SO} timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab2_A$r.log 2>&1 || { echo "A failed"; tail gpurun_out/ab2_A$r.log; exit 1; }
  echo "A$r $(tail -1 gpurun_out/ab2_A$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')"
  env $B_ENV ${B_SO:+RT1_HIP_SO=$B_SO} timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab2_B$r.log 2>&1 || { echo "B failed"; tail gpurun_out/ab2_B$r.log; exit 1; }
  echo "B$r $(tail -1 gpurun_out/ab2_B$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')"
done
