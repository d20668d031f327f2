#!/bin/bash
# full GPU suite + smoke + 1-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r9.log 2>&1 || { echo "pytest failed $?"; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r9.log | head -20; tail -30 gpurun_out/pytest_gpu_r9.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r9.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r9.log 2>&1 || { echo "smoke failed $?"; tail -20 gpurun_out/smoke_r9.log; exit 1; }
tail -2 gpurun_out/smoke_r9.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r9.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/bench_r9.log; exit 1; }
tail -1 gpurun_out/bench_r9.log
PROF_TAG=prof_v8 PROF_STEPS=3 PROF_TITLE="rocprofv3 kernel summary: RT-1 b128 hip backend, eager step (v8: flat BN apply / block tail)" bash tools/gpu_prof.sh || exit 1
