#!/bin/bash
# GPU checkpoint on one MI355X: GPU test suite, smoke, 1-GPU bench, then (optionally) a rocprofv3 kernel summary.
#   TAG=r2a bash tools/gpu/suite.sh            # everything
#   SKIP_TESTS=1 PROF=0 TAG=x bash tools/gpu/suite.sh
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed $?"; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head -20; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed $?"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -2 gpurun_out/smoke_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_$TAG.log
fi
if [ "${PROF:-1}" = "1" ]; then
  PROF_TAG=prof_$TAG PROF_STEPS=3 PROF_TITLE="rocprofv3 kernel summary: RT-1 b128 hip backend, eager step ($TAG)" bash tools/gpu/prof.sh || exit 1
fi
exit 0
