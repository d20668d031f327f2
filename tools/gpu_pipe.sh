#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_backbone_gpu.py -k dwconv > gpurun_out/pipe_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/pipe_test.log; exit 1; }
tail -1 gpurun_out/pipe_test.log
VARIANTS="nopipe" bash tools/gpu_ab.sh || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_pipe.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/bench_pipe.log; exit 1; }
tail -1 gpurun_out/bench_pipe.log
