#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_backbone_gpu.py -k batchnorm > gpurun_out/bn_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/bn_test.log; exit 1; }
tail -1 gpurun_out/bn_test.log
VARIANTS="${BN_VARIANTS:-bn256}" KB_ARGS="${BN_BLOCKS:---blocks 9,14,19,24,25}" bash tools/gpu_ab.sh || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bn.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_bn.log; exit 1; }
tail -1 gpurun_out/bench_bn.log
