#!/bin/bash
# A/B of the depthwise tile-prefetch pipeline: default build (RT1_DW_PF=4) vs variants build/pf0, build/pf2
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_backbone_gpu.py > gpurun_out/pf_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/pf_test.log; exit 1; }
tail -1 gpurun_out/pf_test.log
VARIANTS="${PF_VARIANTS:-pf0 pf2}" bash tools/gpu_ab.sh || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_pf.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_pf.log; exit 1; }
tail -1 gpurun_out/bench_pf.log
