#!/bin/bash
# MFMA depthwise forward: numerics tests, same-box bench A/B (RT1_DW_MFMA=0/1) and an eager rocprof of the new path
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-dwm}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dwmfma_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
AB_ENV=RT1_DW_MFMA TAG=$TAG bash tools/gpu/ab_env.sh || exit 1
PROF_TAG=prof_$TAG PROF_STEPS=3 bash tools/gpu/prof.sh > /dev/null || exit 1
echo done
