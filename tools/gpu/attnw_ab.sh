#!/bin/bash
# attention backward with 8 waves per (batch, head): numerics, step A/B vs 4 waves
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step attnw_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or transformer"
grep -q " passed" gpurun_out/attnw_tests.log && ! grep -q "failed" gpurun_out/attnw_tests.log || exit 1
AB_ENV=RT1_ATTN_BWD_W TAG=attnw bash tools/gpu/ab_env.sh
