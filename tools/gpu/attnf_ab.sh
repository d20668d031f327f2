#!/bin/bash
# attention forward with 8 waves per (batch, head): numerics, step A/B vs 4 waves
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step attnf_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or transformer"
grep -q " passed" gpurun_out/attnf_tests.log && ! grep -q "failed" gpurun_out/attnf_tests.log || exit 1
AB_ENV=RT1_ATTN_FWD_W AB_VALUES="4 8" TAG=attnf bash tools/gpu/ab_env.sh
