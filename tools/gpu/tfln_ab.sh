#!/bin/bash
# resid + next-LayerNorm / LN-backward + bf16 operand fusions: numerics (layer, chained layers, whole model, graph), step A/B
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step tfln_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_graph_gpu.py
grep -q " passed" gpurun_out/tfln_tests.log && ! grep -q "failed" gpurun_out/tfln_tests.log || exit 1
AB_ENV=RT1_TF_FUSE_LN TAG=tfln bash tools/gpu/ab_env.sh
