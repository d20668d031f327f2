#!/bin/bash
# gemm256.hip: numerics vs fp32 torch, then the shape table against the step's current kernels
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step g256_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py ${G256_TEST_ARGS}
run_step g256_bench 400 python -u tools/bench_gemm256.py ${G256_BENCH_ARGS}
run_step g256_breakdown 300 python -u tools/bench_g256_breakdown.py
