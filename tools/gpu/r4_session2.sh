#!/bin/bash
# gemm.hip v2: numerics, then timing against the library / v1
source "$(dirname "$0")/step.sh"
run_step gemm2_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm2_gpu.py
run_step gemm2_bench 300 python -u tools/bench_gemm2.py --iters 20
