#!/bin/bash
# Round-4 GPU session A: gemm.hip v2 numerics, the bench with / without it (the bench also runs its graph == eager
# self-check), the per-shape timing against the library.
source "$(dirname "$0")/step.sh"
run_step gemm2_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm2_gpu.py
run_step bench_g2 300 python -u bench.py --steps 20 --warmup 5
RT1_GEMM2=0 RT1_TF_GEMM2=0 run_step bench_nog2 300 python -u bench.py --steps 20 --warmup 5
run_step gemm2_bench 300 python -u tools/bench_gemm2.py --iters 20
run_step bench_c2 300 env RT1_DW_C2=1 python -u bench.py --steps 20 --warmup 5
