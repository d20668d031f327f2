#!/bin/bash
# transformer projections on gemm2.hip (bias / residual / dropout epilogues, RT1_TF_GEMM2=1) vs hipBLASLt + tf_resid:
# the transformer numerics tests with it on, then the step alternated.
source "$(dirname "$0")/step.sh"
run_step tfg2_tests 300 env RT1_TF_GEMM2=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gemm2_gpu.py tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_gpu.py
for rep in 1 2 3; do
    TAIL=1 run_step tfg2_off_$rep 300 env RT1_TF_GEMM2=0 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step tfg2_on_$rep 300 env RT1_TF_GEMM2=1 python -u bench.py --steps 20 --warmup 5
done
