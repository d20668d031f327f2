#!/bin/bash
# dy-ready A/B: numerics tests with both dy-ready paths on, then bench.py alternating
# staging (RT1_DY_READY=0 RT1_DY_GEMM=0) / projbwd blocks only (RT1_DY_READY=1) / all blocks (+ RT1_DY_GEMM=1).
source "$(dirname "$0")/step.sh"
TAG=${AB_TAG:-dy}
run_step ${TAG}_tests 600 env RT1_DY_READY=1 RT1_DY_GEMM=1 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gemm_gpu.py::test_gemm_se_epilogues tests/test_backbone_gpu.py tests/test_pwgemm_gpu.py \
    tests/test_parity_gpu.py tests/test_graph_gpu.py tests/test_xmode_gpu.py
TAIL=40 run_step ${TAG}_chain 300 python -u tools/bench_dy_chain.py
for rep in $(seq 1 ${AB_REPS:-2}); do
    TAIL=1 run_step ${TAG}_off_$rep 300 env RT1_DY_READY=0 RT1_DY_GEMM=0 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step ${TAG}_pbf_$rep 300 env RT1_DY_READY=1 RT1_DY_GEMM=0 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step ${TAG}_all_$rep 300 env RT1_DY_READY=1 RT1_DY_GEMM=1 python -u bench.py --steps 20 --warmup 5
done
