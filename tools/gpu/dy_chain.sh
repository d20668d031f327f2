#!/bin/bash
# gemm_se numerics + the per-block staging vs dy-ready chain timing (tools/bench_dy_chain.py).
source "$(dirname "$0")/step.sh"
TAG=${AB_TAG:-dyc}
run_step ${TAG}_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gemm_gpu.py::test_gemm_se_epilogues
TAIL=40 run_step ${TAG}_chain 400 python -u tools/bench_dy_chain.py $CHAIN_ARGS
