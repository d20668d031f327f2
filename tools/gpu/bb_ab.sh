#!/bin/bash
# pw_gemm_bn2bwd store loop with loads in flight (RT1_BB_U = 4 default build, 2 variant): numerics, then the projbwd
# blocks' dy-ready chain (tools/bench_dy_chain.py) on both builds
source "$(dirname "$0")/step.sh"
run_step bb_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_pwgemm_gpu.py::test_pw_gemm_bn2bwd_epilogue
TAIL=12 run_step bb_u4 300 python -u tools/bench_dy_chain.py --blocks 0,1,3,4,5,6,7
RT1_HIP_SO=build/v_bbu2/_rt1_hip.cpython-310-x86_64-linux-gnu.so TAIL=12 run_step bb_u2 300 \
    python -u tools/bench_dy_chain.py --blocks 0,1,3,4,5,6,7
