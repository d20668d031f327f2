#!/bin/bash
# Round-4 first GPU session: SE data-parallel probes, the new GPU tests, the bench with its graph == eager self-check,
# the resident input path's device cost and a kernel-trace profile of the bench step.
source "$(dirname "$0")/step.sh"
TAIL=30 run_step se_dp_debug 900 bash tools/gpu/se_dp_debug.sh
run_step pytest_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_imgproc_gpu.py tests/test_distributed_gpu.py
run_step bench 300 python -u bench.py --steps 20 --warmup 5
run_step resident_decode 200 python -u tools/gpu/resident_decode.py
run_step gemm2_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm2_gpu.py
run_step gemm2_bench 300 python -u tools/bench_gemm2.py --iters 20
