#!/bin/bash
# Round-4 GPU session B: the fused-SE data-parallel probes, the new / changed GPU tests, whole-model parity and the
# resident input path's device cost.
source "$(dirname "$0")/step.sh"
TAIL=30 run_step se_dp_debug 900 bash tools/gpu/se_dp_debug.sh
run_step pytest_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_imgproc_gpu.py tests/test_distributed_gpu.py tests/test_parity_gpu.py
run_step resident_decode 200 python -u tools/gpu/resident_decode.py
