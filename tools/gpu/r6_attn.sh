#!/bin/bash
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step attn2_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "attn or attention or full_model or layer"
TAIL=20 run_step r6_trace_attn2 500 bash tools/gpu/trace_now.sh
