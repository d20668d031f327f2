#!/bin/bash
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step tl5_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "token_learner or full_model or tokenizer"
TAIL=20 run_step r6_trace_tl5 500 bash tools/gpu/trace_now.sh
