#!/bin/bash
# one-launch Gram BN constants: tests, trace, same-box A/B against HEAD
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step gram_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_xmode_gpu.py tests/test_parity_gpu.py
TAIL=20 run_step r6_trace_gram 500 bash tools/gpu/trace_now.sh
BASE_TREE=build/base_tree TAG=gram STEPS=20 TAIL=8 run_step gram_ab 900 bash tools/gpu/ab_tree.sh
