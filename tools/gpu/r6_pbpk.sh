#!/bin/bash
# projbwd staging as packed pairs (KO = 2 forms): tests, trace, same-box A/B against base_tree (HEAD)
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step pbpk_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_backbone_gpu.py tests/test_parity_gpu.py
TAIL=20 run_step r6_trace_pbpk 500 bash tools/gpu/trace_now.sh
BASE_TREE=build/base_tree TAG=pbpk STEPS=20 TAIL=8 run_step pbpk_ab 900 bash tools/gpu/ab_tree.sh
