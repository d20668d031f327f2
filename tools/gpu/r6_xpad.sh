#!/bin/bash
# x-mode forward tile with a 16-B pad per staged pixel: tests, kernel trace, same-box A/B against base_tree
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step xpk_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_xmode_gpu.py tests/test_backbone_gpu.py
TAIL=20 run_step r6_trace_xpk 500 bash tools/gpu/trace_now.sh
BASE_TREE=build/base_tree TAG=xpk STEPS=20 TAIL=8 run_step xpk_ab 900 bash tools/gpu/ab_tree.sh
