#!/bin/bash
# TokenLearner backward with the transposed MFMA output layout: tests, trace, same-box A/B against base_tree (HEAD)
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step tl_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "token_learner or full_model or tokenizer"
TAIL=20 run_step r6_trace_tl 500 bash tools/gpu/trace_now.sh
BASE_TREE=build/base_tree TAG=tl STEPS=20 TAIL=8 run_step tl_ab 900 bash tools/gpu/ab_tree.sh
