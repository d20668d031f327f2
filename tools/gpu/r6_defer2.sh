#!/bin/bash
# deferred split-K sums v2 (split groups in the gather reduce, z-mode raw partials only for <= 4 splits, tf_gemm NN only)
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step defer3_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graph_gpu.py tests/test_pwgemm_gpu.py tests/test_parity_gpu.py -k "deferred or multi_reduce or pw_z_finish or full_model"
TAIL=20 run_step r6_trace_defer3 500 bash tools/gpu/trace_now.sh
BASE_TREE=build/base_tree TAG=defer3 STEPS=20 TAIL=8 run_step defer3_ab 900 bash tools/gpu/ab_tree.sh
