#!/bin/bash
# FiLM cmap GEMM + wgrad routing: kernel tests, whole-model parity, then a same-box A/B against HEAD (build/base_tree)
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step film_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_film_gpu.py tests/test_parity_gpu.py
BASE_TREE=build/base_tree TAG=film STEPS=20 TAIL=8 run_step film_ab 900 bash tools/gpu/ab_tree.sh
