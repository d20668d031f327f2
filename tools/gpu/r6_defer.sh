#!/bin/bash
# deferred split-K sums: tests (graph / film / distributed / parity), isolated GEMM configs, then a same-box A/B
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step defer_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graph_gpu.py tests/test_film_gpu.py tests/test_pwgemm_gpu.py tests/test_distributed_gpu.py tests/test_parity_gpu.py
run_step tf_gemms2 300 python -u tools/bench_tf_gemms.py
run_step film_bench 300 python -u tools/bench_film.py
BASE_TREE=build/base_tree TAG=defer STEPS=20 TAIL=8 run_step defer_ab 900 bash tools/gpu/ab_tree.sh
