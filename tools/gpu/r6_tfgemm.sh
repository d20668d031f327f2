#!/bin/bash
# deferred-sum tree: kernel trace; then the transformer projections on gemm.hip small tiles (tf_gemm) A/B
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
TAIL=20 run_step r6_trace_defer 500 bash tools/gpu/trace_now.sh
TESTS="tests/test_parity_gpu.py tests/test_graph_gpu.py" AB_ENV=tf_gemm TAG=tfgemm TAIL=12 run_step tfgemm_ab 900 bash tools/gpu/ab_env.sh
