#!/bin/bash
# gemm.hip small-tile configs on the transformer projections and the FiLM kernels, in isolation
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step tf_gemms2 300 python -u tools/bench_tf_gemms.py
run_step film_bench 300 python -u tools/bench_film.py
