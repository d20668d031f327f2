#!/bin/bash
# Session-3 re-entry checkpoint: one-graph bench on the rebuilt tree, kernel trace categories, library GEMM census.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step r6s3_bench 300 python -u bench.py --steps 20 --warmup 5
TAIL=20 run_step r6s3_trace 500 bash tools/gpu/trace_now.sh
run_step r6s3_census 300 python -u tools/gemm_census.py
