#!/bin/bash
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step reduce_bench 300 python -u tools/bench_reduce.py
