#!/bin/bash
# Round-5 baseline on a fresh box: bench x2, eager kernel trace -> per-step categories
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step r5b_bench1 400 python -u bench.py --steps 20 --warmup 5
run_step r5b_bench2 400 python -u bench.py --steps 20 --warmup 5
bash tools/gpu/trace_now.sh
