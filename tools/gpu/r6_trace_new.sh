#!/bin/bash
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
TAIL=20 run_step r6_trace_new 500 bash tools/gpu/trace_now.sh
run_step tf_gemms 300 python -u tools/bench_tf_gemms.py
