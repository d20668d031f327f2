#!/bin/bash
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
TAIL=20 run_step r6_trace_defer 500 bash tools/gpu/trace_now.sh
