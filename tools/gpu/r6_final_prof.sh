#!/bin/bash
# End-of-session profiles of the committed tree: per-step HBM bytes (PMC FETCH/WRITE passes) and trace categories
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
TAG=r6fb TAIL=6 run_step r6fb_pmc 700 bash tools/gpu/pmc_bytes.sh
run_step r6fb_step 120 python3 tools/pmc_step_bytes.py gpurun_out/r6fb_f gpurun_out/r6fb_w --top 45
TAIL=20 run_step r6fb_trace 500 bash tools/gpu/trace_now.sh
