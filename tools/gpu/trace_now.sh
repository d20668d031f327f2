#!/bin/bash
# Kernel + memory-copy trace of the eager bench step (current build) -> per-step categories (tools/prof_categories.py)
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
rm -rf gpurun_out/trN
TAIL=1 run_step trN 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trN -o run \
    -- python3 bench.py --steps 6 --warmup 2 --graph off --no_check
python3 tools/prof_categories.py --trace gpurun_out/trN > gpurun_out/trN_categories.txt 2>&1
cat gpurun_out/trN_categories.txt
find gpurun_out/trN -name "*.db" -delete
gzip -f gpurun_out/trN/*/*kernel_trace.csv 2>/dev/null || gzip -f $(find gpurun_out/trN -name "*kernel_trace.csv") 2>/dev/null || true
