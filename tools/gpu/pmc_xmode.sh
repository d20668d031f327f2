#!/bin/bash
# block 2's x-mode depthwise kernels: timing (with the stored-y1 forward for comparison), then SQ counters
source "$(dirname "$0")/step.sh"
TAIL=6 run_step xm_time 200 python -u tools/bench_xmode.py --stored
PMC_TOOL="tools/bench_xmode.py --stored" TAG=pmcx timeout -k 10 500 bash tools/gpu/pmc_dw.sh
cat gpurun_out/pmcx_summary.txt | head -40
