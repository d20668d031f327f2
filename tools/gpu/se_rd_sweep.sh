#!/bin/bash
# SE MLP kernels per block (tools/bench_se.py) for several se_rowdot workgroup targets (RT1_SE_RD_WG).
source "$(dirname "$0")/step.sh"
for t in 512 256 128 1024; do
    RT1_SE_RD_WG=$t TAIL=3 run_step se_rd_$t 200 python -u tools/bench_se.py
done
