#!/bin/bash
# k5 unified depthwise backward: 4 vs 2 channels per thread (RT1_DW_C2) with the round-4 ring staging --
# per-block kernel times, then the step.
source "$(dirname "$0")/step.sh"
TAIL=30 run_step c2_dw_off 300 env RT1_DW_C2=0 python -u tools/bench_dw_phases.py --blocks 6,7,13,14,19,20 --tag c2off
TAIL=30 run_step c2_dw_on 300 env RT1_DW_C2=1 python -u tools/bench_dw_phases.py --blocks 6,7,13,14,19,20 --tag c2on
for rep in 1 2; do
    TAIL=1 run_step c2_off_$rep 300 env RT1_DW_C2=0 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step c2_on_$rep 300 env RT1_DW_C2=1 python -u bench.py --steps 20 --warmup 5
done
