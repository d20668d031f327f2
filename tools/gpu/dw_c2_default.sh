#!/bin/bash
# per-layer 2-channel k5 depthwise backward (default) vs the 4-channel form everywhere (RT1_DW_C2=0): numerics, then
# the step alternated.
source "$(dirname "$0")/step.sh"
run_step c2d_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backbone_gpu.py \
    tests/test_parity_gpu.py tests/test_graph_gpu.py
for rep in 1 2 3; do
    TAIL=1 run_step c2d_off_$rep 300 env RT1_DW_C2=0 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step c2d_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
