#!/bin/bash
# Depthwise kernel-parameter variants (build.py --variant <v> -D ..., built on the CPU side): per-block kernel times.
source "$(dirname "$0")/step.sh"
B=${DWV_BLOCKS:-0,1,3,4,6,7,9,10,13,14,19,24,25}
TAIL=20 run_step dwv_base 300 python -u tools/bench_dw_phases.py --blocks $B --tag base
for v in ${DWV_VARIANTS:-v_c4 v_r4 v_lds52}; do
    RT1_HIP_SO=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so TAIL=20 run_step dwv_$v 300 \
        python -u tools/bench_dw_phases.py --blocks $B --tag $v
done
