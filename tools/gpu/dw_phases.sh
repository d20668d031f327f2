#!/bin/bash
# Phase split of the depthwise kernels: tools/bench_dw_phases.py on the default build and on each timing-only build
# (build.py --variant t_<PHASE> -D RT1_DW_TIMING=<mask>, built on the CPU side beforehand).
source "$(dirname "$0")/step.sh"
run_step dwph_base 300 python -u tools/bench_dw_phases.py --tag base
for v in NOSTAGE NOTAPS NOCENTRE NOEPI; do
    RT1_HIP_SO=build/t_$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so run_step dwph_$v 300 \
        python -u tools/bench_dw_phases.py --tag $v
done
