#!/bin/bash
# Same-box A/B of the depthwise staging walk: HEAD build (base_dw), rectangle walk for maps <= 400 px (default
# build), never (ring0), maps <= 2000 px (ring2k); tools/bench_dw_phases.py, two rounds.
source "$(dirname "$0")/step.sh"
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
for rep in 1 2; do
    RT1_HIP_SO=build/base_dw/$SO run_step dwab_base_$rep 300 python -u tools/bench_dw_phases.py --tag base
    run_step dwab_r400_$rep 300 python -u tools/bench_dw_phases.py --tag ring400
    RT1_HIP_SO=build/ring0/$SO run_step dwab_r0_$rep 300 python -u tools/bench_dw_phases.py --tag ring0
    RT1_HIP_SO=build/ring2k/$SO run_step dwab_r2k_$rep 300 python -u tools/bench_dw_phases.py --tag ring2k
done
