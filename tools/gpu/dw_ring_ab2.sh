#!/bin/bash
# Same-box A/B: HEAD build (base_dw) vs the templated rectangle walk (default build, maps <= 2000 px); then the
# backbone numerics and the bench.
source "$(dirname "$0")/step.sh"
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
for rep in 1 2; do
    RT1_HIP_SO=build/base_dw/$SO run_step dwab3_base_$rep 300 python -u tools/bench_dw_phases.py --tag base
    run_step dwab3_tpl_$rep 300 python -u tools/bench_dw_phases.py --tag ring-template
done
run_step backbone8 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backbone_gpu.py
for rep in 1 2; do
    RT1_HIP_SO=build/base_dw/$SO TAIL=1 run_step bench8_base_$rep 300 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step bench8_tpl_$rep 300 python -u bench.py --steps 20 --warmup 5
done
