#!/bin/bash
# BN1 of the wide expand convs from the Gram moments (no bn_stats pass): tests, model numerics, same-box bench A/B
# against the previous commit's build (build/base, RT1_GRAM_BN has no effect there).
source "$(dirname "$0")/step.sh"
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step xm10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xmode_gpu.py
run_step model10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backbone_gpu.py tests/test_parity_gpu.py tests/test_graph_gpu.py
for rep in 1 2; do
    RT1_HIP_SO=build/base/$SO RT1_GRAM_BN=0 TAIL=1 run_step bench10_base_$rep 300 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step bench10_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
