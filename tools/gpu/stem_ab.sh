#!/bin/bash
# stem kernels: numerics, per-kernel time on the HEAD build (build/base) and the working tree, then the step A/B
source "$(dirname "$0")/step.sh"
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step stem_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_backbone_gpu.py -k stem
RT1_HIP_SO=build/base/$SO TAIL=3 run_step stem_k_base 200 python -u tools/bench_stem.py
TAIL=3 run_step stem_k_new 200 python -u tools/bench_stem.py
for rep in 1 2 3; do
    RT1_HIP_SO=build/base/$SO TAIL=1 run_step stem_base_$rep 300 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step stem_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
