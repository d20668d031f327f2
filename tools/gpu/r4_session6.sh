#!/bin/bash
# Staging over the in-image rectangle only (zero ring by LDS stores): depthwise numerics, per-block timing, bench.
source "$(dirname "$0")/step.sh"
run_step backbone6b 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backbone_gpu.py
run_step dwph_ring2 300 python -u tools/bench_dw_phases.py --tag ring2
TAIL=3 run_step bench6b 300 python -u bench.py --steps 20 --warmup 5
run_step parity6b 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_graph_gpu.py
