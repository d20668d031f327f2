#!/bin/bash
# Round-4 GPU session 2: which gradients are not reproducible (eager vs eager, eager vs graph) on one GPU at the bench
# config, bisected over the SE path; then the two-rank SE probes and the new / changed GPU tests.
source "$(dirname "$0")/step.sh"
TAIL=40 run_step det_default 300 python -u tools/step_determinism.py --batch 128
TAIL=40 run_step det_nodrop 300 python -u tools/step_determinism.py --batch 128 --nodrop
TAIL=40 run_step det_sef0 300 env RT1_SE_FUSED=0 python -u tools/step_determinism.py --batch 128
TAIL=40 run_step det_small 300 python -u tools/step_determinism.py --batch 4 --hw 128
TAIL=30 run_step se_dp_debug 900 bash tools/gpu/se_dp_debug.sh
run_step pytest_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_imgproc_gpu.py tests/test_graph_gpu.py tests/test_distributed_gpu.py tests/test_parity_gpu.py
run_step resident_decode 200 python -u tools/gpu/resident_decode.py
