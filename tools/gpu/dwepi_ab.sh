#!/bin/bash
# depthwise forward epilogue (packed stats from the stored word): numerics, per-layer times base vs new, step A/B
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step dwepi_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backbone_gpu.py tests/test_xmode_gpu.py
RT1_HIP_SO=build/base/$SO run_step dwepi_phases_base 200 python -u tools/bench_dw_phases.py --tag base
run_step dwepi_phases_new 200 python -u tools/bench_dw_phases.py --tag new
RT1_HIP_SO=build/base/$SO run_step dwepi_phases_base2 200 python -u tools/bench_dw_phases.py --tag base2
BASE_SO=build/base/$SO TAG=dwepi bash tools/gpu/ab_so.sh
