#!/bin/bash
# SE MLP kernels: numerics, per-block times base (RT1_HIP_SO) vs new, step A/B
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step se_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backbone_gpu.py
RT1_HIP_SO=build/base/$SO run_step se_bench_base 200 python -u tools/bench_se.py
run_step se_bench_new 200 python -u tools/bench_se.py
BASE_SO=build/base/$SO TAG=se bash tools/gpu/ab_so.sh
