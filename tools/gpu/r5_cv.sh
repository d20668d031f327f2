#!/bin/bash
# Block 2 x-mode channel chunk (RT1_DW_CV_AB: 18 = whole row [base], 6, 2 vectors): x-mode numerics per build, the
# two x-mode kernels alone (tools/bench_xmode.py), then the step (bench.py) base vs cv6 vs cv2
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
# the whole GPU suite on the working tree first (round-5 pruning: gemm2 / fp8 / dy-ready / dwmfma removed)
run_step cv_suite 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for v in base cv6 cv2; do
  so=build/$v/$SO; [ "$v" = base ] && so=pytorch_rt1_for_distributed_training_amd/$SO
  RT1_HIP_SO=$so run_step cv_tests_$v 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_xmode_gpu.py
done
for rep in 1 2; do
  for v in base cv6 cv2; do
    so=build/$v/$SO; [ "$v" = base ] && so=pytorch_rt1_for_distributed_training_amd/$SO
    RT1_HIP_SO=$so run_step cv_xb_${v}_$rep 200 python -u tools/bench_xmode.py
  done
done
for rep in 1 2; do
  for v in base cv6 cv2; do
    so=build/$v/$SO; [ "$v" = base ] && so=pytorch_rt1_for_distributed_training_amd/$SO
    RT1_HIP_SO=$so run_step cv_bench_${v}_$rep 300 python -u bench.py --steps 20 --warmup 5
  done
done
