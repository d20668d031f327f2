#!/bin/bash
# centre staging on the 10x10 k5 2-channel form only: kernel tests, replay A/B vs build/phased, bench A/B.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_SO=build/phased/_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step ab4_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_backbone_gpu.py tests/test_xmode_gpu.py tests/test_kernels_gpu.py
run_step dwr_ab4 600 python -u tools/bench_dw_replay.py --ab $BASE_SO
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step ab4_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step ab4_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
