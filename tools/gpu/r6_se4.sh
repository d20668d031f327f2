#!/bin/bash
# se_rowmat final form (16-frame tiles below 300 workgroups, V loaded ahead of the partial sums, conflict-free forward
# V layout) + adaptive se_wsum_part slices: numerics, isolated A/B vs the committed HEAD build, bench A/B.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_SO=build/head2/_rt1_hip.cpython-310-x86_64-linux-gnu.so
run_step se_tests4 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_backbone_gpu.py \
    -k "se_"
run_step se_ab4 300 python -u tools/bench_se.py --ab $BASE_SO
for rep in 1 2 3; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step se4_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step se4_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
