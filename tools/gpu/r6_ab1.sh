#!/bin/bash
# A/B of the phased depthwise staging (in-tree build) against build/base (DW_STAGE_PHASED=0): production-faithful
# depthwise replay (same calls, outputs compared), then bench.py alternated; then the DP traces and the new tests.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
BASE_SO=build/base/_rt1_hip.cpython-310-x86_64-linux-gnu.so
RT1_HIP_SO=$BASE_SO run_step dwr_base 400 python -u tools/bench_dw_replay.py --save /tmp/dwref.pt
run_step dwr_new 400 python -u tools/bench_dw_replay.py --ref /tmp/dwref.pt
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step ab1_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step ab1_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
bash tools/gpu/r6_dp_trace.sh
