#!/bin/bash
# graph-DP per-step cost, part 3: kernel arguments in device memory for the segment graphs; PMC calibration; then the
# centre-staging depthwise A/B (in-tree = LDS-DMA centres, build/phased = none) and the backbone kernel tests.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
for rep in 1 2; do
  TAIL=1 run_step di_graph_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=noreduce TAIL=1 run_step di_none_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  HIP_FORCE_DEV_KERNARG=1 RT1_DP_DIAG=noreduce TAIL=1 run_step di_nonedk_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  HIP_FORCE_DEV_KERNARG=1 TAIL=1 run_step di_graphdk_$rep 300 python -u bench.py --steps 20 --warmup 5
done
run_step pmc_cal 400 bash tools/gpu/pmc_calibrate.sh
run_step dw_cs_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_backbone_gpu.py tests/test_xmode_gpu.py
run_step dwr_cs 600 python -u tools/bench_dw_replay.py --match bwd --ab build/phased/_rt1_hip.cpython-310-x86_64-linux-gnu.so
