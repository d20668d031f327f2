#!/bin/bash
# graph-DP per-step cost, part 2: capture mode (relaxed vs global) of the one-graph step and of the DP segments;
# then the PMC byte-counter calibration on known-byte kernels.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
for rep in 1 2; do
  TAIL=1 run_step dh_graph_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=relaxed1 TAIL=1 run_step dh_relaxed1_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=nosync,notiming,noreduce TAIL=1 run_step dh_none_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  RT1_DP_DIAG=nosync,notiming,noreduce,globalseg TAIL=1 run_step dh_noneglobal_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
done
run_step pmc_cal 400 bash tools/gpu/pmc_calibrate.sh
