#!/bin/bash
# What in an idle RCCL communicator costs the step ~1.1 ms: its high-priority comm stream, its watchdog thread.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
for rep in 1 2; do
  TAIL=1 run_step dl_graph_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=comminit TAIL=1 run_step dl_comminit_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=comminit RT1_COMM_STREAM=normal TAIL=1 run_step dl_comminit_normal_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_DP_DIAG=comminit RT1_COMM_TIMEOUT=0 TAIL=1 run_step dl_comminit_nowd_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_COMM_STREAM=normal TAIL=1 run_step dl_native_normal_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
done
