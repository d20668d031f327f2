#!/bin/bash
# The N > 1 bench path on ONE GPU: a single-rank torch process group over RCCL (RT1_PG_WORLD1=1) driving the
# segmented graph-DP step; test + 300x300 b128 timing against the one-graph step and the native communicator.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step pgw1_test 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu \
    tests/test_distributed_gpu.py -k "single_rank"
for rep in 1 2; do
  TAIL=1 run_step pgw1_graph_$rep 300 python -u bench.py --steps 20 --warmup 5
  RT1_PG_WORLD1=1 MASTER_PORT=2959$rep TAIL=1 run_step pgw1_torchpg_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step pgw1_native_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
done
