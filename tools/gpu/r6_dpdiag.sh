#!/bin/bash
# Per-step cost of the graph-DP path on a world-1 RCCL communicator: which part costs the ~2.4 % against the one-graph
# step (RT1_DP_DIAG knobs), alternated with the one-graph baseline; then the bench A/B of the centre prefetch.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
for rep in 1 2; do
  TAIL=1 run_step dg_graph_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step dg_native_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  RT1_DP_DIAG=nosync TAIL=1 run_step dg_nosync_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  RT1_DP_DIAG=notiming TAIL=1 run_step dg_notiming_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
  RT1_DP_DIAG=nosync,notiming,noreduce TAIL=1 run_step dg_none_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native
done
BASE_SO=build/phased/_rt1_hip.cpython-310-x86_64-linux-gnu.so
for rep in 1 2; do
  RT1_HIP_SO=$BASE_SO TAIL=1 run_step ab3_base_$rep 300 python -u bench.py --steps 20 --warmup 5
  TAIL=1 run_step ab3_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
run_step r6_newtests3 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
    tests/test_distributed_gpu.py::test_drop_graph_on_captured_single_rank_engine tests/test_backbone_gpu.py
