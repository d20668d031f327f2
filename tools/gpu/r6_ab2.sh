#!/bin/bash
# (1) depthwise replay A/B: in-tree (phased staging + centre prefetch) vs build/phased (no prefetch), same inputs;
# (2) graph-DP bucket size sweep on a world-1 RCCL communicator vs the one-graph step; (3) the new GPU tests.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step dwr_ab2 600 python -u tools/bench_dw_replay.py --ab build/phased/_rt1_hip.cpython-310-x86_64-linux-gnu.so
for rep in 1 2; do
  TAIL=1 run_step bk_graph_$rep 300 python -u bench.py --steps 20 --warmup 5
  for cap in 32 64 160; do
    TAIL=1 run_step bk_native${cap}_$rep 300 python -u bench.py --steps 20 --warmup 5 --comm native --bucket_cap_mb $cap
  done
done
run_step r6_newtests2 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
    tests/test_parity_gpu.py::test_full_model_step_hip_bf16_vs_torch_fp32 tests/test_xmode_gpu.py::test_block2_xmode_pair_at_bench_resolution \
    tests/test_distributed_gpu.py::test_bench_graph_mismatch_drops_captured_segments \
    tests/test_distributed_gpu.py::test_bench_capture_failure_on_one_rank_is_collective \
    tests/test_distributed_gpu.py::test_drop_graph_on_captured_single_rank_engine
