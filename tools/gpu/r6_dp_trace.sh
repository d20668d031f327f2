#!/bin/bash
# Kernel traces of the replayed one-graph step and of the segmented graph-DP step on a world-1 RCCL communicator
# (--comm native), 5 steps each: busy vs idle per step (tools/graph_timeline.py).  Then the new GPU tests.
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
rm -rf gpurun_out/gt_graph gpurun_out/gt_native
TAIL=2 run_step gt_graph 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt_graph -o run -- python3 bench.py --steps 5 --warmup 3 --no_check
TAIL=2 run_step gt_native 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt_native -o run -- python3 bench.py --steps 5 --warmup 3 --no_check --comm native
python3 tools/graph_timeline.py gpurun_out/gt_graph --last 5 > gpurun_out/gt_graph_timeline.txt 2>&1; tail -8 gpurun_out/gt_graph_timeline.txt
python3 tools/graph_timeline.py gpurun_out/gt_native --last 5 > gpurun_out/gt_native_timeline.txt 2>&1; tail -8 gpurun_out/gt_native_timeline.txt
find gpurun_out/gt_graph gpurun_out/gt_native -name "*.db" -delete
gzip -f $(find gpurun_out/gt_graph gpurun_out/gt_native -name "*kernel_trace.csv") 2>/dev/null || true
run_step r6_newtests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
    tests/test_parity_gpu.py::test_full_model_step_hip_bf16_vs_torch_fp32 tests/test_xmode_gpu.py::test_block2_xmode_pair_at_bench_resolution \
    tests/test_distributed_gpu.py::test_bench_graph_mismatch_drops_captured_segments \
    tests/test_distributed_gpu.py::test_bench_capture_failure_on_one_rank_is_collective \
    tests/test_distributed_gpu.py::test_drop_graph_on_captured_single_rank_engine
