#!/bin/bash
# Round-4 GPU session 4: the fused SE on the data-parallel path after the packed-fp32 op_sel fix -- the DP tests
# (graph == eager, eager == eager over 8 steps), the SE debug probe over 10 steps, the backbone numerics; the bench
# and a kernel-trace profile of the eager step (categories per step).
source "$(dirname "$0")/step.sh"
export TMPDIR=/tmp
run_step dist4 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_distributed_gpu.py
rm -rf gpurun_out/sedump4
TAIL=14 run_step sedbg4 400 env RT1_SE_DEBUG=1 RT1_SE_DUMP=gpurun_out/sedump4 \
    python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29591 \
    tools/dp_gpu_check.py --eager2 --steps 10
run_step backbone4 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backbone_gpu.py
TAIL=3 run_step bench4 300 python -u bench.py --steps 20 --warmup 5
rm -rf gpurun_out/trace4
run_step trace4 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trace4 -o run \
    -- python3 bench.py --steps 6 --warmup 2 --graph off --no_check
python3 tools/prof_categories.py --trace gpurun_out/trace4 > gpurun_out/trace4_categories.txt 2>&1
cat gpurun_out/trace4_categories.txt | head -20
