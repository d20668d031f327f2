#!/bin/bash
# Round-4 GPU session 3: graph == eager at the bench config after the deterministic FiLM bias gradient (with and
# without the fused SE path); the two-rank fused-SE probe with input dumps and their one-process replay; the gemm2
# pipeline-variant sweep; the bench.
source "$(dirname "$0")/step.sh"
TAIL=12 run_step det3_default 300 python -u tools/step_determinism.py --batch 128
TAIL=12 run_step det3_sef0 300 env RT1_SE_FUSED=0 python -u tools/step_determinism.py --batch 128
rm -rf gpurun_out/sedump
TAIL=20 run_step sedbg3 300 env RT1_SE_FUSED=force RT1_SE_DEBUG=1 RT1_SE_DUMP=gpurun_out/sedump \
    python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 \
    tools/dp_gpu_check.py --eager2
if ls gpurun_out/sedump/*.pt > /dev/null 2>&1; then
    TAIL=10 run_step se_replay 200 python -u tools/se_replay.py gpurun_out/sedump
fi
run_step gemm2_test3 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm2_gpu.py
TAIL=30 run_step gemm2_sweep 300 python -u tools/bench_gemm2.py --iters 20
TAIL=4 run_step bench3 300 python -u bench.py --steps 20 --warmup 5
