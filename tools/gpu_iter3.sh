#!/bin/bash
# encoder numerics + per-layer kernel bench + end-to-end bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_backbone_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_enc.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_enc.log
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/pytest_enc.log | head -20; exit 1; }
timeout -k 10 300 python tools/bench_kernels.py --frames 768 --res 300 > gpurun_out/kbench.log 2>&1 || { echo "kbench failed $?"; tail gpurun_out/kbench.log; exit 1; }
tail -1 gpurun_out/kbench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed $?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
