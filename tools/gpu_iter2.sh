#!/bin/bash
# kernel unit tests (pw GEMM / fused backward), comm probe, encoder tests, microbench, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/test_pwgemm_gpu.py -q -x > gpurun_out/pytest_pw.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_pw.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|error" gpurun_out/pytest_pw.log | head -20; exit 1; fi
timeout -k 10 120 python tools/debug/comm_probe.py > gpurun_out/comm_probe.log 2>&1 || { echo "comm probe rc=$?"; grep -v "^Extension" gpurun_out/comm_probe.log | tail -5; exit 1; }
tail -1 gpurun_out/comm_probe.log
ITER_BENCH=1 bash tools/gpu_iter.sh
