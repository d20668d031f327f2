#!/bin/bash
# new kernels (fused head, long-history attention backward) + whole GPU suite + bench (T=6 and T=15)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "long_kernel or fused_head" > gpurun_out/pytest_new.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_new.log
[ $rc -eq 0 ] || { echo "new-kernel tests failed rc=$rc"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "gpu suite failed rc=$rc"; grep -E "^E |Error" gpurun_out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_t6.log 2>&1 || { echo "bench t6 failed $?"; tail -20 gpurun_out/bench_t6.log; exit 1; }
tail -1 gpurun_out/bench_t6.log
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --seq_len 15 --batch_per_gpu 64 > gpurun_out/bench_t15.log 2>&1 || { echo "bench t15 failed $?"; tail -20 gpurun_out/bench_t15.log; exit 1; }
tail -1 gpurun_out/bench_t15.log
