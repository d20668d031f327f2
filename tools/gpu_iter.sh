#!/bin/bash
# one build->measure iteration: encoder kernel tests, per-layer microbench, flagship bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_backbone_gpu.py -q -s > gpurun_out/pytest_enc.log 2>&1; rc=$?
grep -E "passed|failed|encoder fwd|grad err" gpurun_out/pytest_enc.log | tail -4
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed $rc"; exit 1; fi
timeout -k 10 600 python tools/bench_kernels.py --frames 768 --res 300 > gpurun_out/kbench.log 2>&1 || { echo "kbench failed $?"; tail -5 gpurun_out/kbench.log; exit 1; }
tail -1 gpurun_out/kbench.log
if [ -n "$ITER_BENCH" ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -5 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
