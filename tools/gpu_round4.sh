#!/bin/bash
# MI355X pass: full GPU test suite, bench eager vs hipGraph, depthwise per-layer microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[gpu] $*"; }
fatal() { local rc=$1; shift; echo "[gpu] FATAL rc=$rc: $*"; exit 1; }
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

step "pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q -s -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -8
ok_or_testfail $rc || fatal $rc "pytest crashed"

step "bench hip b128 graph=off"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --graph off > gpurun_out/bench_eager.log 2>&1 || fatal $? "bench eager"
tail -1 gpurun_out/bench_eager.log
step "bench hip b128 graph=auto"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_graph.log 2>&1 || fatal $? "bench graph"
grep -i "capture" gpurun_out/bench_graph.log; tail -1 gpurun_out/bench_graph.log
if [ -n "$KBENCH" ]; then
  step "kbench"
  timeout -k 10 600 python tools/bench_kernels.py --frames 768 --res 300 ${KBLOCKS:+--blocks $KBLOCKS} > gpurun_out/kbench.log 2>&1 || fatal $? "kbench"
  cat gpurun_out/kbench.log
fi
step done
