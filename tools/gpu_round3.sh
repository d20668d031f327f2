#!/bin/bash
# MI355X pass: kernel numerics, fused-backend bench b128, kernel-trace profile b128.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[gpu] $*"; }
fatal() { local rc=$1; shift; echo "[gpu] FATAL rc=$rc: $*"; exit 1; }
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

step "pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q -s > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|per-block" gpurun_out/pytest_gpu.log | tail -5
ok_or_testfail $rc || fatal $rc "pytest crashed"

step "bench hip b128"
timeout -k 10 600 python bench.py --backend hip --steps 10 --warmup 3 --batch_per_gpu 128 > gpurun_out/bench_hip_b128.log 2>&1 || fatal $? "bench hip b128"
tail -1 gpurun_out/bench_hip_b128.log

step "rocprof hip b128"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_hip_b128 -o run -- python3 $R/bench.py --backend hip --steps 2 --warmup 1 --batch_per_gpu 128 > $R/gpurun_out/prof_hip_b128.log 2>&1 || fatal $? "rocprof hip"
cd $R && python tools/rocprof_summary.py gpurun_out/prof_hip_b128 --out gpurun_out/prof_hip_b128.md --title "fused HIP backend, batch 128 (768 frames 300x300), 3 steps" > /dev/null
step done
