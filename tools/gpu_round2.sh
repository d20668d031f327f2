#!/bin/bash
# MI355X pass: kernel numerics, fused-backend bench, kernel-trace profiles (fused + eager).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[gpu] $*"; }
fatal() { local rc=$1; shift; echo "[gpu] FATAL rc=$rc: $*"; exit 1; }
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

step "pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:randomly > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
ok_or_testfail $rc || fatal $rc "pytest crashed"

step "bench hip b32"
timeout -k 10 600 python bench.py --backend hip --steps 5 --warmup 2 --batch_per_gpu 32 > gpurun_out/bench_hip_b32.log 2>&1 || fatal $? "bench hip b32"
tail -1 gpurun_out/bench_hip_b32.log

step "bench hip b128"
timeout -k 10 600 python bench.py --backend hip --steps 5 --warmup 2 --batch_per_gpu 128 > gpurun_out/bench_hip_b128.log 2>&1 || fatal $? "bench hip b128"
tail -1 gpurun_out/bench_hip_b128.log

step "rocprof hip b32"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_hip_b32 -o run -- python3 $R/bench.py --backend hip --steps 2 --warmup 1 --batch_per_gpu 32 > $R/gpurun_out/prof_hip_b32.log 2>&1 || fatal $? "rocprof hip"
cd $R && python tools/rocprof_summary.py gpurun_out/prof_hip_b32 --out gpurun_out/prof_hip_b32.md --title "fused HIP backend, batch 32 (192 frames 300x300), 3 steps" > /dev/null

step "rocprof eager b8"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_torch_b8 -o run -- python3 $R/bench.py --backend torch --steps 2 --warmup 1 --batch_per_gpu 8 > $R/gpurun_out/prof_torch_b8.log 2>&1 || fatal $? "rocprof eager"
cd $R && python tools/rocprof_summary.py gpurun_out/prof_torch_b8 --out gpurun_out/prof_torch_b8.md --title "eager PyTorch/MIOpen baseline, batch 8 (48 frames 300x300), 3 steps" > /dev/null
step done
