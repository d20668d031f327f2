#!/bin/bash
# First MI355X pass: kernel tests, eager-baseline bench, kernel-trace profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch; print(torch.cuda.get_device_name(0), torch.cuda.mem_get_info())" > gpurun_out/env.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit 1; fi
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench.py --steps 4 --warmup 2 --batch_per_gpu 32 > gpurun_out/bench_b32.log 2>&1 || { echo "bench32 failed"; tail -30 gpurun_out/bench_b32.log; exit 1; }
tail -1 gpurun_out/bench_b32.log
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_b128.log 2>&1 || { echo "bench128 failed"; tail -30 gpurun_out/bench_b128.log; exit 1; }
tail -1 gpurun_out/bench_b128.log
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_eager -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --batch_per_gpu 32 > $GRAFT_REPO_ROOT/gpurun_out/prof_eager.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_eager.log; exit 1; }
echo done
