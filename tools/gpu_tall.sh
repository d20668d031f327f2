#!/bin/bash
# pwtall.hip: numerics tests, microbench vs hipBLASLt, then bench.py A/B (RT1_PW_TALL=0 vs default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pwgemm_gpu.py -k tall > gpurun_out/tall_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/tall_test.log; exit 1; }
tail -2 gpurun_out/tall_test.log
PYTHONPATH=. timeout -k 10 300 python -u tools/debug/tall_sweep.py > gpurun_out/tall_sweep.log 2>&1 || { echo "sweep failed $?"; tail -30 gpurun_out/tall_sweep.log; exit 1; }
cat gpurun_out/tall_sweep.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tall_bench_on.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/tall_bench_on.log; exit 1; }
tail -1 gpurun_out/tall_bench_on.log
RT1_PW_TALL=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tall_bench_off.log 2>&1 || { echo "bench off failed $?"; tail -30 gpurun_out/tall_bench_off.log; exit 1; }
tail -1 gpurun_out/tall_bench_off.log
