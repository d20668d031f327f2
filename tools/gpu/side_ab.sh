#!/bin/bash
# A/B: weight gradients on a side stream (RT1_WGRAD_SIDE) and the XCD-grouped wgrad launch (build/wg_ungrouped)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_side0.log 2>&1 || { echo "side0 failed"; tail gpurun_out/ab_side0.log; exit 1; }
tail -1 gpurun_out/ab_side0.log
RT1_WGRAD_SIDE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_side1.log 2>&1 || { echo "side1 failed"; tail gpurun_out/ab_side1.log; exit 1; }
tail -1 gpurun_out/ab_side1.log
timeout -k 10 300 python -u tools/bench_wgrad.py > gpurun_out/ab_wg_grouped.log 2>&1 || exit 1
RT1_HIP_SO=build/wg_ungrouped/_rt1_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python -u tools/bench_wgrad.py > gpurun_out/ab_wg_ungrouped.log 2>&1 || exit 1
tail -1 gpurun_out/ab_wg_grouped.log; tail -1 gpurun_out/ab_wg_ungrouped.log
