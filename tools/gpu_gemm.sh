#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_pwgemm_gpu.py -q -x > gpurun_out/pytest_pw.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_pw.log
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/pytest_pw.log | head -10; exit 1; fi
timeout -k 10 500 python tools/bench_gemms.py --use-ext > gpurun_out/gemms_ext.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/gemms_ext.log; exit 1; }
head -24 gpurun_out/gemms_ext.log; tail -1 gpurun_out/gemms_ext.log
