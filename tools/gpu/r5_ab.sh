#!/bin/bash
# 5-output depthwise strips (RT1_DW_R5 mask): depthwise GPU tests, then bench.py with RT1_DW_R5=0 / 1 / 3 alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backbone_gpu.py tests/test_xmode_gpu.py > gpurun_out/r5_tests.log 2>&1 || { echo "tests failed $?"; grep -E "FAILED|Error|assert" gpurun_out/r5_tests.log | head -30; tail -30 gpurun_out/r5_tests.log; exit 1; }
tail -1 gpurun_out/r5_tests.log
for rep in 1 2; do
  for v in 0 1 3; do
    RT1_DW_R5=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_${v}_$rep.log 2>&1 || { echo "bench $v failed $?"; tail -20 gpurun_out/r5_${v}_$rep.log; exit 1; }
    echo "RT1_DW_R5=$v rep$rep: $(tail -1 gpurun_out/r5_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
