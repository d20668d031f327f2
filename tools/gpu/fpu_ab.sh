#!/bin/bash
# frame_pool loads in flight (RT1_FP_U 4 / 8): tests with 8, then bench.py alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
RT1_FP_U=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_backbone_gpu.py > gpurun_out/fpu_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/fpu_tests.log; exit 1; }
tail -1 gpurun_out/fpu_tests.log
for rep in 1 2; do
  for v in 4 8; do
    RT1_FP_U=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fpu_${v}_$rep.log 2>&1 || { echo "bench $v failed $?"; tail -20 gpurun_out/fpu_${v}_$rep.log; exit 1; }
    echo "RT1_FP_U=$v rep$rep: $(tail -1 gpurun_out/fpu_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
