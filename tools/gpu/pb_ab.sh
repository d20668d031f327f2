#!/bin/bash
# projbwd.hip variants (prefetch depth / occupancy) on tools/bench_proj_bwd.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_backbone_gpu.py -k proj_bwd -x -q --timeout 120 --timeout-method thread > gpurun_out/pb_test.log 2>&1 || { tail -20 gpurun_out/pb_test.log; exit 1; }
tail -n1 gpurun_out/pb_test.log
timeout -k 10 200 python -u tools/bench_proj_bwd.py > gpurun_out/pb_default.log 2>&1 || exit 1
echo "== default"; tail -n1 gpurun_out/pb_default.log
for v in $VARIANTS; do
  RT1_HIP_SO=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 200 python -u tools/bench_proj_bwd.py > gpurun_out/pb_$v.log 2>&1 || exit 1
  echo "== $v"; tail -n1 gpurun_out/pb_$v.log
done
