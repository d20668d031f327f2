#!/bin/bash
# unified depthwise backward: numerics (fused-kernel tests, both variants) then per-layer timing vs the two-pass kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dwu}
timeout -k 10 300 python -u -m pytest tests/test_backbone_gpu.py -k "dw_bwd_fused" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_test.log 2>&1 || { echo "test failed $?"; tail -40 gpurun_out/${TAG}_test.log; exit 1; }
tail -2 gpurun_out/${TAG}_test.log
timeout -k 10 300 python -u tools/bench_dw_fused.py ${DWU_ARGS} > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed $?"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
cat gpurun_out/${TAG}_bench.log
