#!/bin/bash
# A/B of the fused stride-1 depthwise backward (tools/bench_dw_fused.py) and the per-layer dw kernels
# (tools/bench_kernels.py) for the default build and each variant .so named in $VARIANTS (build/<name>/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dwf}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for v in default $VARIANTS; do
  so=""; [ "$v" != default ] && so=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so
  RT1_HIP_SO=$so timeout -k 10 300 python -u tools/bench_dw_fused.py > gpurun_out/${TAG}_$v.log 2>&1 || { echo "$v failed"; tail gpurun_out/${TAG}_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${TAG}_$v.log
  if [ -n "$KB" ]; then
    RT1_HIP_SO=$so timeout -k 10 300 python -u tools/bench_kernels.py --frames 768 --res 300 > gpurun_out/${TAG}_kb_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/${TAG}_kb_$v.log
  fi
done
