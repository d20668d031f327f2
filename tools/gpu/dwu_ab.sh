#!/bin/bash
# A/B of the unified depthwise backward: tools/bench_dw_fused.py on the default build and each variant .so in $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_dw_fused.py ${DWU_ARGS} > gpurun_out/dwab_default.log 2>&1 || { echo "default failed $?"; tail gpurun_out/dwab_default.log; exit 1; }
echo "== default"; grep -v amdgpu.ids gpurun_out/dwab_default.log
for v in $VARIANTS; do
  RT1_HIP_SO=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python -u tools/bench_dw_fused.py ${DWU_ARGS} > gpurun_out/dwab_$v.log 2>&1 || { echo "$v failed $?"; tail gpurun_out/dwab_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/dwab_$v.log
done
