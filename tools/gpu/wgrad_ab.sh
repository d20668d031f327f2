#!/bin/bash
# A/B of the 1x1-conv weight-gradient kernel: tools/bench_wgrad.py on the default build and each variant in $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_wgrad.py ${WG_ARGS} > gpurun_out/wgab_default.log 2>&1 || { echo "default failed $?"; tail gpurun_out/wgab_default.log; exit 1; }
echo "== default"; grep -v amdgpu.ids gpurun_out/wgab_default.log
for v in $VARIANTS; do
  RT1_HIP_SO=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python -u tools/bench_wgrad.py ${WG_ARGS} > gpurun_out/wgab_$v.log 2>&1 || { echo "$v failed $?"; tail gpurun_out/wgab_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/wgab_$v.log
done
