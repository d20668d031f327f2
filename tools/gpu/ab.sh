#!/bin/bash
# A/B: per-layer depthwise/BN microbench for the default build and each variant .so given in $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_kernels.py --frames 768 --res 300 ${KB_ARGS} > gpurun_out/kb_default.log 2>&1 || { echo "default failed $?"; tail gpurun_out/kb_default.log; exit 1; }
tail -1 gpurun_out/kb_default.log
for v in $VARIANTS; do
  RT1_HIP_SO=build/$v/_rt1_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python tools/bench_kernels.py --frames 768 --res 300 ${KB_ARGS} > gpurun_out/kb_$v.log 2>&1 || { echo "$v failed $?"; tail gpurun_out/kb_$v.log; exit 1; }
  echo "== $v"; tail -1 gpurun_out/kb_$v.log
done
