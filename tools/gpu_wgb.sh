#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in ${WGB_LIST:-256 512 1024 2048}; do
  timeout -k 10 300 python tools/bench_kernels.py --frames 768 --res 300 --${WGB_ARG:-wgrad_blocks} $b ${KB_ARGS} > gpurun_out/kb_wgb$b.log 2>&1 || { echo "kb $b failed"; tail -5 gpurun_out/kb_wgb$b.log; exit 1; }
  echo "== $b"; tail -1 gpurun_out/kb_wgb$b.log
done
