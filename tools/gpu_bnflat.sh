#!/bin/bash
# A/B of the flat BN apply kernels (RT1_BN_FLAT=1, default) against the row layout (RT1_BN_FLAT=0):
# numerics (backbone GPU tests), per-layer microbench, end-to-end bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_backbone_gpu.py > gpurun_out/bnflat_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/bnflat_test.log; exit 1; }
tail -1 gpurun_out/bnflat_test.log
for f in 0 1; do
  RT1_BN_FLAT=$f timeout -k 10 300 python tools/bench_kernels.py --frames 768 --res 300 ${KB_ARGS} > gpurun_out/kb_flat$f.log 2>&1 || { echo "kb flat=$f failed $?"; tail gpurun_out/kb_flat$f.log; exit 1; }
  echo "== flat=$f"; tail -1 gpurun_out/kb_flat$f.log
done
for f in 0 1; do
  RT1_BN_FLAT=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_flat$f.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_flat$f.log; exit 1; }
  echo "== bench flat=$f"; tail -1 gpurun_out/bench_flat$f.log
done
