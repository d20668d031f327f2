#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_backbone_gpu.py -k stem > gpurun_out/stem_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/stem_test.log; exit 1; }
tail -1 gpurun_out/stem_test.log
timeout -k 10 300 python -u tools/debug/stem_bench.py > gpurun_out/stem_bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/stem_bench.log; exit 1; }
echo "== mfma"; grep max_blocks gpurun_out/stem_bench.log
RT1_HIP_SO=build/stemvalu/_rt1_hip.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python -u tools/debug/stem_bench.py > gpurun_out/stem_bench_valu.log 2>&1 || { echo "bench valu failed"; tail gpurun_out/stem_bench_valu.log; exit 1; }
echo "== valu"; grep max_blocks gpurun_out/stem_bench_valu.log
