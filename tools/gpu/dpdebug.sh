#!/bin/bash
# graph-capture kernel tests, the graph-DP debug variants and the 1-GPU replay-determinism probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dbg}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_capture_gpu.py tests/test_graph_gpu.py > gpurun_out/${TAG}_gcap.log 2>&1 || { echo "graph tests failed"; grep -E "FAIL|Error|assert" gpurun_out/${TAG}_gcap.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_gcap.log
rm -f /tmp/rt1_gconc_*
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 tools/scratch/graph_concurrency_probe.py > gpurun_out/${TAG}_gconc.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/${TAG}_gconc.log; exit 1; }
grep -E "^\[|^rank" gpurun_out/${TAG}_gconc.log
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 tools/scratch/dp_graph_debug.py > gpurun_out/${TAG}_dpdbg.log 2>&1 || { echo "dp debug failed"; tail -20 gpurun_out/${TAG}_dpdbg.log; exit 1; }
grep -E "^\[cap|^     |graph replay" gpurun_out/${TAG}_dpdbg.log | head -40
