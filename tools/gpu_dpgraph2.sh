#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/graph_dp_nccl1.py > gpurun_out/graph_dp_nccl1.log 2>&1 || { echo "nccl1 check failed $?"; tail -30 gpurun_out/graph_dp_nccl1.log; exit 1; }
tail -3 gpurun_out/graph_dp_nccl1.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dp_gpu_check.py --graph > gpurun_out/dp_graph_check.log 2>&1 || { echo "dp graph check failed $?"; tail -30 gpurun_out/dp_graph_check.log; exit 1; }
grep -E "graph-DP|losses" gpurun_out/dp_graph_check.log
