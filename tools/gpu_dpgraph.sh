#!/bin/bash
# 2 ranks on one GPU over gloo: eager DP check, then hipGraph-DP vs eager-DP, then a 2-rank bench with graphs
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dp_gpu_check.py --graph > gpurun_out/dp_graph_check.log 2>&1 || { echo "dp graph check failed $?"; tail -30 gpurun_out/dp_graph_check.log; exit 1; }
grep -E "graph-DP|losses" gpurun_out/dp_graph_check.log
RT1_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 6 --warmup 3 --batch_per_gpu 32 --graph on > gpurun_out/dp_graph_bench.log 2>&1 || { echo "bench failed $?"; tail -30 gpurun_out/dp_graph_bench.log; exit 1; }
tail -1 gpurun_out/dp_graph_bench.log
